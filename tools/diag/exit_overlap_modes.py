"""Which part of a retiring ROCm process's teardown slows the next process's runtime start-up.

A tenant (torch, 6 GiB, GEMMs) ends in one of several ways; a starter that already imported
torch then times ``torch.cuda.init()`` and its first allocation. ``--when reaped``: the starter
goes once the tenant was reaped (the kubelet's order); ``--when ack``: as soon as the tenant says
it is leaving (the bench's cooperative stop). One JSON line per trial.

    python tools/diag/exit_overlap_modes.py --trials 3
"""
import argparse
import json
import subprocess
import sys
import time

TENANT = r"""
import ctypes, json, os, sys, torch
x = torch.full((6 << 30,), 7, dtype=torch.uint8, device="cuda")
y = torch.randn(4096, 4096, device="cuda")
for _ in range(20):
    y = y @ y.T / 4096.0
torch.cuda.synchronize()
print(json.dumps({"ready": True}), flush=True)
mode = sys.stdin.readline().strip()
if mode in ("free", "reset"):
    del x, y
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
if mode == "reset":
    lib = next(ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln)
    ctypes.CDLL(lib).hipDeviceReset()
print(json.dumps({"leaving": True}), flush=True)
os._exit(0)
"""

STARTER = r"""
import json, sys, time
import torch
sys.stdout.write("go\n"); sys.stdout.flush()
sys.stdin.readline()
t2 = time.perf_counter()
torch.cuda.init()
t3 = time.perf_counter()
z = torch.zeros(1 << 20, device="cuda")
torch.cuda.synchronize()
t4 = time.perf_counter()
print(json.dumps({"cuda_init_ms": round((t3 - t2) * 1e3, 1), "first_alloc_ms": round((t4 - t3) * 1e3, 1)}), flush=True)
"""


def trial(mode: str, when: str, pause_s: float) -> dict:
    st = subprocess.Popen([sys.executable, "-c", STARTER], stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    assert st.stdout.readline().strip() == "go"
    t = subprocess.Popen([sys.executable, "-c", TENANT], stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    assert json.loads(t.stdout.readline())["ready"]
    t0 = time.perf_counter()
    t.stdin.write(mode + "\n")
    t.stdin.flush()
    assert json.loads(t.stdout.readline())["leaving"]
    t_ack = time.perf_counter()
    if when == "reaped":
        t.wait(60)
    time.sleep(pause_s)
    t_go = time.perf_counter()
    st.stdin.write("\n")
    st.stdin.flush()
    r = json.loads(st.stdout.readline())
    st.wait(60)
    t.wait(60)
    return dict(r, mode=mode, when=when, pause_s=pause_s, leave_ms=round((t_ack - t0) * 1e3, 1),
                go_after_ack_ms=round((t_go - t_ack) * 1e3, 1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=3)
    ap.add_argument("--modes", default="exit,free,reset")
    ap.add_argument("--whens", default="ack,reaped")
    a = ap.parse_args()
    for i in range(a.trials):
        for mode in a.modes.split(","):
            for when in a.whens.split(","):
                print(json.dumps(dict(trial(mode, when, 0.0), trial=i)), flush=True)
        print(json.dumps(dict(trial("exit", "reaped", 1.0), trial=i)), flush=True)


if __name__ == "__main__":
    main()
