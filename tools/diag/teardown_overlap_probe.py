"""How much a ROCm process's teardown slows the next process's runtime start-up.

One tenant (6 GiB + some GEMMs, as in the bench's pods) is stopped with SIGTERM; the next
process's ``torch.cuda.init()`` + first allocation is timed right after the first one was reaped
(``overlap``) and after a 2 s pause (``idle``). Prints one JSON line per trial. The bench's
unmodified-tenant comparator (``bench.py --tenant-stop sigterm``) pays ``overlap`` on every step.

    python tools/diag/teardown_overlap_probe.py --trials 4
"""
import argparse
import json
import os
import signal
import subprocess
import sys
import time

TENANT = r"""
import json, sys, time, torch
x = torch.full((int(sys.argv[1]) << 30,), 7, dtype=torch.uint8, device="cuda")
y = torch.randn(4096, 4096, device="cuda")
for _ in range(20):
    y = y @ y.T / 4096.0
torch.cuda.synchronize()
print(json.dumps({"ready": True}), flush=True)
time.sleep(600)
"""

STARTER = r"""
import json, sys, time
t0 = time.perf_counter()
import torch
t1 = time.perf_counter()
sys.stdout.write("go\n"); sys.stdout.flush()
sys.stdin.readline()
t2 = time.perf_counter()
torch.cuda.init()
t3 = time.perf_counter()
z = torch.zeros(1 << 20, device="cuda")
torch.cuda.synchronize()
t4 = time.perf_counter()
print(json.dumps({"cuda_init_ms": (t3 - t2) * 1e3, "first_alloc_ms": (t4 - t3) * 1e3}), flush=True)
"""


def trial(pause_s: float, env: dict, gib: int = 6) -> dict:
    st = subprocess.Popen([sys.executable, "-c", STARTER], stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    assert st.stdout.readline().strip() == "go"          # torch imported, no GPU touched yet
    t = subprocess.Popen([sys.executable, "-c", TENANT, str(gib)], stdout=subprocess.PIPE, text=True, env=env)
    assert t.stdout.readline()
    t0 = time.perf_counter()
    t.send_signal(signal.SIGTERM)
    t.wait(60)
    exit_ms = (time.perf_counter() - t0) * 1e3
    time.sleep(pause_s)
    st.stdin.write("\n")
    st.stdin.flush()
    r = json.loads(st.stdout.readline())
    st.wait(60)
    return dict(r, exit_ms=round(exit_ms, 1), pause_s=pause_s, gib=gib)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=3)
    ap.add_argument("--gib", default="6", help="tenant's driver allocation, GiB (comma list)")
    ap.add_argument("--pauses", default="0,2", help="seconds between the reap and the next start (comma list)")
    a = ap.parse_args()
    env = dict(os.environ)
    for i in range(a.trials):
        for gib in (int(x) for x in a.gib.split(",")):
            for pause in (float(x) for x in a.pauses.split(",")):
                r = trial(pause, env, gib)
                print(json.dumps(dict(r, trial=i)), flush=True)


if __name__ == "__main__":
    main()
