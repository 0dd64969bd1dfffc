"""Round-6 probe on MI355X: what a pod under a broker grant gets today from the paths the arena
does not interpose yet, and how long an uncooperative tenant's granules take to come back.

* ``ipc``: torch.multiprocessing sharing of a CUDA tensor (hipIpcGetMemHandle on arena memory),
  and the raw hipIpcGetMemHandle / hipMemRetainAllocationHandle return codes.
* ``rccl``: a single-rank ``init_process_group("nccl")`` + ``all_reduce`` in the shimmed pod.
* ``sigterm``: a tenant holding 8 GiB of its arena is SIGTERMed (default handler, no release
  call); how long until the broker has its granules back, against a cooperative release.

Prints one JSON line per step. Usage: python tools/diag/r6_arena_probe.py [out.jsonl]
"""
from __future__ import annotations

import json
import os
import signal
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
GIB = 1 << 30

TENANT = r"""
import ctypes, json, os, sys, time, traceback
import torch
mode = sys.argv[1]
out = {"mode": mode}
lib = ctypes.CDLL(None)
x = torch.full((2 << 30,), 3, dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
a = [ctypes.c_uint64() for _ in range(2)]
out["arena"] = lib.gpushare_shim_arena_stats(*[ctypes.byref(v) for v in a])
out["arena_size"] = a[0].value
hip = ctypes.CDLL("libamdhip64.so")
if mode == "ipc":
    h = ctypes.create_string_buffer(64)
    out["ipc_get"] = hip.hipIpcGetMemHandle(h, ctypes.c_void_p(x.data_ptr()))
    hh = ctypes.c_void_p()
    out["retain"] = hip.hipMemRetainAllocationHandle(ctypes.byref(hh), ctypes.c_void_p(x.data_ptr()))
    out["retain_handle"] = hh.value or 0
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q, r = ctx.Queue(), ctx.Queue()
    import probe_child
    p = ctx.Process(target=probe_child.child, args=(q, r))
    p.start()
    try:
        q.put(x[:1 << 20])
        out["mp_share"] = r.get(timeout=90)
    except Exception as e:
        out["mp_share"] = ["parent_err", f"{type(e).__name__}: {e}"[:300]]
    p.join(30)
    out["child_exit"] = p.exitcode
elif mode == "rccl":
    import torch.distributed as dist
    try:
        dist.init_process_group("nccl", init_method="tcp://127.0.0.1:29517", rank=0, world_size=1)
        y = torch.ones(1 << 20, device="cuda")
        dist.all_reduce(y)
        torch.cuda.synchronize()
        out["all_reduce"] = float(y[0].item())
        dist.destroy_process_group()
    except Exception as e:
        out["rccl_err"] = f"{type(e).__name__}: {e}"[:400]
elif mode in ("hold", "coop"):
    y = torch.full((6 << 30,), 1, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    if mode == "coop":
        del x, y
        torch.cuda.empty_cache()
        lib.gpushare_shim_arena_release.restype = ctypes.c_int
        out["released"] = lib.gpushare_shim_arena_release()
    print(json.dumps(out), flush=True)
    if mode == "coop":
        os._exit(0)
    time.sleep(600)
print(json.dumps(out), flush=True)
"""

CHILD = r"""
def child(q, r):
    try:
        t = q.get(timeout=60)
        r.put(("ok", int(t[:1024].sum().item())))
    except Exception as e:
        r.put(("err", f"{type(e).__name__}: {e}"[:300]))
"""


def main():
    from aliyun_gpushare_device_plugin_amd.quota.hbmbroker import HBMBroker
    from aliyun_gpushare_device_plugin_amd.utils.native import ensure_built, preload

    out_path = sys.argv[1] if len(sys.argv) > 1 else None
    res = []

    def emit(d):
        res.append(d)
        print(json.dumps(d), flush=True)
        if out_path:
            with open(out_path, "a") as f:
                f.write(json.dumps(d) + "\n")

    def rd(p):
        try:
            return open(p).read().strip()
        except OSError as e:
            return str(e)
    emit({"ptrace_scope": rd("/proc/sys/kernel/yama/ptrace_scope"), "kernel": os.uname().release})
    tmp = f"/tmp/r6probe-{os.getpid()}"
    os.makedirs(tmp, exist_ok=True)
    with open(os.path.join(tmp, "probe_child.py"), "w") as f:
        f.write(CHILD)
    b = HBMBroker(os.path.join(tmp, "hbm.sock"), device=0, gib=24, wait_s=20)
    b.start()
    t = time.time() + 60
    while b.stat()["granules"] < b.stat()["granules_max"] and time.time() < t:
        time.sleep(0.2)
    env0 = dict(os.environ, LD_PRELOAD=preload(ensure_built("hipshim")), GPUSHARE_QUOTA_BYTES=str(16 * GIB),
                GPUSHARE_HBM_BROKER=b.socket_path, PYTHONPATH=tmp + os.pathsep + ROOT)
    try:
        for i, mode in enumerate(("ipc", "rccl")):
            tok = f"{mode}{i}" * 4
            b.grant(tok, 12 * GIB)
            r = subprocess.run([sys.executable, "-c", TENANT, mode], env=dict(env0, GPUSHARE_HBM_TOKEN=tok),
                               capture_output=True, text=True, timeout=240)
            lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
            emit({"step": mode, "rc": r.returncode, "out": lines, "stderr": r.stderr[-1500:]})
        for mode in ("coop", "hold", "coop", "hold"):
            tok = f"t{len(res)}" * 8
            b.grant(tok, 12 * GIB)
            st0 = b.stat()
            p = subprocess.Popen([sys.executable, "-c", TENANT, mode], env=dict(env0, GPUSHARE_HBM_TOKEN=tok),
                                 stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
            line = p.stdout.readline()
            t0 = time.time()
            if mode == "hold":
                p.send_signal(signal.SIGTERM)
            rc = p.wait(60)
            t_exit = time.time() - t0
            st = b.stat()
            while (st["free"] < st["granules"] or st["quarantined"] or st["scrubbing"]) and time.time() - t0 < 30:
                time.sleep(0.002)
                st = b.stat()
            emit({"step": "stop_" + mode, "rc": rc, "tenant": line.strip(), "exit_ms": t_exit * 1e3,
                  "back_ms": (time.time() - t0) * 1e3, "quarantine_ms_last": st["quarantine_ms_last"],
                  "releases": st["releases"], "free": st["free"], "granules": st["granules"],
                  "policy": st["release_policy"], "takes_before": st0["takes"]})
    finally:
        b.stop()


if __name__ == "__main__":
    main()
