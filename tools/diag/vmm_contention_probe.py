"""Two processes on one GPU: does memory from the HBM broker's arena change how they share it?

``reader``: streams a large buffer (``x.sum()``, HBM-bound like a decode step), timing each pass;
``gemm``: back-to-back bf16 GEMMs (compute-bound like a prefill). Each process takes its memory
from a broker arena (quota shim + grant) or from the driver, per ``--arena`` (``rg``: both, ``r``:
the reader only, ``g``: the GEMM only, ``none``). Prints one JSON line per configuration: each
process's rate alone and together.

    python tools/diag/vmm_contention_probe.py --configs rg,r,g,none --seconds 5
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

WORK = r"""
import json, os, sys, time, torch
kind, seconds, start = sys.argv[1], float(sys.argv[2]), sys.argv[3]
if kind == "reader":
    x = torch.ones(int(os.environ.get("READ_GIB", "16")) << 29, dtype=torch.bfloat16, device="cuda")
    op = lambda: x.sum()
    unit = x.numel() * 2
else:
    n = 8192
    a = torch.randn(n, n, dtype=torch.bfloat16, device="cuda")
    b = torch.randn(n, n, dtype=torch.bfloat16, device="cuda")
    op = lambda: a @ b
    unit = 2 * n ** 3
for _ in range(3):
    op()
torch.cuda.synchronize()
print(json.dumps({"ready": True}), flush=True)
while not os.path.exists(start):
    time.sleep(0.005)
t0 = time.perf_counter()
n = 0
lat = []
while time.perf_counter() - t0 < seconds:
    t = time.perf_counter()
    op()
    torch.cuda.synchronize()
    lat.append(time.perf_counter() - t)
    n += 1
dt = time.perf_counter() - t0
lat.sort()
print(json.dumps({"kind": kind, "iters": n, "rate": n * unit / dt / 1e12, "p50_ms": lat[len(lat) // 2] * 1e3}),
      flush=True)
"""


def run(procs, seconds):
    start = os.path.join(tempfile.mkdtemp(), "go")
    ps = []
    for kind, env in procs:
        ps.append(subprocess.Popen([sys.executable, "-c", WORK, kind, str(seconds), start], env=env,
                                   stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    for p in ps:
        line = p.stdout.readline()
        if not line:
            raise RuntimeError(p.stderr.read()[-2000:])
    open(start, "w").close()
    out = []
    for p in ps:
        out.append(json.loads(p.stdout.readline()))
        p.wait(60)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="rg,r,g,none")
    ap.add_argument("--seconds", type=float, default=5.0)
    a = ap.parse_args()
    from aliyun_gpushare_device_plugin_amd.quota.hbmbroker import HBMBroker
    from aliyun_gpushare_device_plugin_amd.utils.native import ensure_built, preload

    d = tempfile.mkdtemp(prefix="gs-hbm-", dir="/tmp")
    broker = HBMBroker.for_gpu(d, 0, device=0, reserve_gib=12)
    broker.start()
    shim = preload(ensure_built("hipshim"))
    try:
        for cfg in a.configs.split(","):
            envs = {}
            for i, kind in enumerate(("reader", "gemm")):
                env = dict(os.environ, LD_PRELOAD=shim, GPUSHARE_QUOTA_BYTES=str(40 << 30))
                if kind[0] in cfg:
                    tok = f"{kind}-{cfg}".ljust(32, "x")[:32]
                    broker.grant(tok, 38 << 30, 40 << 30)
                    env.update(GPUSHARE_HBM_BROKER=broker.socket_path, GPUSHARE_HBM_TOKEN=tok)
                envs[kind] = env
            alone_r = run([("reader", envs["reader"])], a.seconds)[0]
            alone_g = run([("gemm", envs["gemm"])], a.seconds)[0]
            both = run([("reader", envs["reader"]), ("gemm", envs["gemm"])], a.seconds)
            print(json.dumps({"arena": cfg, "reader_alone_TBps": round(alone_r["rate"], 3),
                              "gemm_alone_TFLOPs": round(alone_g["rate"] * 1e3, 1),
                              "reader_both_TBps": round(both[0]["rate"], 3),
                              "gemm_both_TFLOPs": round(both[1]["rate"] * 1e3, 1),
                              "reader_p50_ms": [alone_r["p50_ms"], both[0]["p50_ms"]]}), flush=True)
    finally:
        broker.stop()


if __name__ == "__main__":
    main()
