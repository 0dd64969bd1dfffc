#!/usr/bin/env python3
"""GEMM microbenchmark: our gfx950 MFMA kernel vs torch (hipBLASLt) on the same random bf16
data, interleaved rounds in one process (cdna_hip_programming.md §5.4 rules 24/25).

python tools/bench_gemm.py [--shapes 4096x4096x4096,8192x8192x8192] [--rounds 5] [--iters 20]
Writes a JSON summary to stdout (and --out if given).
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from aliyun_gpushare_device_plugin_amd.ops import gemm_nt  # noqa: E402
from aliyun_gpushare_device_plugin_amd.ops.gemm import GEMM_AUTO, GEMM_V1, set_gemm_variant  # noqa: E402


def time_fn(fn, iters):
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    start.record()
    for _ in range(iters):
        fn()
    end.record()
    end.synchronize()
    return start.elapsed_time(end) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="4096x4096x4096,8192x8192x8192,4096x14336x4096,4096x4096x14336,"
                                        "8192x6144x4096,16384x4096x4096")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", default=None)
    ap.add_argument("--variants", default="1,2", help="extra kernel variants to time besides auto")
    a = ap.parse_args()
    res = []
    variants = [int(v) for v in a.variants.split(",") if v]
    for s in a.shapes.split(","):
        M, N, K = map(int, s.split("x"))
        x = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        w = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        def run_variant(v):
            def f():
                set_gemm_variant(v)
                gemm_nt(x, w, out=out)
            return f

        fns = {"ours": run_variant(GEMM_AUTO), **{f"v{v}": run_variant(v) for v in variants},
               "torch": lambda: torch.matmul(x, w.t(), out=out)}
        for f in fns.values():
            for _ in range(3):
                f()
        torch.cuda.synchronize()
        times = {k: [] for k in fns}
        names = list(fns)
        for r in range(a.rounds):   # order rotated every round (a fixed order biases by slot)
            for k in names[r % len(names):] + names[:r % len(names)]:
                times[k].append(time_fn(fns[k], a.iters))
        set_gemm_variant(GEMM_AUTO)
        flop = 2.0 * M * N * K
        row = {"shape": [M, N, K]}
        for k, t in times.items():
            med = statistics.median(t)
            row[f"{k}_ms"] = round(med, 4)
            row[f"{k}_tflops"] = round(flop / med / 1e9, 1)
        row["speedup"] = round(row["torch_ms"] / row["ours_ms"], 3)
        res.append(row)
        print(json.dumps(row), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
