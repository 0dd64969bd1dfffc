#!/usr/bin/env python3
"""Phase-B schedule sweep of the 4-wave GEMM (placement of the LDS DMA and the fragment reads,
``set_gemm_w4_sched``) against torch.matmul (hipBLASLt), interleaved rounds in one process (order
rotated every round), event timing of 20 back-to-back launches. Each schedule's output is checked against torch's first.

python tools/gemm_sched_sweep.py [--shapes 4096x4096x4096,...] [--scheds 0,1,2,3,4,5]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from aliyun_gpushare_device_plugin_amd.ops import gemm_nt  # noqa: E402
from aliyun_gpushare_device_plugin_amd.ops.gemm import set_gemm_w4_sched  # noqa: E402


def time_fn(fn, iters=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="4096x4096x4096,4096x4096x1024,8192x8192x8192,4096x4096x14336")
    ap.add_argument("--scheds", default="0,10,11")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    scheds = [int(s) for s in a.scheds.split(",")]
    rows = []
    for shape in a.shapes.split(","):
        M, N, K = map(int, shape.split("x"))
        x = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        w = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        ref = torch.matmul(x, w.t()).float()
        row = {"shape": [M, N, K]}

        def ours(s):
            def f():
                set_gemm_w4_sched(s)
                gemm_nt(x, w, out=out)
            return f

        fns = {f"s{s}": ours(s) for s in scheds}
        fns["torch"] = lambda: torch.matmul(x, w.t(), out=out)
        for s in scheds:
            ours(s)()
            torch.cuda.synchronize()
            err = ((out.float() - ref).abs().max() / ref.abs().max()).item()
            row[f"s{s}_rel_err"] = round(err, 5)
            if err > 2e-2:
                raise SystemExit(f"schedule {s} wrong at {shape}: rel err {err}")
        for f in fns.values():
            time_fn(f, 5)
        t = {k: [] for k in fns}
        names = list(fns)
        for r in range(a.rounds):   # rotate the order every round: a fixed order biases by position
            for k in names[r % len(names):] + names[:r % len(names)]:
                t[k].append(time_fn(fns[k]))
        set_gemm_w4_sched(0)
        flop = 2.0 * M * N * K
        for k, v in t.items():
            us = statistics.median(v)
            row[k + "_us"] = round(us, 1)
            row[k + "_tflops"] = round(flop / us / 1e6, 1)
        for s in scheds:
            row[f"s{s}_vs_torch"] = round(row["torch_us"] / row[f"s{s}_us"], 3)
        rows.append(row)
        print(json.dumps(row), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
