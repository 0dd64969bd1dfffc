#!/usr/bin/env python3
"""Back-to-back vs isolated GEMM dispatches (ours vs torch.matmul/hipBLASLt), event-timed.

Isolated: synchronize before each launch and time that one launch with events, so no dispatch can
overlap its neighbour. Back-to-back: 20 launches between two events. The difference per launch is
what a kernel gains from overlapping with the previous/next dispatch
(profiles/gemm_kernel_trace_4096.md).
"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from aliyun_gpushare_device_plugin_amd.ops import gemm_nt  # noqa: E402


def isolated(fn, n=20):
    ts = []
    for _ in range(n):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    return statistics.median(ts)


def b2b(fn, n=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(n):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / n


out = []
for shape in (sys.argv[1] if len(sys.argv) > 1 else "4096x4096x1024,4096x4096x4096,8192x8192x8192").split(","):
    M, N, K = map(int, shape.split("x"))
    a = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
    b = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    fns = {"ours": lambda: gemm_nt(a, b, out=c), "torch": lambda: torch.matmul(a, b.t(), out=c)}
    for f in fns.values():
        b2b(f, 5)
    row = {"shape": [M, N, K]}
    for rnd in range(3):
        for name, f in fns.items():
            row.setdefault(name + "_isolated_us", []).append(isolated(f))
            row.setdefault(name + "_b2b_us", []).append(b2b(f))
    out.append({k: (round(statistics.median(v), 1) if isinstance(v, list) and k != "shape" else v)
                for k, v in row.items()})
    print(json.dumps(out[-1]), flush=True)
