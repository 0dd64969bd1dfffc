#!/usr/bin/env python3
"""Sweep the GEMM tile-rasterisation group height (GROUP_M) for the default kernel."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from aliyun_gpushare_device_plugin_amd.ops import gemm_nt  # noqa: E402
from aliyun_gpushare_device_plugin_amd.ops.gemm import set_gemm_group_m  # noqa: E402


def t(fn, iters=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


res = []
for shape in sys.argv[1].split(",") if len(sys.argv) > 1 else ["4096x4096x4096", "8192x8192x8192", "4096x14336x4096"]:
    M, N, K = map(int, shape.split("x"))
    x = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
    w = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    row = {"shape": shape}
    gms = [int(g) for g in os.environ.get("GMS", "1,2,4,8,16,32").split(",")]
    times = {g: [] for g in gms}
    times["torch"] = []
    for g in gms:
        set_gemm_group_m(g)
        gemm_nt(x, w, out=out)
    for _ in range(int(os.environ.get("ROUNDS", "5"))):
        for g in gms:
            set_gemm_group_m(g)
            times[g].append(t(lambda: gemm_nt(x, w, out=out)))
        times["torch"].append(t(lambda: torch.matmul(x, w.t(), out=out)))
    set_gemm_group_m(0)
    for g in times:
        row[f"gm{g}_tflops" if g != "torch" else "torch_tflops"] = round(2.0 * M * N * K / statistics.median(times[g]) / 1e9, 1)
    print(json.dumps(row), flush=True)
    res.append(row)
