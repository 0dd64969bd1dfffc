#!/usr/bin/env python3
"""Run each GEMM implementation a few times on fixed shapes (for rocprofv3 --pmc passes).

Dispatch order per shape: each variant of PROF_VARIANTS (default "0,1": auto, 2-stage) x R, each
4-wave schedule of PROF_SCHEDS (default none; e.g. "0,9" = streamed vs write-back C stores) x R, then
torch/hipBLASLt x R; the per-dispatch counter rows are attributed by kernel name.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from aliyun_gpushare_device_plugin_amd.ops import gemm_nt  # noqa: E402
from aliyun_gpushare_device_plugin_amd.ops.gemm import GEMM_AUTO, GEMM_V1, set_gemm_variant, set_gemm_w4_sched  # noqa: E402

R = int(os.environ.get("PROF_REPS", "3"))
for s in (sys.argv[1] if len(sys.argv) > 1 else "8192x8192x8192,4096x4096x4096").split(","):
    M, N, K = map(int, s.split("x"))
    x = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
    w = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    for variant in [int(v) for v in os.environ.get("PROF_VARIANTS", f"{GEMM_AUTO},{GEMM_V1}").split(",") if v]:
        set_gemm_variant(variant)
        for _ in range(R):
            gemm_nt(x, w, out=out)
    set_gemm_variant(GEMM_AUTO)
    for sched in [int(v) for v in os.environ.get("PROF_SCHEDS", "").split(",") if v]:
        set_gemm_w4_sched(sched)
        for _ in range(R):
            gemm_nt(x, w, out=out)
    set_gemm_w4_sched(0)
    for _ in range(R):
        torch.matmul(x, w.t(), out=out)
    torch.cuda.synchronize()
print("done")
