#!/usr/bin/env python3
"""Time a 4096^3 bf16 GEMM (hand-written MFMA kernel and torch.matmul) in THIS process, so the
caller can compare HSA_CU_MASK / ROC_GLOBAL_CU_MASK settings (the env is read at runtime init)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from aliyun_gpushare_device_plugin_amd.ops import gemm_nt  # noqa: E402


def timeit(fn, n=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


n = int(os.environ.get("GEMM_N", "4096"))
a = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
b = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
ms_ours = timeit(lambda: gemm_nt(a, b))
ms_torch = timeit(lambda: a @ b.t())
fl = 2.0 * n ** 3
print(json.dumps({"HSA_CU_MASK": os.environ.get("HSA_CU_MASK"), "ROC_GLOBAL_CU_MASK": os.environ.get("ROC_GLOBAL_CU_MASK"),
                  "n": n, "ours_ms": round(ms_ours, 4), "ours_tflops": round(fl / ms_ours / 1e9, 1),
                  "torch_ms": round(ms_torch, 4), "torch_tflops": round(fl / ms_torch / 1e9, 1)}), flush=True)
