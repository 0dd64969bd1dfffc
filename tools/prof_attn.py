#!/usr/bin/env python3
"""Run each attention kernel variant 3x at one shape (for rocprofv3 --pmc passes)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from aliyun_gpushare_device_plugin_amd.ops.attention import attention, set_attention_variant  # noqa: E402

B, S, Hq, Hkv, D = 4, 2048, 32, 8, 128
q = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16)
k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
for var in (1, 2, 3):
    set_attention_variant(var)
    for _ in range(3):
        attention(q, k, v, causal=True)
torch.cuda.synchronize()
print("done")
