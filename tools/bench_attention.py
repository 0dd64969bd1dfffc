#!/usr/bin/env python3
"""Flash-attention forward (native/kernels/attention.hip) vs torch SDPA on the Llama-3-8B prefill
shape; interleaved rounds, median; FLOPs counted causal (half of 4*B*Hq*S^2*D)."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from aliyun_gpushare_device_plugin_amd.ops.attention import ATTN_AUTO, ATTN_V1, attention, set_attention_variant  # noqa: E402


def timed(fn, iters=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


res = []
for (B, S, Hq, Hkv, D) in [(4, 2048, 32, 8, 128), (1, 8192, 32, 8, 128), (8, 1024, 32, 8, 128)]:
    q = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
    qt, kt, vt = q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)   # [B, H, S, D] views for SDPA

    def ours():
        set_attention_variant(ATTN_AUTO)
        attention(q, k, v, causal=True)

    def v1():
        set_attention_variant(ATTN_V1)
        attention(q, k, v, causal=True)

    def w8():
        set_attention_variant(3)
        attention(q, k, v, causal=True)

    def ref():
        F.scaled_dot_product_attention(qt, kt, vt, is_causal=True, enable_gqa=True)

    fns = {"ours": ours, "v1": v1, "w8": w8, "sdpa": ref}
    for f in fns.values():
        f()
    torch.cuda.synchronize()
    times = {k_: [] for k_ in fns}
    for _ in range(5):
        for k_, f in fns.items():
            times[k_].append(timed(f))
    set_attention_variant(ATTN_AUTO)
    flop = 4.0 * B * Hq * S * S * D / 2
    row = {"shape": [B, S, Hq, Hkv, D]}
    for k_, t in times.items():
        med = statistics.median(t)
        row[f"{k_}_ms"] = round(med, 4)
        row[f"{k_}_tflops"] = round(flop / med / 1e9, 1)
    row["speedup_vs_sdpa"] = round(row["sdpa_ms"] / row["ours_ms"], 3)
    print(json.dumps(row), flush=True)
    res.append(row)
