#!/usr/bin/env python3
"""Flash-attention forward kernel variants, causal and full, TF/s (event-timed median).

usage: attn_sweep.py [variant ...]   (default: 2 3 4; 0 = auto)
Shapes: the Llama-3-8B prefill shapes (Hq 32, Hkv 8) plus the H 64 / Hkv 8 / N 2048 full-attention
shape. Full: 4 B Hq S^2 D FLOPs; causal: half. One JSON line per (shape, causal)."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from aliyun_gpushare_device_plugin_amd.ops.attention import ATTN_AUTO, attention, set_attention_variant  # noqa: E402


def timed(fn, iters=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def main():
    variants = [int(x) for x in sys.argv[1:]] or [2, 3, 4]
    shapes = [(16, 2048, 64, 8, 128, False), (4, 2048, 32, 8, 128, True), (1, 8192, 32, 8, 128, True),
              (8, 1024, 32, 8, 128, True), (4, 2048, 32, 8, 128, False)]
    for (B, S, Hq, Hkv, D, causal) in shapes:
        torch.manual_seed(0)
        q = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16)
        k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
        v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
        ref = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2),
                                             is_causal=causal, enable_gqa=True).transpose(1, 2)
        row = {"shape": [B, S, Hq, Hkv, D], "causal": causal}
        flop = 4.0 * B * Hq * S * S * D / (2 if causal else 1)
        fns = {}
        for var in variants:
            def f(var=var):
                set_attention_variant(var)
                return attention(q, k, v, causal=causal)
            out = f()
            err = (out.float() - ref.float()).abs().max().item()
            row[f"v{var}_maxerr"] = round(err, 4)
            fns[f"v{var}"] = f
        fns["sdpa"] = lambda: F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2),
                                                             is_causal=causal, enable_gqa=True)
        torch.cuda.synchronize()
        times = {k_: [] for k_ in fns}
        names = list(fns)
        for r in range(5):   # order rotated every round (a fixed order biases by slot)
            for k_ in names[r % len(names):] + names[:r % len(names)]:
                times[k_].append(timed(fns[k_]))
        for k_, t in times.items():
            med = statistics.median(t)
            row[f"{k_}_tflops"] = round(flop / med / 1e9, 1)
        set_attention_variant(ATTN_AUTO)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
