#!/usr/bin/env python3
"""Decode attention in model-like conditions: cache capacity (Smax) larger than the live context,
ragged last split. Cycles over 8 caches (> L2 + MALL), event-timed per call, prints JSON lines."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from aliyun_gpushare_device_plugin_amd import ops  # noqa: E402


def run(B, ctx, smax, Hq=32, Hkv=8, D=128, layers=8, iters=64):
    caches = []
    for _ in range(layers):
        kc, vc = ops.kv_cache(B, Hkv, smax, D)
        kc.normal_()
        vc.normal_()
        caches.append((kc, vc))
    lens = torch.full((B,), ctx, dtype=torch.int32, device="cuda")
    q = torch.randn(B, Hq * D, device="cuda", dtype=torch.bfloat16)
    ws = ops.DecodeWorkspace(B, Hq, caches[0][0].shape[2], D)
    out = torch.empty(B, Hq * D, device="cuda", dtype=torch.bfloat16)
    for i in range(layers):
        ops.decode_attention(q, *caches[i], lens, ws, out)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for i in range(iters):
        ops.decode_attention(q, *caches[i % layers], lens, ws, out)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / iters
    nbytes = 2 * B * Hkv * ctx * D * 2
    return {"B": B, "ctx": ctx, "smax": caches[0][0].shape[2], "us": round(dt * 1e6, 1), "GBps": round(nbytes / dt / 1e9)}


if __name__ == "__main__":
    for B, ctx, smax in ((32, 1024, 1024), (32, 1024, 2048), (32, 1090, 2048), (32, 1090, 1280), (32, 1280, 2048),
                         (32, 1024, 4096), (32, 2048, 2048)):
        print(json.dumps(run(B, ctx, smax)), flush=True)
