#!/usr/bin/env python3
"""Segment anatomy of the ping-pong attention kernel (variant 10 = the default configuration plus
s_memtime stamps at every segment barrier of block 0, native/kernels/attention.hip).

For each shape prints, per half (waves 0-3 / 4-7), the median cycles a wave spends working in its
MFMA segments and in its softmax segments, and the median barrier wait, plus the median whole
segment (barrier to barrier). s_memtime counts at the constant 100 MHz reference clock on CDNA,
so the tool also reports the kernel's event-timed duration to convert."""
import ctypes
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from aliyun_gpushare_device_plugin_amd.ops import _lib  # noqa: E402
from aliyun_gpushare_device_plugin_amd.ops.attention import ATTN_AUTO, attention, set_attention_variant  # noqa: E402

SEGS = 160


def trace():
    buf = (ctypes.c_ulonglong * (8 * SEGS * 2))()
    _lib.check(_lib.lib().gs_attn_trace(ctypes.cast(buf, ctypes.c_void_p), len(buf)), "gs_attn_trace")
    return [[(buf[(w * SEGS + k) * 2], buf[(w * SEGS + k) * 2 + 1]) for k in range(SEGS)] for w in range(8)]


def main():
    for (B, S, Hq, Hkv, D, causal) in [(16, 2048, 64, 8, 128, False), (1, 8192, 32, 8, 128, True)]:
        q = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16)
        k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
        v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
        set_attention_variant(10)
        for _ in range(3):
            attention(q, k, v, causal=causal)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        attention(q, k, v, causal=causal)
        e.record()
        e.synchronize()
        set_attention_variant(ATTN_AUTO)
        t = trace()
        nkt = (S + 63) // 64
        G = 2 * nkt + 2
        out = {"shape": [B, S, Hq, Hkv, D], "causal": causal, "kernel_ms": round(s.elapsed_time(e), 4),
               "segments": G}
        # segment k of a wave: starts at t[w][k][1] (k >= 1; after the barrier opening it), its work
        # ends at t[w][k][0] (before the barrier closing it); the wait is t[w][k+1][1] - t[w][k][0]
        for half in (0, 1):
            work_m, work_v, wait, whole = [], [], [], []
            for w in range(4 * half, 4 * half + 4):
                for kk in range(2, min(G, SEGS) - 2):
                    st, en, nx = t[w][kk][1], t[w][kk][0], t[w][kk + 1][1]
                    if not (st and en and nx):
                        continue
                    local = kk - half
                    (work_m if local % 2 == 0 else work_v).append(en - st)
                    wait.append(nx - en)
                    whole.append(nx - st)
            med = lambda xs: statistics.median(xs) if xs else None  # noqa: E731
            out[f"half{half}"] = {"mfma_seg_work": med(work_m), "softmax_seg_work": med(work_v),
                                  "barrier_wait": med(wait), "segment": med(whole)}
        t0 = min(t[w][1][1] for w in range(8) if t[w][1][1])
        t1 = max(t[w][G - 1][0] for w in range(8) if t[w][min(G, SEGS) - 1][0]) if G <= SEGS else None
        out["block0_ticks"] = (t1 - t0) if t1 else None
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
