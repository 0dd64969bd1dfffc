#!/usr/bin/env python3
"""Serving benchmark: Llama-3-8B bf16 greedy decode with a KV cache on one MI355X.

* decode attention kernel alone vs a PyTorch SDPA decode over the same cache (effective HBM GB/s);
* full decode step: eager launches vs one hipGraph replay per step (tokens/s, ms/step).
Random-init weights (no checkpoints offline); synthetic prompt. Output: JSON lines (and --out).
"""
import argparse
import itertools
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402

from aliyun_gpushare_device_plugin_amd import ops  # noqa: E402


def timed(fn, n, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n


def attn_micro(B, ctx, Hq=32, Hkv=8, D=128, layers=8):
    """Cycles over ``layers`` separate caches (> 1 GB together) so K/V come from HBM, not from the
    256 MB Infinity Cache (a single re-read cache fits in it and reads ~1.7x faster)."""
    caches = []
    for _ in range(layers):
        kc, vc = ops.kv_cache(B, Hkv, ctx, D)
        kc.normal_()
        vc.normal_()
        caches.append((kc, vc))
    lens = torch.full((B,), ctx, dtype=torch.int32, device="cuda")
    q = torch.randn(B, Hq * D, device="cuda", dtype=torch.bfloat16)
    ws = ops.DecodeWorkspace(B, Hq, caches[0][0].shape[2], D)
    out = torch.empty(B, Hq * D, device="cuda", dtype=torch.bfloat16)
    it = {"i": 0}

    def ours():
        kc, vc = caches[it["i"] % layers]
        it["i"] += 1
        return ops.decode_attention(q, kc, vc, lens, ws, out)

    t_ours = timed(ours, 8 * layers)
    from aliyun_gpushare_device_plugin_amd.ops import _lib
    t_pol = {}
    for rnd in range(2):                       # K/V load policy A/B (plain / non-temporal), rotated
        for ntl in ((0, 1) if rnd == 0 else (1, 0)):
            _lib.lib().gs_decode_attn_set_nt(ntl)
            t = timed(ours, 8 * layers)
            t_pol[ntl] = min(t, t_pol.get(ntl, t))
    _lib.lib().gs_decode_attn_set_nt(1)
    qs = q.view(B, Hq, 1, D)

    def sdpa():
        kc, vc = caches[it["i"] % layers]
        it["i"] += 1
        return torch.nn.functional.scaled_dot_product_attention(qs, kc[:, :, :ctx], vc[:, :, :ctx], enable_gqa=True)

    t_sdpa = timed(sdpa, 8 * layers)
    del caches
    nbytes = 2 * B * Hkv * ctx * D * 2
    return {"bench": "decode_attention", "B": B, "ctx": ctx, "ours_us": round(t_ours * 1e6, 1),
            "plain_us": round(t_pol[0] * 1e6, 1), "nt_us": round(t_pol[1] * 1e6, 1),
            "ours_GBps": round(nbytes / t_ours / 1e9, 1), "sdpa_us": round(t_sdpa * 1e6, 1),
            "sdpa_GBps": round(nbytes / t_sdpa / 1e9, 1), "speedup": round(t_sdpa / t_ours, 2)}


class _Rot:
    """``copies`` weights of one shape, handed out round-robin: together > 1 GiB, so a timed loop
    streams W from HBM as a decode step does (one 235 MB weight re-read back to back stays in the
    256 MB Infinity Cache and flatters every kernel, most of all one that loads W cached)."""

    def __init__(self, N, K):
        n = -(-(1 << 30) // (N * K * 2)) + 1
        self.ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) for _ in range(n)]
        self.i = 0

    def next(self):
        self.i += 1
        return self.ws[self.i % len(self.ws)]


def gemm_micro(M, N, K):
    from aliyun_gpushare_device_plugin_amd.ops.gemm import set_skinny_nt

    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    rot = _Rot(N, K)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    nbytes = N * K * 2
    res = {"bench": "skinny_gemm", "M": M, "N": N, "K": K, "w_copies": len(rot.ws)}
    from aliyun_gpushare_device_plugin_amd.ops.gemm import SKINNY_AUTO, SKINNY_LDS, SKINNY_REG, set_skinny_variant

    set_skinny_variant(SKINNY_REG)
    for nt in (1, 2, 4):
        set_skinny_nt(nt)
        t = timed(lambda: ops.skinny_linear(x, rot.next(), out=out), 50)
        res[f"reg_nt{nt}_us"] = round(t * 1e6, 1)
    set_skinny_nt(0)
    set_skinny_variant(SKINNY_LDS)
    from aliyun_gpushare_device_plugin_amd.ops import _lib

    for tgt in (1, 256, 512, 1024, 2048):
        _lib.lib().gs_skinny_set_wg_target(tgt)
        res[f"lds_wg{tgt}_us"] = round(timed(lambda: ops.skinny_linear(x, rot.next(), out=out), 50) * 1e6, 1)
    _lib.lib().gs_skinny_set_wg_target(512)
    res["lds_us"] = res["lds_wg512_us"]
    for nw in (4, 2):
        _lib.lib().gs_skinny_set_lds_waves(nw)
        res[f"lds_nw{nw}_us"] = round(timed(lambda: ops.skinny_linear(x, rot.next(), out=out), 50) * 1e6, 1)
    _lib.lib().gs_skinny_set_lds_waves(0)
    pf0 = _lib.lib().gs_skinny_get_prefetch()
    for rnd in range(2):                   # k-slices in flight, order rotated per round
        for pf in ((0, 1, 2, 3, 4) if rnd == 0 else (4, 3, 2, 1, 0)):
            _lib.lib().gs_skinny_set_prefetch(pf)
            t = timed(lambda: ops.skinny_linear(x, rot.next(), out=out), 50) * 1e6
            res[f"lds_pf{pf}_us"] = round(min(t, res.get(f"lds_pf{pf}_us", t)), 1)
    _lib.lib().gs_skinny_set_prefetch(pf0)
    if N % 64 == 0 and (N // 2) % 32 == 0 and N // 64 >= 256:    # fused SwiGLU (gate/up shape)
        from aliyun_gpushare_device_plugin_amd.ops.gemm import interleave_gate_up
        wils = [interleave_gate_up(v) for v in rot.ws]
        wi = itertools.count()
        for rnd in range(2):
            for pf in ((1, 2, 3, 4) if rnd == 0 else (4, 3, 2, 1)):
                _lib.lib().gs_skinny_set_prefetch(pf)
                t = timed(lambda: ops.skinny_swiglu(x, wils[next(wi) % len(wils)]), 50) * 1e6
                res[f"swiglu_pf{pf}_us"] = round(min(t, res.get(f"swiglu_pf{pf}_us", t)), 1)
        _lib.lib().gs_skinny_set_prefetch(pf0)
    set_skinny_variant(SKINNY_AUTO)
    res["ntauto_us"] = round(timed(lambda: ops.skinny_linear(x, rot.next(), out=out), 50) * 1e6, 1)
    t_ours = res["ntauto_us"] * 1e-6
    t_blas = timed(lambda: torch.matmul(x, rot.next().t()), 50)
    res.update({"ours_GBps": round(nbytes / t_ours / 1e9, 1), "hipblaslt_us": round(t_blas * 1e6, 1),
                "hipblaslt_GBps": round(nbytes / t_blas / 1e9, 1), "speedup": round(t_blas / t_ours, 2)})
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--prompt", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--max-ctx", type=int, default=2048)
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--out", default=None)
    ap.add_argument("--micro-only", action="store_true")
    ap.add_argument("--no-gemm-micro", action="store_true")
    ap.add_argument("--no-attn-micro", action="store_true")
    ap.add_argument("--attn-nt", type=int, default=-1, help="decode attention K/V loads: 0 plain, 1 nt")
    ap.add_argument("--reduce-static", type=int, default=-1, help="skinny split reductions: 1 static counts, 0 loop")
    ap.add_argument("--prefetch", type=int, default=0,
                    help="skinny schedule: 0 auto, 1 one k-slice in flight, 2 two, 3 wave K split, 4 nt W")
    ap.add_argument("--gemms", default="hipblaslt,skinny,skinny_rope",
                    help="decode-step configurations to time")
    a = ap.parse_args()
    if a.reduce_static >= 0:
        from aliyun_gpushare_device_plugin_amd.ops import _lib
        _lib.check(_lib.lib().gs_skinny_set_reduce_static(a.reduce_static), "gs_skinny_set_reduce_static")
    if a.attn_nt >= 0:
        from aliyun_gpushare_device_plugin_amd.ops import _lib
        _lib.check(_lib.lib().gs_decode_attn_set_nt(a.attn_nt), "gs_decode_attn_set_nt")
    if a.prefetch:
        from aliyun_gpushare_device_plugin_amd.ops import _lib
        _lib.check(_lib.lib().gs_skinny_set_prefetch(a.prefetch), "gs_skinny_set_prefetch")
    lines = []

    def emit(d):
        print(json.dumps(d), flush=True)
        lines.append(d)

    for B, ctx in (((32, 1024), (32, 4096), (8, 8192), (64, 2048)) if not a.no_attn_micro else ()):
        emit(attn_micro(B, ctx))
    for M in ((8, 32, 64) if not a.no_gemm_micro else ()):
        for N, K in ((6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336), (128256, 4096)):
            emit(gemm_micro(M, N, K))

    from aliyun_gpushare_device_plugin_amd.models.llama import LlamaConfig, LlamaModel
    from aliyun_gpushare_device_plugin_amd.models.llama_serve import LlamaServer

    if a.micro_only:
        return
    model = LlamaModel(LlamaConfig.llama3_8b(n_layers=a.layers), "cuda", seed=1)
    prompt = torch.randint(0, model.cfg.vocab, (a.batch, a.prompt), device="cuda")
    cfgs = {"hipblaslt": ("hipblaslt", False, False), "skinny": ("skinny", True, False),
            "skinny_rope": ("skinny", True, True)}
    for gemm, fold, rope in [cfgs[k] for k in a.gemms.split(",") if k]:
        srv = LlamaServer(model, a.batch, a.max_ctx, gemm=gemm)
        srv.fold_norm = srv.fold_norm and fold
        srv.fuse_rope = srv.fuse_rope and rope
        torch.cuda.synchronize()
        t = time.perf_counter()
        srv.prefill(prompt)
        torch.cuda.synchronize()
        t_prefill = time.perf_counter() - t
        res = {"bench": "llama3_8b_decode", "gemm": gemm, "skinny_schedule": a.prefetch or "auto", "attn_nt": a.attn_nt,
               "reduce_static": a.reduce_static,
               "fold_norm": srv.fold_norm, "fuse_rope": srv.fuse_rope,
               "batch": a.batch, "prompt": a.prompt, "layers": a.layers,
               "kv_cache_gib": round(srv.kv_bytes() / 2**30, 2),
               "weights_gib": round(model.weight_bytes() / 2**30, 2), "prefill_s": round(t_prefill, 3)}
        half = a.steps // 2
        for mode, use_graph in (("eager", False), ("graph", True)):
            if use_graph:
                srv.capture()
            srv.step(use_graph)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(half):
                srv.step(use_graph)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t) / half
            res[f"{mode}_ms_per_step"] = round(dt * 1e3, 3)
            res[f"{mode}_tokens_per_s"] = round(a.batch / dt, 1)
        res["context_after"] = srv.host_len
        res["graph_speedup"] = round(res["eager_ms_per_step"] / res["graph_ms_per_step"], 2)
        # bytes a step must read: weights (minus the embedding table) + the KV cache up to the context
        kv = 2 * model.cfg.n_layers * a.batch * model.cfg.n_kv_heads * srv.host_len * model.cfg.head_dim * 2
        step_bytes = model.weight_bytes() - model.embed.numel() * 2 + kv
        res["graph_effective_TBps"] = round(step_bytes / (res["graph_ms_per_step"] * 1e-3) / 1e12, 2)
        emit(res)
        del srv
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            for d in lines:
                f.write(json.dumps(d) + "\n")


if __name__ == "__main__":
    main()
