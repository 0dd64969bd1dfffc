"""Causal / full GQA attention on the flash-style gfx950 kernel (native/kernels/attention.hip)."""
from __future__ import annotations

import math

import torch

from . import _lib


ATTN_AUTO, ATTN_V1 = 0, 1


def set_attention_variant(v: int) -> None:
    """``ATTN_AUTO``: the 32x32-MFMA kernels for D = 128 (ping-pong 8-wave block for full
    attention and causal S >= 2048, 4-wave otherwise; 16x16 kernel for D = 64);
    ``ATTN_V1``: always the 4-wave 16x16 kernel (A/B measurement, tests)."""
    _lib.check(_lib.lib().gs_attn_set_variant(int(v)), "gs_attn_set_variant")


def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool = True,
              scale: float | None = None, _debug_gather: bool = False) -> torch.Tensor:
    """``q`` [B, S, Hq, D], ``k``/``v`` [B, S, Hkv, D] (token-major; q/k/v may be strided views
    of one fused QKV buffer as long as heads and head_dim are contiguous). Returns a
    contiguous [B, S, Hq, D] bf16 tensor."""
    for t, nm in ((q, "q"), (k, "k"), (v, "v")):
        if t.dtype != torch.bfloat16 or not t.is_cuda or t.dim() != 4:
            raise ValueError(f"attention: {nm} must be a 4-D bf16 GPU tensor")
        if t.stride(3) != 1 or t.stride(2) != t.shape[3] or t.stride(0) != t.shape[1] * t.stride(1):
            raise ValueError(f"attention: {nm} needs contiguous [H, D] per token and uniform token stride")
    B, S, Hq, D = q.shape
    Hkv = k.shape[2]
    if k.shape != (B, S, Hkv, D) or v.shape != k.shape or Hq % Hkv or D not in (64, 128):
        raise ValueError("attention: shape mismatch (needs D in {64,128} and Hq % Hkv == 0)")
    out = torch.empty((B, S, Hq, D), dtype=torch.bfloat16, device=q.device)
    sc = 1.0 / math.sqrt(D) if scale is None else float(scale)
    rc = _lib.lib().gs_flash_attn_fwd_bf16(q.data_ptr(), k.data_ptr(), v.data_ptr(), out.data_ptr(), B, S, Hq,
                                           Hkv, D, q.stride(1), k.stride(1), v.stride(1), sc,
                                           int(bool(causal)) | (2 if _debug_gather else 0),
                                           _lib.stream_ptr(q.device))
    _lib.check(rc, "gs_flash_attn_fwd_bf16")
    return out


def reference_attention(q, k, v, causal=True, scale=None):
    """fp32 PyTorch reference with GQA head repetition."""
    B, S, Hq, D = q.shape
    rep = Hq // k.shape[2]
    qf = q.float().transpose(1, 2)
    kf = k.float().repeat_interleave(rep, 2).transpose(1, 2)
    vf = v.float().repeat_interleave(rep, 2).transpose(1, 2)
    o = torch.nn.functional.scaled_dot_product_attention(qf, kf, vf, is_causal=causal, scale=scale)
    return o.transpose(1, 2)
