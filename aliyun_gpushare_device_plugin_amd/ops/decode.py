"""Decode-phase attention over a KV cache and the KV append (native/kernels/decode_attention.hip).

Both ops take their per-sequence lengths / positions from device tensors and never synchronise
with the host, so a whole decode step can be captured once in a hipGraph and replayed
(models/llama_serve.py). Shapes and strides are validated on the host before any launch; the
kernels additionally clamp lengths to the cache capacity and skip positions outside it.
"""
from __future__ import annotations

import math

import torch

from . import _lib

CHUNK = 256          # positions per split workgroup (kernel constant)


def kv_cache(B: int, Hkv: int, Smax: int, D: int = 128, device="cuda") -> tuple[torch.Tensor, torch.Tensor]:
    """K and V caches ``[B, Hkv, Smax, D]`` bf16 (Smax rounded up to the split size)."""
    Smax = -(-Smax // CHUNK) * CHUNK
    mk = lambda: torch.zeros((B, Hkv, Smax, D), dtype=torch.bfloat16, device=device)  # noqa: E731
    return mk(), mk()


def _check_cache(kc: torch.Tensor, vc: torch.Tensor):
    if kc.dtype != torch.bfloat16 or vc.dtype != torch.bfloat16 or kc.shape != vc.shape or kc.dim() != 4:
        raise ValueError("caches must be equal-shape bf16 [B, Hkv, Smax, D]")
    if not (kc.is_contiguous() and vc.is_contiguous()) or kc.shape[3] != 128 or kc.shape[2] % CHUNK:
        raise ValueError("caches must be contiguous with D = 128 and Smax % 256 == 0")


def _rows(t: torch.Tensor, B: int, width: int, name: str) -> int:
    """Row stride of a [B, width] bf16 view whose rows may be slices of a wider buffer."""
    if t.dtype != torch.bfloat16 or not t.is_cuda or t.dim() != 2 or t.shape != (B, width) or t.stride(1) != 1:
        raise ValueError(f"{name}: expected a bf16 GPU [B, {width}] view with contiguous rows")
    if t.stride(0) % 8 or t.data_ptr() % 16:
        raise ValueError(f"{name}: rows must be 16-byte aligned")
    return t.stride(0)


def _ints(t: torch.Tensor, B: int, name: str):
    if t.dtype != torch.int32 or not t.is_cuda or t.shape != (B,) or not t.is_contiguous():
        raise ValueError(f"{name}: expected a contiguous int32 GPU tensor of shape [B]")


def kv_append(k: torch.Tensor, v: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
              pos: torch.Tensor) -> None:
    """``cache[b, :, pos[b]] = new[b]`` for K and V; ``k``/``v`` are ``[B, Hkv * D]`` (may be
    strided slices of the fused QKV output)."""
    _check_cache(k_cache, v_cache)
    B, Hkv, Smax, D = k_cache.shape
    ks = _rows(k, B, Hkv * D, "k")
    if _rows(v, B, Hkv * D, "v") != ks:
        raise ValueError("k and v must share a row stride")
    _ints(pos, B, "pos")
    rc = _lib.lib().gs_kv_append_bf16(k.data_ptr(), v.data_ptr(), ks, k_cache.data_ptr(), v_cache.data_ptr(),
                                      pos.data_ptr(), B, Hkv, D, Smax, _lib.stream_ptr(k.device))
    _lib.check(rc, "gs_kv_append_bf16")


def rope_kv_append(qkv: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, pos: torch.Tensor,
                   k_cache: torch.Tensor, v_cache: torch.Tensor, n_heads: int) -> None:
    """One launch for a decode step's RoPE(q), RoPE(k) (in place in the fused ``qkv`` rows
    ``[B, (Hq + 2 Hkv) * D]``) and the append of rotated k and raw v at ``pos[b]``. Equivalent to
    ``rope_(q); rope_(k); kv_append(k, v)``; positions are not range-checked on the host (the
    kernel clamps table reads and skips cache writes outside it) so the call is graph-safe."""
    _check_cache(k_cache, v_cache)
    B, Hkv, Smax, D = k_cache.shape
    width = (n_heads + 2 * Hkv) * D
    qs = _rows(qkv, B, width, "qkv") if qkv.shape[1] == width else -1
    if qs < 0:
        raise ValueError("rope_kv_append: qkv must be [B, (Hq + 2 Hkv) * D]")
    _ints(pos, B, "pos")
    if (cos.dtype != torch.float32 or sin.shape != cos.shape or cos.dim() != 2 or cos.shape[1] != D // 2
            or not cos.is_contiguous() or not sin.is_contiguous()):
        raise ValueError("rope_kv_append: tables must be contiguous float32 [rows, D / 2]")
    rc = _lib.lib().gs_rope_kv_append_bf16(qkv.data_ptr(), qs, cos.data_ptr(), sin.data_ptr(), cos.shape[0],
                                           pos.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(), B, n_heads, Hkv,
                                           D, Smax, _lib.stream_ptr(qkv.device))
    _lib.check(rc, "gs_rope_kv_append_bf16")


class DecodeWorkspace:
    """Split partials for :func:`decode_attention` (allocated once, reused by every layer/step)."""

    def __init__(self, B: int, Hq: int, Smax: int, D: int = 128, device="cuda"):
        ns = Smax // CHUNK
        self.o = torch.empty((B, Hq, ns, D), dtype=torch.float32, device=device)
        self.ml = torch.empty((B, Hq, ns, 2), dtype=torch.float32, device=device)


def decode_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, lens: torch.Tensor,
                     ws: DecodeWorkspace | None = None, out: torch.Tensor | None = None,
                     scale: float | None = None) -> torch.Tensor:
    """One query token per sequence: ``q`` ``[B, Hq * D]`` (may be a slice of the QKV output)
    attends to positions ``[0, lens[b])`` of its cache rows. Returns ``[B, Hq * D]`` bf16."""
    _check_cache(k_cache, v_cache)
    B, Hkv, Smax, D = k_cache.shape
    Hq = q.shape[1] // D if q.dim() == 2 else -1
    if Hq <= 0 or Hq % Hkv or (Hq // Hkv) not in (1, 2, 4, 8):
        raise ValueError("decode_attention: Hq must be Hkv x {1, 2, 4, 8}")
    qs = _rows(q, B, Hq * D, "q")
    _ints(lens, B, "lens")
    ws = ws or DecodeWorkspace(B, Hq, Smax, D, q.device)
    if ws.o.shape != (B, Hq, Smax // CHUNK, D):
        raise ValueError("decode_attention: workspace shape mismatch")
    out = torch.empty((B, Hq * D), dtype=torch.bfloat16, device=q.device) if out is None else out
    if out.shape != (B, Hq * D) or out.dtype != torch.bfloat16 or not out.is_contiguous():
        raise ValueError("decode_attention: out must be contiguous bf16 [B, Hq * D]")
    sc = 1.0 / math.sqrt(D) if scale is None else float(scale)
    rc = _lib.lib().gs_decode_attn_bf16(q.data_ptr(), qs, k_cache.data_ptr(), v_cache.data_ptr(), lens.data_ptr(),
                                        ws.o.data_ptr(), ws.ml.data_ptr(), out.data_ptr(), B, Hq, Hkv, D, Smax,
                                        sc, _lib.stream_ptr(q.device))
    _lib.check(rc, "gs_decode_attn_bf16")
    return out


def reference_decode_attention(q, k_cache, v_cache, lens, scale=None):
    """fp32 PyTorch reference (per sequence, GQA by head repetition)."""
    B, Hkv, Smax, D = k_cache.shape
    Hq = q.shape[1] // D
    rep = Hq // Hkv
    sc = 1.0 / math.sqrt(D) if scale is None else scale
    outs = []
    for b in range(B):
        n = int(lens[b])
        qb = q[b].float().view(Hq, 1, D)
        kb = k_cache[b, :, :n].float().repeat_interleave(rep, 0)
        vb = v_cache[b, :, :n].float().repeat_interleave(rep, 0)
        p = torch.softmax((qb @ kb.transpose(1, 2)) * sc, -1)
        outs.append((p @ vb).reshape(Hq * D))
    return torch.stack(outs)
