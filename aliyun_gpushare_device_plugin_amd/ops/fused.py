"""Fused memory-bound ops for the demo Llama workload (native/kernels/elementwise.hip)."""
from __future__ import annotations

import torch

from . import _lib


def _bf16_cuda(t: torch.Tensor, name: str):
    if t.dtype != torch.bfloat16 or not t.is_cuda or not t.is_contiguous():
        raise ValueError(f"{name}: expected a contiguous bf16 GPU tensor")


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float = 1e-5, residual: torch.Tensor | None = None):
    """``rmsnorm(x [+ residual]) * w``. With ``residual`` it returns ``(y, x + residual)``
    (the updated residual stream) from one pass over memory."""
    _bf16_cuda(x, "x")
    _bf16_cuda(w, "w")
    H = x.shape[-1]
    M = x.numel() // H
    if w.numel() != H or H % 8 or H > 8192:
        raise ValueError("rmsnorm needs H % 8 == 0, H <= 8192 and w of length H")
    y = torch.empty_like(x)
    if residual is not None:
        _bf16_cuda(residual, "residual")
        if residual.shape != x.shape:
            raise ValueError("residual shape mismatch")
        r_out = torch.empty_like(x)
        rc = _lib.lib().gs_rmsnorm_bf16(x.data_ptr(), residual.data_ptr(), r_out.data_ptr(), w.data_ptr(),
                                        y.data_ptr(), M, H, float(eps), _lib.stream_ptr(x.device))
        _lib.check(rc, "gs_rmsnorm_bf16")
        return y, r_out
    rc = _lib.lib().gs_rmsnorm_bf16(x.data_ptr(), None, None, w.data_ptr(), y.data_ptr(), M, H, float(eps),
                                    _lib.stream_ptr(x.device))
    _lib.check(rc, "gs_rmsnorm_bf16")
    return y


def silu_mul(gu: torch.Tensor, interleaved: bool = False) -> torch.Tensor:
    """``silu(gu[..., :F]) * gu[..., F:]`` for the concatenated gate|up projection, or with
    ``interleaved=True`` for the gate/up-interleaved-by-16 layout of ``ops.interleave_gate_up``
    weights (read in place, no de-interleave copy)."""
    _bf16_cuda(gu, "gu")
    F2 = gu.shape[-1]
    if F2 % (32 if interleaved else 16) or not gu.is_contiguous():
        raise ValueError("silu_mul needs a contiguous tensor whose last dim is a multiple of 16 (32 interleaved)")
    F = F2 // 2
    M = gu.numel() // F2
    y = torch.empty((*gu.shape[:-1], F), dtype=gu.dtype, device=gu.device)
    fn = _lib.lib().gs_silu_mul_il_bf16 if interleaved else _lib.lib().gs_silu_mul_bf16
    rc = fn(gu.data_ptr(), y.data_ptr(), M, F, _lib.stream_ptr(gu.device))
    _lib.check(rc, "gs_silu_mul_bf16")
    return y


def rope_tables(seq_len: int, head_dim: int, theta: float = 500000.0, device="cuda"):
    """Host-side precomputed cos/sin tables (Appendix B: no trig on the device)."""
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    ang = torch.outer(torch.arange(seq_len, dtype=torch.float64), inv)
    return ang.cos().float().to(device).contiguous(), ang.sin().float().to(device).contiguous()


def rope_(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, nheads: int, head_dim: int,
          seq_len: int, positions: torch.Tensor | None = None, validate: bool = True) -> torch.Tensor:
    """In-place rotate-half RoPE on ``x`` viewed as ``[T, nheads, head_dim]`` with token
    stride ``x.stride(-2)`` (so q/k slices of a fused qkv buffer work without copies).
    ``validate=False`` skips the host-side range check of ``positions`` (it synchronises), for
    callers that guarantee the range themselves and capture the launch in a hipGraph."""
    if x.dtype != torch.bfloat16 or not x.is_cuda or x.stride(-1) != 1:
        raise ValueError("rope_: expected bf16 GPU tensor with contiguous last dim")
    if head_dim % 8 or cos.dim() != 2 or cos.shape[0] < seq_len or cos.shape[1] != head_dim // 2 \
            or sin.shape != cos.shape or not cos.is_contiguous() or not sin.is_contiguous():
        raise ValueError("rope_: tables must be contiguous [>= seq_len, head_dim/2]")
    x2 = x.reshape(-1, x.shape[-1]) if x.dim() > 2 else x
    T, stride = x2.shape[0], x2.stride(0)
    if x2.shape[-1] < nheads * head_dim:
        raise ValueError("rope_: row narrower than nheads*head_dim")
    pos = None
    if positions is not None:
        if positions.dtype != torch.int32 or not positions.is_contiguous():
            positions = positions.to(torch.int32).contiguous()
        if positions.numel() != T:
            raise ValueError("rope_: positions must have one entry per token")
        if validate and (int(positions.max()) >= cos.shape[0] or int(positions.min()) < 0):
            raise ValueError("rope_: position outside the table")
        pos = positions.data_ptr()
    rc = _lib.lib().gs_rope_bf16(x2.data_ptr(), cos.data_ptr(), sin.data_ptr(), pos, T, nheads, head_dim, stride,
                                 seq_len, _lib.stream_ptr(x.device))
    _lib.check(rc, "gs_rope_bf16")
    return x


def argmax_rows(x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """Greedy sampling: ``torch.argmax(x, -1)`` for bf16 ``x`` ``[B, V]`` (rows may be strided;
    first index of the maximum, NaN counted as the maximum) into int64 ``out`` ``[B]``, one
    launch (torch's argmax is a generic reduction plus a copy into the token buffer)."""
    if x.dtype != torch.bfloat16 or not x.is_cuda or x.dim() != 2 or x.stride(1) != 1:
        raise ValueError("argmax_rows: expected a bf16 GPU [B, V] tensor with contiguous rows")
    B, V = x.shape
    if x.stride(0) % 8 or x.data_ptr() % 16:
        raise ValueError("argmax_rows: rows must be 16-byte aligned")
    out = torch.empty(B, dtype=torch.long, device=x.device) if out is None else out
    if out.dtype != torch.long or out.shape != (B,) or not out.is_contiguous() or out.device != x.device:
        raise ValueError("argmax_rows: out must be a contiguous int64 [B] tensor on x's device")
    rc = _lib.lib().gs_argmax_rows_bf16(x.data_ptr(), x.stride(0), B, V, out.data_ptr(), _lib.stream_ptr(x.device))
    _lib.check(rc, "gs_argmax_rows_bf16")
    return out
