"""``linear`` on the gfx950 MFMA GEMM (native/kernels/gemm_bf16.hip).

``linear(x, w, bias=None, residual=None, silu=False)`` = ``epilogue(x @ w.T)`` for bf16
tensors with fused bias / SiLU / residual-add epilogue. ``Linear`` wraps it in an autograd
Function whose backward also runs on the same NT kernel (operands transposed once):
``dX = dY · W`` as NT with ``Wᵀ``; ``dW = dYᵀ · X`` as NT with ``Xᵀ``.
All shape/alignment requirements are validated on the host before any launch.
"""
from __future__ import annotations

import torch

from . import _lib

EP_BIAS, EP_SILU, EP_RESID, EP_SWIGLU = 1, 2, 4, 8
GEMM_AUTO, GEMM_V1, GEMM_PINGPONG, GEMM_W4 = 0, 1, 2, 4


def set_gemm_group_m(g: int) -> None:
    """Tile-rasterisation group height (rows of tiles sharing an XCD's L2 walk); 0 = default."""
    _lib.check(_lib.lib().gs_gemm_set_group_m(int(g)), "gs_gemm_set_group_m")


def set_gemm_w4_sched(s: int) -> None:
    """Phase-B placement of DMA and fragment reads in the plain 4-wave product (0 = default,
    1..5 = the alternatives in native/kernels/gemm_bf16_w4.hip), for schedule sweeps."""
    _lib.check(_lib.lib().gs_gemm_w4_set_sched(int(s)), "gs_gemm_w4_set_sched")


def set_gemm_variant(v: int) -> None:
    """Kernel selection (A/B measurement, tests): ``GEMM_AUTO`` = the 4-wave AGPR kernel
    (native/kernels/gemm_bf16_w4.hip) for M%256 == N%256 == K%128 == 0 with ldc%8 == 0, else the
    ping-pong 8-phase kernel when aligned, else the 2-stage kernel; ``GEMM_V1`` forces the 2-stage
    kernel, ``GEMM_PINGPONG`` the ping-pong one, ``GEMM_W4`` the 4-wave one where it applies."""
    _lib.check(_lib.lib().gs_gemm_set_variant(int(v)), "gs_gemm_set_variant")


def _check_operand(t: torch.Tensor, name: str):
    if t.dtype != torch.bfloat16:
        raise TypeError(f"{name}: expected bfloat16, got {t.dtype}")
    if not t.is_cuda:
        raise ValueError(f"{name}: expected a GPU tensor")
    if t.stride(-1) != 1:
        raise ValueError(f"{name}: last dimension must be contiguous")


def interleave_gate_up(w: torch.Tensor) -> torch.Tensor:
    """``[gate; up]`` weight rows ([2F, K], gate rows first) -> the layout the fused SwiGLU epilogue
    reads: blocks of 16 gate rows followed by the 16 up rows of the same features."""
    F2, K = w.shape
    if F2 % 32:
        raise ValueError("gate|up rows must be a multiple of 32")
    g, u = w[: F2 // 2], w[F2 // 2:]
    return torch.stack((g.reshape(-1, 16, K), u.reshape(-1, 16, K)), 1).reshape(F2, K).contiguous()


def deinterleave_gate_up(w: torch.Tensor) -> torch.Tensor:
    """Inverse of :func:`interleave_gate_up`: ``[2F, K]`` interleaved rows -> ``[gate; up]``."""
    F2, K = w.shape
    v = w.reshape(F2 // 32, 2, 16, K)
    return torch.cat((v[:, 0].reshape(-1, K), v[:, 1].reshape(-1, K)), 0)


def gemm_nt_repeat(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor, reps: int) -> torch.Tensor:
    """``out = a @ b^T`` computed ``reps`` times in ONE dispatch of the 4-wave kernel (grid.y = reps):
    the GEMM player's burst without a drain at every kernel boundary. Same FLOPs as ``reps`` calls of
    :func:`gemm_nt`; every repetition stores identical values to ``out``. Falls back to a loop of
    :func:`gemm_nt` for shapes the 4-wave kernel does not take (M, N % 256, K % 128, 16-B rows)."""
    _check_operand(a, "a")
    _check_operand(b, "b")
    M, K = a.shape
    N = b.shape[0]
    ok = (b.shape[1] == K and out.shape == (M, N) and out.dtype == torch.bfloat16 and out.stride(1) == 1
          and 1 <= reps <= 65535 and M % 256 == 0 and N % 256 == 0 and K % 128 == 0
          and a.stride(1) == 1 and b.stride(1) == 1 and out.stride(0) % 8 == 0 and out.data_ptr() % 16 == 0
          and a.stride(0) % 8 == 0 and b.stride(0) % 8 == 0 and a.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0)
    if ok:
        rc = _lib.lib().gs_gemm_bf16_nt_repeat(a.data_ptr(), b.data_ptr(), out.data_ptr(), M, N, K, a.stride(0),
                                               b.stride(0), out.stride(0), reps, _lib.stream_ptr(a.device))
        _lib.check(rc, "gs_gemm_bf16_nt_repeat")   # shapes were checked above: any error is real
        return out
    for _ in range(reps):
        gemm_nt(a, b, out=out)
    return out


def gemm_nt(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor | None = None, bias: torch.Tensor | None = None,
            residual: torch.Tensor | None = None, silu: bool = False, swiglu: bool = False) -> torch.Tensor:
    """``out[M,N] = epi(a[M,K] @ b[N,K]^T)``; a and b are 2-D row-major (K contiguous).

    ``swiglu=True``: b holds gate/up rows interleaved by :func:`interleave_gate_up` and the result
    is ``out[M, N/2] = silu(gate) * up`` computed in the GEMM epilogue (aligned shapes only:
    M % 256 == N % 256 == K % 128 == 0; see :func:`linear_swiglu` for the general entry)."""
    _check_operand(a, "a")
    _check_operand(b, "b")
    if a.dim() != 2 or b.dim() != 2 or a.shape[1] != b.shape[1]:
        raise ValueError(f"gemm_nt shapes {tuple(a.shape)} x {tuple(b.shape)}^T")
    M, K = a.shape
    N = b.shape[0]
    if K % 64 or N % 4:
        raise ValueError(f"gemm_nt needs K % 64 == 0 and N % 4 == 0 (K={K}, N={N})")
    lda, ldb = a.stride(0), b.stride(0)
    if lda % 8 or ldb % 8 or a.data_ptr() % 16 or b.data_ptr() % 16:
        a, b = a.contiguous(), b.contiguous()
        lda, ldb = a.stride(0), b.stride(0)
        if lda % 8 or ldb % 8:
            raise ValueError("gemm_nt needs 16-byte aligned rows")
    No = N // 2 if swiglu else N
    if swiglu and (bias is not None or residual is not None or silu or M % 256 or N % 256 or K % 128):
        raise ValueError("swiglu GEMM: no other epilogue, and M % 256 == N % 256 == K % 128 == 0")
    if out is None:
        out = torch.empty((M, No), dtype=torch.bfloat16, device=a.device)
    elif out.shape != (M, No) or out.dtype != torch.bfloat16 or out.stride(1) != 1 or out.stride(0) % 4:
        raise ValueError("bad out tensor")
    flags = EP_SWIGLU if swiglu else 0
    bptr = rptr = None
    if bias is not None:
        if bias.numel() != N or bias.dtype != torch.bfloat16 or not bias.is_contiguous():
            raise ValueError("bias must be a contiguous bf16 vector of length N")
        flags |= EP_BIAS
        bptr = bias.data_ptr()
    if silu:
        flags |= EP_SILU
    if residual is not None:
        if residual.shape != (M, N) or residual.dtype != torch.bfloat16 or residual.stride() != out.stride():
            raise ValueError("residual must match out's shape and strides")
        flags |= EP_RESID
        rptr = residual.data_ptr()
    rc = _lib.lib().gs_gemm_bf16_nt(a.data_ptr(), b.data_ptr(), out.data_ptr(), bptr, rptr, M, N, K, lda, ldb,
                                    out.stride(0), flags, _lib.stream_ptr(a.device))
    _lib.check(rc, "gs_gemm_bf16_nt")
    return out


def linear_swiglu(x: torch.Tensor, w_interleaved: torch.Tensor) -> torch.Tensor:
    """``silu(x @ gate.T) * (x @ up.T)`` for x ``[..., K]`` and gate/up weights interleaved by
    :func:`interleave_gate_up`; fused into the GEMM epilogue when the shape is aligned, else a
    plain GEMM followed by the silu_mul kernel on the de-interleaved activations."""
    from .fused import silu_mul

    lead = x.shape[:-1]
    x2 = x.reshape(-1, x.shape[-1])
    N, K = w_interleaved.shape
    if x2.shape[0] % 256 == 0 and N % 256 == 0 and K % 128 == 0 and x2.stride(-1) == 1:
        y = gemm_nt(x2, w_interleaved, swiglu=True)
    else:
        gu = gemm_nt(x2, w_interleaved)                                  # [M, N] interleaved
        gu = gu.view(-1, N // 32, 2, 16).permute(0, 2, 1, 3).reshape(-1, N).contiguous()
        y = silu_mul(gu)
    return y.reshape(*lead, N // 2)


def linear(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None,
           residual: torch.Tensor | None = None, silu: bool = False) -> torch.Tensor:
    """``epi(x @ w.T)`` for x of any leading shape ``[..., K]``."""
    lead = x.shape[:-1]
    x2 = x.reshape(-1, x.shape[-1])
    r2 = residual.reshape(-1, w.shape[0]) if residual is not None else None
    y = gemm_nt(x2, w, bias=bias, residual=r2, silu=silu)
    return y.reshape(*lead, w.shape[0])


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return linear(x, w)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        g2 = gy.reshape(-1, gy.shape[-1]).contiguous()
        x2 = x.reshape(-1, x.shape[-1])
        gx = gw = None
        if ctx.needs_input_grad[0]:
            gx = gemm_nt(g2, w.t().contiguous()).reshape(x.shape)          # [M,N]·[N,K]
        if ctx.needs_input_grad[1]:
            M = x2.shape[0]
            pad = (-M) % 64   # the contraction (over M) must be a multiple of 64: zero rows add 0
            if pad:
                g2 = torch.nn.functional.pad(g2, (0, 0, 0, pad))
                x2 = torch.nn.functional.pad(x2, (0, 0, 0, pad))
            gw = gemm_nt(g2.t().contiguous(), x2.t().contiguous())         # [N,M]·[M,K]
        return gx, gw


def linear_autograd(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    return _LinearFn.apply(x, w)


def set_skinny_nt(nt: int) -> None:
    """Force the skinny GEMM's features-per-wave factor (1, 2 or 4 tiles of 16); 0 = heuristic."""
    _lib.check(_lib.lib().gs_skinny_set_nt(int(nt)), "gs_skinny_set_nt")


SKINNY_AUTO, SKINNY_REG, SKINNY_LDS = 0, 1, 2


def set_skinny_variant(v: int) -> None:
    """``SKINNY_AUTO``: LDS-staged kernel when K % 256 == 0, else the register kernel;
    ``SKINNY_REG`` / ``SKINNY_LDS`` force one (A/B measurement, tests)."""
    _lib.check(_lib.lib().gs_skinny_set_variant(int(v)), "gs_skinny_set_variant")


def skinny_ssq_ok(N: int, K: int) -> bool:
    """Whether ``skinny_linear(..., ssq_out=...)`` can emit row sums of squares for an ``[N, K]``
    weight: the split reduction writes them, so the shape must split and N % 1024 == 0."""
    return N % 1024 == 0 and K % 256 == 0 and _lib.lib().gs_skinny_splits(N, K) > 1


def skinny_rope_ok(N: int, K: int) -> bool:
    """Whether ``skinny_linear(..., rope=...)`` can apply RoPE and the KV append in its split
    reduction for an ``[N, K]`` QKV weight (the shape must split)."""
    return N % 128 == 0 and K % 256 == 0 and _lib.lib().gs_skinny_splits(N, K) > 1


class _SkinnyOpts:
    """Per-launch options of the native skinny GEMM (set just before the call, cleared after)."""

    def __init__(self, ssq_out=None, norm=None, rope=None):
        self.ssq_out, self.norm, self.rope = ssq_out, norm, rope

    def __enter__(self):
        try:
            return self._arm()
        except BaseException:
            # a partly armed state (RoPE/KV pointers set, opts refused) must never leak into the
            # next unrelated skinny_linear on this thread
            _lib.lib().gs_skinny_clear_opts()
            raise

    def _arm(self):
        if self.rope is not None:
            cos, sin, pos, kc, vc, hq = self.rope
            B, hkv, smax, _ = kc.shape
            _lib.check(_lib.lib().gs_skinny_set_rope(cos.data_ptr(), sin.data_ptr(), cos.shape[0], pos.data_ptr(),
                                                     kc.data_ptr(), vc.data_ptr(), hq, hkv, smax),
                       "gs_skinny_set_rope")
        if self.ssq_out is None and self.norm is None:
            return self
        ssq, w, eps = self.norm if self.norm is not None else (None, None, 0.0)
        nch = ssq.shape[0] if ssq is not None else 0
        _lib.check(_lib.lib().gs_skinny_set_opts(self.ssq_out.data_ptr() if self.ssq_out is not None else None,
                                                 ssq.data_ptr() if ssq is not None else None,
                                                 w.data_ptr() if w is not None else None, nch, float(eps)),
                   "gs_skinny_set_opts")
        return self

    def __exit__(self, *exc):
        if self.ssq_out is not None or self.norm is not None or self.rope is not None:
            _lib.lib().gs_skinny_clear_opts()


def _check_norm(norm, M: int, K: int):
    if norm is None:
        return
    ssq, w, _ = norm
    if ssq.dtype != torch.float32 or ssq.dim() != 2 or ssq.shape[1] != M or not ssq.is_contiguous():
        raise ValueError("norm: ssq must be contiguous float32 [chunks, M]")
    _check_operand(w, "norm weight")
    if w.shape != (K,) or not w.is_contiguous():
        raise ValueError("norm: weight must be contiguous [K]")


def _check_rope(rope, M: int, N: int, K: int, residual):
    cos, sin, pos, kc, vc, hq = rope
    if residual is not None or not skinny_rope_ok(N, K):
        raise ValueError("skinny_linear: rope needs a split shape (skinny_rope_ok) and no residual")
    if (kc.dim() != 4 or kc.shape != vc.shape or kc.dtype != torch.bfloat16 or vc.dtype != torch.bfloat16
            or not kc.is_contiguous() or not vc.is_contiguous() or kc.shape[0] != M or kc.shape[3] != 128):
        raise ValueError("skinny_linear: rope caches must be contiguous bf16 [M, Hkv, Smax, 128]")
    if N != (hq + 2 * kc.shape[1]) * 128:
        raise ValueError("skinny_linear: rope needs N = (n_heads + 2 Hkv) * 128")
    if pos.dtype != torch.int32 or pos.shape != (M,) or not pos.is_contiguous():
        raise ValueError("skinny_linear: rope positions must be contiguous int32 [M]")
    if (cos.dtype != torch.float32 or sin.shape != cos.shape or cos.dim() != 2 or cos.shape[1] != 64
            or not cos.is_contiguous() or not sin.is_contiguous()):
        raise ValueError("skinny_linear: rope tables must be contiguous float32 [rows, 64]")
    for t in (cos, sin, pos, kc, vc):
        if t.device != kc.device:
            raise ValueError("skinny_linear: rope tensors must share a device")


def skinny_linear(x: torch.Tensor, w: torch.Tensor, residual: torch.Tensor | None = None,
                  out: torch.Tensor | None = None, norm_weight: torch.Tensor | None = None, eps: float = 1e-5,
                  ssq_out: torch.Tensor | None = None, norm: tuple | None = None, rope: tuple | None = None):
    """Decode-shaped ``x @ w.T (+ residual)`` for ``x`` ``[M <= 64, K]`` on the split-K skinny
    kernel (native/kernels/gemm_skinny.hip): an HBM stream over ``w`` with the batch as the MFMA's
    16-row operand. ``out`` may be ``residual`` itself (in-place residual add). With
    ``norm_weight`` it returns ``(out, rmsnorm(out) * norm_weight)``, the norm computed in the same
    pass that reduces the K splits (one launch less per residual projection).

    Folded RMSNorm across two projections: ``ssq_out`` (float32 ``[N / 1024, M]``, see
    ``skinny_ssq_ok``) makes this call's split reduction also write the row sums of squares of the
    stored output; a later call with ``norm=(ssq, weight, eps)`` and ``x`` = that output multiplies
    by ``weight`` and ``rsqrt(mean + eps)`` while staging ``x`` — ``rmsnorm(x) * weight`` without a
    norm kernel in between.

    Decode QKV projection: ``rope=(cos, sin, pos, k_cache, v_cache, n_heads)`` makes the split
    reduction also do ``ops.rope_kv_append``'s work (RoPE of the q and k heads at ``pos[b]``, k / v
    appended to the caches) — one launch less per layer; see ``skinny_rope_ok``."""
    _check_operand(x, "x")
    _check_operand(w, "w")
    if x.dim() != 2 or w.dim() != 2 or x.shape[1] != w.shape[1]:
        raise ValueError("skinny_linear: x [M, K] and w [N, K] expected")
    M, K = x.shape
    N = w.shape[0]
    if not 1 <= M <= 64 or N % 64 or K % 32:
        raise ValueError("skinny_linear: needs 1 <= M <= 64, N % 64 == 0, K % 32 == 0")
    if x.stride(0) % 8 or w.stride(0) % 8 or x.data_ptr() % 16 or w.data_ptr() % 16:
        raise ValueError("skinny_linear: rows must be 16-byte aligned")
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=x.device)
    if out.shape != (M, N) or out.dtype != torch.bfloat16 or out.stride(1) != 1 or out.stride(0) % 4:
        raise ValueError("skinny_linear: out must be bf16 [M, N] with contiguous rows")
    rptr = None
    if residual is not None:
        if residual.shape != (M, N) or residual.dtype != torch.bfloat16 or residual.stride() != out.stride():
            raise ValueError("skinny_linear: residual must match out's shape and strides")
        rptr = residual.data_ptr()
    L = _lib.lib()
    splits = L.gs_skinny_splits(N, K)
    part = torch.empty(splits * M * N, dtype=torch.float32, device=x.device) if splits > 1 else None
    pptr = part.data_ptr() if part is not None else None
    if ssq_out is not None:
        if norm_weight is not None or not skinny_ssq_ok(N, K):
            raise ValueError("skinny_linear: ssq_out needs a split shape with N % 1024 == 0 and no norm_weight")
        if ssq_out.dtype != torch.float32 or tuple(ssq_out.shape) != (N // 1024, M) or not ssq_out.is_contiguous():
            raise ValueError("skinny_linear: ssq_out must be contiguous float32 [N / 1024, M]")
    _check_norm(norm, M, K)
    if rope is not None:
        _check_rope(rope, M, N, K, residual)
    if norm_weight is None:
        with _SkinnyOpts(ssq_out, norm, rope):
            rc = L.gs_skinny_gemm_bf16(x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), out.data_ptr(), rptr,
                                       out.stride(0), M, N, K, splits, pptr, _lib.stream_ptr(x.device))
        _lib.check(rc, "gs_skinny_gemm_bf16")
        return out
    if norm is not None or rope is not None:
        raise ValueError("skinny_linear: norm_weight excludes norm and rope")
    _check_operand(norm_weight, "norm_weight")
    if norm_weight.shape != (N,) or not norm_weight.is_contiguous() or N > 8192 or out.stride(0) % 8:
        raise ValueError("skinny_linear: norm_weight must be contiguous [N] with N <= 8192")
    xn = torch.empty((M, N), dtype=torch.bfloat16, device=x.device)
    rc = L.gs_skinny_gemm_norm_bf16(x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), out.data_ptr(), rptr,
                                    out.stride(0), M, N, K, splits, pptr, norm_weight.data_ptr(), xn.data_ptr(),
                                    N, float(eps), _lib.stream_ptr(x.device))
    _lib.check(rc, "gs_skinny_gemm_norm_bf16")
    return out, xn


def skinny_swiglu(x: torch.Tensor, w_il: torch.Tensor, norm: tuple | None = None) -> torch.Tensor | None:
    """Decode MLP up-projection with the SwiGLU fused into the skinny GEMM's epilogue:
    ``silu(x @ gate.T) * (x @ up.T)`` for ``w_il`` ``[2F, K]`` in the ``interleave_gate_up``
    layout, one launch, ``[M, F]`` out. Returns ``None`` where the shape needs split-K (narrow
    weights): the caller then runs ``skinny_linear`` + ``silu_mul(interleaved=True)``."""
    _check_operand(x, "x")
    _check_operand(w_il, "w_il")
    if x.dim() != 2 or w_il.dim() != 2 or x.shape[1] != w_il.shape[1]:
        raise ValueError("skinny_swiglu: x [M, K] and w_il [2F, K] expected")
    M, K = x.shape
    F = w_il.shape[0] // 2
    if x.stride(0) % 8 or w_il.stride(0) % 8 or x.data_ptr() % 16 or w_il.data_ptr() % 16:
        raise ValueError("skinny_swiglu: rows must be 16-byte aligned")
    _check_norm(norm, M, K)
    y = torch.empty((M, F), dtype=torch.bfloat16, device=x.device)
    with _SkinnyOpts(None, norm):
        rc = _lib.lib().gs_skinny_swiglu_bf16(x.data_ptr(), x.stride(0), w_il.data_ptr(), w_il.stride(0),
                                              y.data_ptr(), F, M, F, K, _lib.stream_ptr(x.device))
    if rc == 1:            # GS_EINVAL: shape outside the fused path
        return None
    _lib.check(rc, "gs_skinny_swiglu_bf16")
    return y

