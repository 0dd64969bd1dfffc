"""Loader for ``libgpushare_kernels.so`` (hand-written gfx950 HIP kernels, native/kernels/).

The library is loaded with ctypes into the PyTorch process; it links the same
``libamdhip64.so.7`` soname PyTorch already loaded, so kernels run on PyTorch's streams.
There is deliberately no eager fallback: on a GPU box a missing or failing kernel raises.
"""
from __future__ import annotations

import ctypes
import threading

from ..utils.native import ensure_built

_lib = None
_lock = threading.Lock()

_c = ctypes
_P, _I, _F = _c.c_void_p, _c.c_int, _c.c_float

SIGNATURES = {
    "gs_gemm_bf16_nt": [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P],
    "gs_gemm_bf16_nt_repeat": [_P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P],
    "gs_gemm_set_variant": [_I],
    "gs_gemm_set_group_m": [_I],
    "gs_gemm_w4_set_sched": [_I],
    "gs_rmsnorm_bf16": [_P, _P, _P, _P, _P, _I, _I, _F, _P],
    "gs_silu_mul_bf16": [_P, _P, _I, _I, _P],
    "gs_rope_bf16": [_P, _P, _P, _P, _I, _I, _I, _I, _I, _P],
    "gs_flash_attn_fwd_bf16": [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _F, _I, _P],
    "gs_attn_set_variant": [_I],
    "gs_attn_trace": [_P, _I],
    "gs_cu_census": [_P, _I, _I, _P],
    "gs_decode_attn_bf16": [_P, _I, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _F, _P],
    "gs_kv_append_bf16": [_P, _P, _I, _P, _P, _P, _I, _I, _I, _I, _P],
    "gs_skinny_gemm_bf16": [_P, _I, _P, _I, _P, _P, _I, _I, _I, _I, _I, _P, _P],
    "gs_skinny_splits": [_I, _I],
    "gs_skinny_swiglu_bf16": [_P, _I, _P, _I, _P, _I, _I, _I, _I, _P],
    "gs_skinny_set_opts": [_P, _P, _P, _I, _F],
    "gs_skinny_clear_opts": [],
    "gs_skinny_gemm_norm_bf16": [_P, _I, _P, _I, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P, _I, _F, _P],
    "gs_rope_kv_append_bf16": [_P, _I, _P, _P, _I, _P, _P, _P, _I, _I, _I, _I, _I, _P],
    "gs_silu_mul_il_bf16": [_P, _P, _I, _I, _P],
    "gs_skinny_set_nt": [_I],
    "gs_skinny_set_variant": [_I],
    "gs_skinny_set_wg_target": [_I],
    "gs_skinny_set_rope": [_P, _P, _I, _P, _P, _P, _I, _I, _I],
    "gs_skinny_set_lds_waves": [_I],
    "gs_skinny_set_prefetch": [_I],
    "gs_skinny_get_prefetch": [],
    "gs_decode_attn_set_nt": [_I],
    "gs_skinny_set_reduce_static": [_I],
    "gs_argmax_rows_bf16": [_P, _I, _I, _I, _P, _P],
}

ERRORS = {1: "invalid arguments", 2: "kernel launch failed"}


class KernelError(RuntimeError):
    pass


def lib():
    global _lib
    with _lock:
        if _lib is None:
            L = ctypes.CDLL(ensure_built("kernels"))
            for name, argtypes in SIGNATURES.items():
                fn = getattr(L, name, None)
                if fn is None:
                    continue
                fn.argtypes = argtypes
                fn.restype = _I
            _lib = L
    return _lib


def check(rc: int, what: str):
    if rc != 0:
        raise KernelError(f"{what}: {ERRORS.get(rc, rc)}")


def stream_ptr(device=None) -> int:
    import torch

    return torch.cuda.current_stream(device).cuda_stream


def loaded_path() -> str | None:
    return getattr(_lib, "_name", None)
