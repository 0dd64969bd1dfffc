"""Hand-written gfx950 HIP kernels exposed to PyTorch (MFMA GEMM, fused norm/act/RoPE, attention)."""
from .gemm import (deinterleave_gate_up, gemm_nt, gemm_nt_repeat, interleave_gate_up, linear, linear_autograd,  # noqa: F401
                   linear_swiglu, skinny_linear, skinny_rope_ok, skinny_ssq_ok,
                   skinny_swiglu)
from .fused import argmax_rows, rmsnorm, rope_, rope_tables, silu_mul  # noqa: F401
from .attention import attention, reference_attention  # noqa: F401
from .census import cu_census  # noqa: F401
from .decode import DecodeWorkspace, decode_attention, kv_append, kv_cache, rope_kv_append  # noqa: F401
