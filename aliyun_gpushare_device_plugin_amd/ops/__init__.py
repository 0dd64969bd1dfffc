"""Hand-written gfx950 HIP kernels exposed to PyTorch (MFMA GEMM, fused norm/act/RoPE, attention)."""
from .gemm import gemm_nt, linear, linear_autograd  # noqa: F401
from .fused import rmsnorm, rope_, rope_tables, silu_mul  # noqa: F401
from .attention import attention, reference_attention  # noqa: F401
