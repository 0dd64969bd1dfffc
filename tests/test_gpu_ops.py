"""Numerics of the hand-written gfx950 kernels against plain PyTorch fp32 references."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _seed():
    torch.manual_seed(0)


def ref_linear(a, b, bias=None, residual=None, silu=False):
    y = a.float() @ b.float().t()
    if bias is not None:
        y = y + bias.float()
    if silu:
        y = torch.nn.functional.silu(y)
    if residual is not None:
        y = y + residual.float()
    return y


def assert_close_bf16(out, ref, k):
    # bf16 output rounding (2^-8 relative) + fp32 accumulation over k terms of O(1) products
    err = (out.float() - ref).abs()
    tol = 2e-2 * ref.abs() + 2e-3 * (k ** 0.5)
    bad = (err > tol).sum().item()
    assert bad == 0, f"{bad} elements out of tolerance, max err {err.max().item()}"


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 768, 256), (4096, 4096, 4096), (1, 256, 128),
                                   (300, 1000, 192), (8192, 1024, 512), (17, 4, 64)])
def test_gemm_nt_matches_fp32(M, N, K):
    from aliyun_gpushare_device_plugin_amd.ops import gemm_nt
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    out = gemm_nt(a, b)
    torch.cuda.synchronize()
    assert_close_bf16(out, ref_linear(a, b), K)


@pytest.mark.parametrize("M,N,K,reps", [(256, 256, 128, 1), (512, 768, 256, 3), (2048, 1024, 1024, 5),
                                        (300, 256, 192, 2)])
def test_gemm_nt_repeat_matches_fp32(M, N, K, reps):
    """One dispatch of `reps` identical GEMMs (grid.y) gives the single GEMM's result; the
    unaligned shape takes the loop fallback."""
    from aliyun_gpushare_device_plugin_amd.ops import gemm_nt, gemm_nt_repeat
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    out = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
    gemm_nt_repeat(a, b, out, reps)
    torch.cuda.synchronize()
    assert_close_bf16(out, ref_linear(a, b), K)
    assert torch.equal(out, gemm_nt(a, b))


@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (256, 256, 64), (512, 768, 256), (2048, 1024, 4096),
                                   (4096, 4096, 4096)])
def test_gemm_pingpong_matches_v1_and_fp32(M, N, K):
    """The 8-phase ping-pong and 4-wave kernels (aligned shapes) against fp32 and the 2-stage kernel."""
    from aliyun_gpushare_device_plugin_amd.ops import gemm_nt
    from aliyun_gpushare_device_plugin_amd.ops.gemm import GEMM_AUTO, GEMM_V1, set_gemm_variant
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    try:
        set_gemm_variant(GEMM_V1)
        o1 = gemm_nt(a, b)
        outs = []
        for v in (2, 4):
            set_gemm_variant(v)
            outs.append(gemm_nt(a, b))
        torch.cuda.synchronize()
    finally:
        set_gemm_variant(GEMM_AUTO)
    ref = ref_linear(a, b)
    for o2 in outs:
        assert_close_bf16(o2, ref, K)
        # same fp32 accumulation order per k-step -> bitwise-identical or 1-ulp bf16 differences
        assert (o1.float() - o2.float()).abs().max().item() <= (o1.float().abs().max().item() * 2 ** -7)


@pytest.mark.parametrize("sched", range(16))
@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (512, 768, 512), (2048, 1024, 1024)])
def test_gemm_w4_schedules_bitwise_equal(sched, M, N, K):
    """Every phase-B schedule of the 4-wave kernel moves only where DMA and fragment reads issue,
    not the accumulation order: bitwise-equal to the default schedule and within fp32 tolerance."""
    from aliyun_gpushare_device_plugin_amd.ops import gemm_nt
    from aliyun_gpushare_device_plugin_amd.ops.gemm import set_gemm_w4_sched
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    try:
        set_gemm_w4_sched(0)
        o0 = gemm_nt(a, b)
        set_gemm_w4_sched(sched)
        o = gemm_nt(a, b)
        torch.cuda.synchronize()
    finally:
        set_gemm_w4_sched(0)
    assert torch.equal(o, o0)
    assert_close_bf16(o, ref_linear(a, b), K)


def test_gemm_identity_asymmetric():
    """A = I with an asymmetric B catches a transposed C-write (guide §3)."""
    from aliyun_gpushare_device_plugin_amd.ops import gemm_nt
    K = 256
    a = torch.eye(K, device="cuda", dtype=torch.bfloat16)
    b = (torch.arange(512 * K, device="cuda") % 251).reshape(512, K).to(torch.bfloat16)
    out = gemm_nt(a, b)   # = I @ b^T = b^T
    assert torch.equal(out, b.t().contiguous())


@pytest.mark.parametrize("variant", [0, 2, 4])
def test_gemm_identity_asymmetric_aligned(variant):
    """Same check on an aligned shape for every kernel (auto = 4-wave, ping-pong, 4-wave forced)."""
    from aliyun_gpushare_device_plugin_amd.ops import gemm_nt
    from aliyun_gpushare_device_plugin_amd.ops.gemm import GEMM_AUTO, set_gemm_variant
    K = 512
    a = torch.eye(K, device="cuda", dtype=torch.bfloat16)
    b = (torch.arange(768 * K, device="cuda") % 251).reshape(768, K).to(torch.bfloat16)
    try:
        set_gemm_variant(variant)
        out = gemm_nt(a, b)
        torch.cuda.synchronize()
    finally:
        set_gemm_variant(GEMM_AUTO)
    assert torch.equal(out, b.t().contiguous())


@pytest.mark.parametrize("variant", [0, 2, 4])
def test_gemm_fused_epilogues_aligned(variant):
    from aliyun_gpushare_device_plugin_amd.ops import gemm_nt
    from aliyun_gpushare_device_plugin_amd.ops.gemm import GEMM_AUTO, set_gemm_variant
    M, N, K = 512, 768, 1024
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.1
    bias = torch.randn(N, device="cuda", dtype=torch.bfloat16)
    res = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    try:
        set_gemm_variant(variant)
        out = gemm_nt(a, b, bias=bias, residual=res, silu=True)
        torch.cuda.synchronize()
    finally:
        set_gemm_variant(GEMM_AUTO)
    assert_close_bf16(out, ref_linear(a, b, bias, res, silu=True), K)


@pytest.mark.parametrize("M,F,K", [(256, 128, 128), (512, 1024, 512), (8192, 2048, 4096), (300, 256, 192)])
def test_linear_swiglu_matches_fp32(M, F, K):
    """Fused SwiGLU epilogue (aligned) and its unfused fallback against silu(x g^T) * (x u^T)."""
    from aliyun_gpushare_device_plugin_amd.ops import deinterleave_gate_up, interleave_gate_up, linear_swiglu
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(2 * F, K, device="cuda", dtype=torch.bfloat16) * 0.05
    wi = interleave_gate_up(w)
    assert torch.equal(deinterleave_gate_up(wi), w)
    out = linear_swiglu(x, wi)
    torch.cuda.synchronize()
    g, u = ref_linear(x, w[:F]), ref_linear(x, w[F:])
    ref = torch.nn.functional.silu(g) * u
    assert out.shape == (M, F)
    assert_close_bf16(out, ref, K)


def test_gemm_fused_epilogues():
    from aliyun_gpushare_device_plugin_amd.ops import gemm_nt
    M, N, K = 384, 512, 320
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.1
    bias = torch.randn(N, device="cuda", dtype=torch.bfloat16)
    res = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    out = gemm_nt(a, b, bias=bias, residual=res, silu=True)
    assert_close_bf16(out, ref_linear(a, b, bias, res, silu=True), K)


def test_gemm_strided_views():
    from aliyun_gpushare_device_plugin_amd.ops import gemm_nt
    big = torch.randn(512, 1024, device="cuda", dtype=torch.bfloat16)
    a = big[:, 256:768]            # lda = 1024, K = 512
    b = torch.randn(256, 512, device="cuda", dtype=torch.bfloat16)
    assert_close_bf16(gemm_nt(a, b), ref_linear(a, b), 512)


def test_gemm_rejects_bad_shapes():
    from aliyun_gpushare_device_plugin_amd.ops import gemm_nt
    a = torch.randn(64, 100, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(ValueError):
        gemm_nt(a, torch.randn(64, 100, device="cuda", dtype=torch.bfloat16))


def test_linear_autograd_backward():
    from aliyun_gpushare_device_plugin_amd.ops import linear_autograd
    x = torch.randn(4, 50, 256, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    w = (torch.randn(512, 256, device="cuda", dtype=torch.bfloat16) * 0.05).requires_grad_()
    y = linear_autograd(x, w)
    gy = torch.randn_like(y)
    y.backward(gy)
    xr, wr = x.detach().float().requires_grad_(), w.detach().float().requires_grad_()
    (xr @ wr.t()).backward(gy.float())
    assert_close_bf16(x.grad, xr.grad, 512)
    assert_close_bf16(w.grad, wr.grad, 200)


def test_rmsnorm_and_residual():
    from aliyun_gpushare_device_plugin_amd.ops import rmsnorm
    x = torch.randn(37, 4096, device="cuda", dtype=torch.bfloat16)
    r = torch.randn(37, 4096, device="cuda", dtype=torch.bfloat16)
    w = torch.rand(4096, device="cuda", dtype=torch.bfloat16) + 0.5
    y = rmsnorm(x, w, 1e-5)
    xf = x.float()
    ref = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-5) * w.float()
    assert torch.allclose(y.float(), ref, rtol=2e-2, atol=2e-2)
    y2, h = rmsnorm(x, w, 1e-5, residual=r)
    hf = (x.float() + r.float()).to(torch.bfloat16).float()
    assert torch.equal(h, (x.float() + r.float()).to(torch.bfloat16))
    ref2 = hf * torch.rsqrt(hf.pow(2).mean(-1, keepdim=True) + 1e-5) * w.float()
    assert torch.allclose(y2.float(), ref2, rtol=2e-2, atol=2e-2)


def test_silu_mul():
    from aliyun_gpushare_device_plugin_amd.ops import silu_mul
    gu = torch.randn(33, 2 * 1408, device="cuda", dtype=torch.bfloat16)
    y = silu_mul(gu)
    ref = torch.nn.functional.silu(gu[:, :1408].float()) * gu[:, 1408:].float()
    assert torch.allclose(y.float(), ref, rtol=2e-2, atol=2e-2)


def test_rope_matches_reference():
    from aliyun_gpushare_device_plugin_amd.ops import rope_, rope_tables
    T, H, D = 96, 8, 128
    cos, sin = rope_tables(T, D)
    qkv = torch.randn(T, (H + 2) * D, device="cuda", dtype=torch.bfloat16)
    q = qkv[:, : H * D]
    ref = q.float().reshape(T, H, D)
    c, s = cos[:, None, :].float(), sin[:, None, :].float()
    x1, x2 = ref[..., : D // 2], ref[..., D // 2:]
    want = torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], -1)
    untouched = qkv[:, H * D:].clone()
    rope_(q, cos, sin, H, D, T)
    assert torch.allclose(q.float().reshape(T, H, D), want, rtol=2e-2, atol=2e-2)
    assert torch.equal(qkv[:, H * D:], untouched)
