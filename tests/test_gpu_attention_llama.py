"""Flash-attention kernel and the Llama-3-8B-shaped demo model vs fp32 PyTorch references."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,S,Hq,Hkv,D,causal", [(1, 64, 4, 4, 128, True), (2, 256, 8, 2, 128, True),
                                                  (1, 200, 4, 1, 128, True), (2, 128, 4, 4, 64, False),
                                                  (1, 1000, 32, 8, 128, True), (1, 333, 8, 8, 64, True)])
def test_flash_attention_matches_fp32(B, S, Hq, Hkv, D, causal):
    from aliyun_gpushare_device_plugin_amd.ops import attention, reference_attention
    torch.manual_seed(0)
    q = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
    out = attention(q, k, v, causal=causal)
    ref = reference_attention(q, k, v, causal=causal)
    err = (out.float() - ref).abs().max().item()
    assert err < 3e-2, err


@pytest.mark.parametrize("B,S,Hq,Hkv,causal", [(1, 64, 4, 4, True), (2, 300, 8, 2, True), (1, 1000, 32, 8, True),
                                                (2, 520, 4, 1, False), (1, 2048, 8, 8, True), (3, 17, 2, 2, True),
                                                (1, 4160, 8, 2, True), (3, 700, 6, 3, False),
                                                (2, 1024, 8, 2, False), (1, 2048, 16, 8, False)])
def test_attention_kernels_agree_with_fp32(B, S, Hq, Hkv, causal):
    """D = 128: auto, the 4-wave 16x16 kernel, the 4- and 8-wave 32x32-MFMA kernels and the
    ping-pong variants, vs fp32 (head counts with and without the XCD-grouped block order:
    B*Hq % 8 == 0 or not; S a multiple of the 64-key tile or ragged, so both the masked and the
    unmasked path run on every kernel's last tile)."""
    from aliyun_gpushare_device_plugin_amd.ops import attention, reference_attention
    from aliyun_gpushare_device_plugin_amd.ops.attention import ATTN_AUTO, ATTN_V1, set_attention_variant
    torch.manual_seed(1)
    q = torch.randn(B, S, Hq, 128, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(B, S, Hkv, 128, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(B, S, Hkv, 128, device="cuda", dtype=torch.bfloat16)
    ref = reference_attention(q, k, v, causal=causal)
    try:
        for var in (ATTN_AUTO, ATTN_V1, 2, 3, 7, 8, 9, 11, 12, 13, 14, 20):
            set_attention_variant(var)
            out = attention(q, k, v, causal=causal)
            torch.cuda.synchronize()
            err = (out.float() - ref).abs().max().item()
            assert err < 3e-2, (var, err)
    finally:
        set_attention_variant(ATTN_AUTO)


def test_attention_on_fused_qkv_views():
    from aliyun_gpushare_device_plugin_amd.ops import attention, reference_attention
    B, S, Hq, Hkv, D = 2, 192, 8, 2, 128
    qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
    q = qkv[:, :Hq * D].view(B, S, Hq, D)
    k = qkv[:, Hq * D:(Hq + Hkv) * D].view(B, S, Hkv, D)
    v = qkv[:, (Hq + Hkv) * D:].view(B, S, Hkv, D)
    err = (attention(q, k, v).float() - reference_attention(q, k, v)).abs().max().item()
    assert err < 3e-2, err


def test_attention_peaked_softmax_rescale():
    """Force the online-softmax rescale: a late key dominates every query row."""
    from aliyun_gpushare_device_plugin_amd.ops import attention, reference_attention
    B, S, H, D = 1, 512, 2, 128
    q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16) * 0.1
    k[:, 300] = q[:, 400] * 4          # spike at key 300 for late rows
    v = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
    err = (attention(q, k, v).float() - reference_attention(q, k, v)).abs().max().item()
    assert err < 5e-2, err


def test_llama_tiny_matches_reference():
    from aliyun_gpushare_device_plugin_amd.models.llama import LlamaConfig, LlamaModel, reference_forward
    cfg = LlamaConfig.tiny()
    m = LlamaModel(cfg, "cuda", seed=1)
    tok = torch.randint(0, cfg.vocab, (2, 128), device="cuda")
    out = m.forward(tok).float()
    ref = reference_forward(m, tok)
    rel = (out - ref).norm() / ref.norm()
    assert rel < 3e-2, rel.item()


def test_llama3_8b_shapes_run():
    from aliyun_gpushare_device_plugin_amd.models.llama import LlamaConfig, LlamaModel
    cfg = LlamaConfig.llama3_8b(n_layers=2)
    m = LlamaModel(cfg, "cuda")
    tok = torch.randint(0, cfg.vocab, (1, 512), device="cuda")
    out = m.forward(tok)
    assert out.shape == (1, cfg.vocab) and torch.isfinite(out.float()).all()
    full = LlamaConfig.llama3_8b().n_params()
    assert abs(full - 8.03e9) / 8.03e9 < 0.01   # full config = Llama-3-8B size
