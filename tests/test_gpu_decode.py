"""Serving path on MI355X: decode attention over a KV cache, KV append, and the hipGraph-captured
Llama decode step, each against a plain PyTorch fp32 reference."""
import pytest
import torch

from aliyun_gpushare_device_plugin_amd import ops
from aliyun_gpushare_device_plugin_amd.ops.decode import reference_decode_attention

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("G", [1, 2, 4, 8])
def test_decode_attention_matches_fp32(G):
    """vs fp32; cache rows past each sequence hold NaN (stale or never-written rows must not leak
    into the result)."""
    torch.manual_seed(G)
    B, Hkv, D = 3, 2, 128
    kc, vc = ops.kv_cache(B, Hkv, 1000, D)                 # Smax rounds up to 1024
    assert kc.shape[2] == 1024
    kc.normal_()
    vc.normal_()
    lens = torch.tensor([1, 300, 1000], dtype=torch.int32, device="cuda")
    for b, n in enumerate(lens.tolist()):
        kc[b, :, n:] = float("nan")
        vc[b, :, n:] = float("nan")
    wide = torch.randn(B, G * Hkv * D + 256, device="cuda", dtype=torch.bfloat16)   # q as a strided slice
    q = wide[:, 128:128 + G * Hkv * D]
    out = ops.decode_attention(q, kc, vc, lens)
    ref = reference_decode_attention(q, kc, vc, lens)
    err = (out.float() - ref).abs().max().item()
    assert err < 2e-2, err
    from aliyun_gpushare_device_plugin_amd.ops import _lib
    try:
        for ntl in (0, 1):                          # K/V load policy: same arithmetic, same bits
            _lib.check(_lib.lib().gs_decode_attn_set_nt(ntl), "gs_decode_attn_set_nt")
            assert torch.equal(ops.decode_attention(q, kc, vc, lens), out)
    finally:
        _lib.lib().gs_decode_attn_set_nt(1)


def test_kv_append_writes_exactly_the_new_rows():
    B, Hkv, D = 4, 8, 128
    kc, vc = ops.kv_cache(B, Hkv, 512, D)
    qkv = torch.randn(B, 3 * Hkv * D, device="cuda", dtype=torch.bfloat16)
    k, v = qkv[:, :Hkv * D], qkv[:, Hkv * D:2 * Hkv * D]
    pos = torch.tensor([0, 7, 511, 600], dtype=torch.int32, device="cuda")   # 600: outside, skipped
    ops.kv_append(k, v, kc, vc, pos)
    torch.cuda.synchronize()
    for b, p in enumerate(pos.tolist()):
        if p < 512:
            assert torch.equal(kc[b, :, p], k[b].view(Hkv, D)) and torch.equal(vc[b, :, p], v[b].view(Hkv, D))
    assert int((kc != 0).sum()) == 3 * Hkv * D and int((vc != 0).sum()) == 3 * Hkv * D


def _small_model():
    from aliyun_gpushare_device_plugin_amd.models.llama import LlamaConfig, LlamaModel

    cfg = LlamaConfig.tiny(d_model=512, n_heads=4, n_kv_heads=1, head_dim=128, d_ff=1024, vocab=1024, max_seq=1024)
    return LlamaModel(cfg, "cuda", seed=3)


def test_decode_steps_match_full_recompute_and_graph_matches_eager():
    from aliyun_gpushare_device_plugin_amd.models.llama import reference_forward
    from aliyun_gpushare_device_plugin_amd.models.llama_serve import LlamaServer

    model = _small_model()
    torch.manual_seed(0)
    prompt = torch.randint(0, model.cfg.vocab, (2, 40), device="cuda")
    eager, graph = LlamaServer(model, 2, 256), LlamaServer(model, 2, 256)
    eager.prefill(prompt)
    graph.prefill(prompt)
    seq = prompt
    for _ in range(3):
        nxt = eager.tok.clone()
        le = eager.step(use_graph=False).float()
        lg = graph.step(use_graph=True).float()
        seq = torch.cat([seq, nxt[:, None]], 1)
        ref = reference_forward(model, seq)
        scale = ref.abs().max().item()
        assert (le - ref).abs().max().item() < 0.05 * scale
        assert (lg - le).abs().max().item() < 1e-2 * scale
        assert torch.equal(graph.tok, eager.tok)
    assert graph.host_len == 43 and int(graph.pos[0]) == 43


@pytest.mark.parametrize("use_graph", [False, True])
def test_high_priority_stream_steps_match_the_normal_ones(use_graph):
    """Decode steps on a high-priority stream (``priority="high"``, eager or graph replay) give
    the same tokens and logits as on the current stream, and the caller's stream sees them."""
    from aliyun_gpushare_device_plugin_amd.models.llama_serve import LlamaServer

    model = _small_model()
    torch.manual_seed(1)
    prompt = torch.randint(0, model.cfg.vocab, (4, 33), device="cuda")
    hi, lo = LlamaServer(model, 4, 128, priority="high"), LlamaServer(model, 4, 128)
    assert hi.stream is not None and hi.stream.priority == torch.cuda.Stream.priority_range()[1]
    assert lo.stream is None
    hi.prefill(prompt)
    lo.prefill(prompt)
    for _ in range(4):
        a = hi.step(use_graph=use_graph).float().clone()      # read on the caller's stream, no sync
        b = lo.step(use_graph=use_graph).float()
        assert (a - b).abs().max().item() <= 1e-2 * b.abs().max().item()
        assert torch.equal(hi.tok, lo.tok)
    with torch.cuda.stream(hi.stream):                 # the caller on the server's own stream
        a = hi.step(use_graph=use_graph).float().clone()
    b = lo.step(use_graph=use_graph).float()
    torch.cuda.synchronize()
    assert (a - b).abs().max().item() <= 1e-2 * b.abs().max().item()
    with pytest.raises(ValueError):
        LlamaServer(model, 4, 128, priority="urgent")


_SKINNY_SHAPES = [(1, 256, 512), (7, 512, 4096), (16, 1024, 1024), (32, 4096, 4096),
                  (33, 6144, 4096), (64, 256, 14336), (32, 4096, 14336), (5, 192, 96)]


# variants 2/3 (LDS-staged kernel) exist only for K % 256 == 0; other shapes run variant 1 alone
@pytest.mark.parametrize("M,N,K,variant", [(*s, v) for s in _SKINNY_SHAPES for v in (1, 2, 3)
                                           if v == 1 or s[2] % 256 == 0])
def test_skinny_linear_matches_fp32(M, N, K, variant):
    from aliyun_gpushare_device_plugin_amd.ops import _lib
    from aliyun_gpushare_device_plugin_amd.ops.gemm import SKINNY_AUTO, set_skinny_variant

    set_skinny_variant(min(variant, 2))
    _lib.lib().gs_skinny_set_lds_waves(2 if variant == 3 else 0)     # 3 = LDS kernel with 2-wave workgroups
    try:
        _check_skinny(M, N, K)
    finally:
        set_skinny_variant(SKINNY_AUTO)
        _lib.lib().gs_skinny_set_lds_waves(0)


def _check_skinny(M, N, K):
    torch.manual_seed(M * 7 + N)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
    ref = x.float() @ w.float().t()
    y = ops.skinny_linear(x, w)
    assert (y.float() - ref).abs().max().item() < 2e-2 * ref.abs().max().item() + 1e-2
    r = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    want = ref + r.float()
    y2 = ops.skinny_linear(x, w, residual=r, out=r)            # in-place residual add
    assert y2.data_ptr() == r.data_ptr()
    assert (r.float() - want).abs().max().item() < 2e-2 * want.abs().max().item() + 1e-2


@pytest.mark.parametrize("M,Hq,Hkv,K", [(32, 32, 8, 4096), (5, 8, 2, 1024), (64, 16, 4, 2048)])
def test_skinny_rope_epilogue_matches_separate_launch(M, Hq, Hkv, K):
    """QKV projection whose split reduction applies RoPE and appends k / v: bit-identical to the
    plain projection followed by ops.rope_kv_append, including rows whose position is outside the
    cache (rotated, not appended)."""
    torch.manual_seed(M + Hq)
    N, Smax, rows = (Hq + 2 * Hkv) * 128, 256, 300
    assert ops.skinny_rope_ok(N, K)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
    cos, sin = ops.rope_tables(rows, 128, 500000.0, "cuda")
    pos = torch.randint(0, Smax, (M,), device="cuda", dtype=torch.int32)
    pos[0] = Smax                                   # outside the cache: rotated, not appended
    if M > 1:
        pos[1] = -1
    kc1, vc1 = ops.kv_cache(M, Hkv, Smax, 128, "cuda")
    kc1.normal_()
    vc1.normal_()
    kc2, vc2 = kc1.clone(), vc1.clone()
    y1 = ops.skinny_linear(x, w, rope=(cos, sin, pos, kc1, vc1, Hq))
    y2 = ops.skinny_linear(x, w)
    ops.rope_kv_append(y2, cos, sin, pos, kc2, vc2, Hq)
    assert torch.equal(y1, y2)
    assert torch.equal(kc1, kc2) and torch.equal(vc1, vc2)
    with pytest.raises(ValueError):
        ops.skinny_linear(x, w, residual=y2.clone(), rope=(cos, sin, pos, kc1, vc1, Hq))


def test_skinny_linear_on_strided_rows():
    x_wide = torch.randn(8, 1024 + 64, device="cuda", dtype=torch.bfloat16)
    x = x_wide[:, 64:]                                          # 16-B aligned slice, row stride 1088
    w = torch.randn(512, 1024, device="cuda", dtype=torch.bfloat16) * 0.05
    ref = x.float() @ w.float().t()
    assert (ops.skinny_linear(x, w).float() - ref).abs().max().item() < 2e-2 * ref.abs().max().item()


def test_decode_step_hipblaslt_and_skinny_agree():
    from aliyun_gpushare_device_plugin_amd.models.llama_serve import LlamaServer

    model = _small_model()
    prompt = torch.randint(0, model.cfg.vocab, (4, 24), device="cuda")
    a, b = LlamaServer(model, 4, 128, gemm="skinny"), LlamaServer(model, 4, 128, gemm="hipblaslt")
    a.prefill(prompt)
    b.prefill(prompt)
    la, lb = a.step().float(), b.step().float()
    assert (la - lb).abs().max().item() < 2e-2 * lb.abs().max().item()


def test_fused_rope_kv_append_equals_the_three_ops():
    from aliyun_gpushare_device_plugin_amd.ops import rope_, rope_tables

    B, Hq, Hkv, D = 3, 8, 2, 128
    cos, sin = rope_tables(512, D, 500000.0, "cuda")
    qkv = torch.randn(B, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
    pos = torch.tensor([0, 17, 300], dtype=torch.int32, device="cuda")
    ka, va = ops.kv_cache(B, Hkv, 512, D)
    kb, vb = ops.kv_cache(B, Hkv, 512, D)
    ref = qkv.clone()
    q, k, v = ref[:, :Hq * D], ref[:, Hq * D:(Hq + Hkv) * D], ref[:, (Hq + Hkv) * D:]
    rope_(q, cos, sin, Hq, D, 512, positions=pos)
    rope_(k, cos, sin, Hkv, D, 512, positions=pos)
    ops.kv_append(k, v, ka, va, pos)
    ops.rope_kv_append(qkv, cos, sin, pos, kb, vb, Hq)
    torch.cuda.synchronize()
    assert torch.equal(qkv[:, :(Hq + Hkv) * D], ref[:, :(Hq + Hkv) * D])
    assert torch.equal(ka, kb) and torch.equal(va, vb)


def test_silu_mul_interleaved_layout():
    gu = torch.randn(5, 2 * 1024, device="cuda", dtype=torch.bfloat16)
    deint = gu.view(5, -1, 2, 16).transpose(1, 2).reshape(5, -1).contiguous()
    assert torch.equal(ops.silu_mul(gu, interleaved=True), ops.silu_mul(deint))


@pytest.mark.parametrize("K", [4096, 14336, 512])
def test_skinny_linear_fused_rmsnorm(K):
    torch.manual_seed(K)
    M, N = 32, 4096
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
    r = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    g = torch.rand(N, device="cuda", dtype=torch.bfloat16) + 0.5
    want_h = ops.skinny_linear(x, w, residual=r.clone())
    want_x = ops.rmsnorm(want_h, g, 1e-5)
    h, xn = ops.skinny_linear(x, w, residual=r, out=r, norm_weight=g, eps=1e-5)
    assert h.data_ptr() == r.data_ptr()
    assert (h.float() - want_h.float()).abs().max().item() <= 1e-2 * want_h.float().abs().max().item()
    assert (xn.float() - want_x.float()).abs().max().item() < 3e-2


@pytest.mark.parametrize("M", [1, 17, 32, 64])
def test_skinny_swiglu_matches_fp32(M):
    """SwiGLU fused into the skinny GEMM's epilogue (interleaved gate/up weights) vs fp32."""
    from aliyun_gpushare_device_plugin_amd.ops.gemm import interleave_gate_up
    torch.manual_seed(M)
    F, K = 8192, 1024
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    g = torch.randn(F, K, device="cuda", dtype=torch.bfloat16) * 0.05
    u = torch.randn(F, K, device="cuda", dtype=torch.bfloat16) * 0.05
    y = ops.skinny_swiglu(x, interleave_gate_up(torch.cat((g, u), 0)))
    assert y is not None and y.shape == (M, F)
    ref = torch.nn.functional.silu(x.float() @ g.float().t()) * (x.float() @ u.float().t())
    err = (y.float() - ref).abs().max().item()
    assert err < 2e-2 * ref.abs().max().item() + 1e-3, err
    assert ops.skinny_swiglu(x, interleave_gate_up(torch.cat((g[:512], u[:512]), 0))) is None   # split-K shape


def test_decode_step_with_folded_rmsnorm_matches_unfolded():
    """1024-wide model: the o / down projections emit row sums of squares and the next projection
    normalises while staging its input (no RMSNorm kernels), and the QKV reduction applies RoPE and
    appends to the caches; logits match the unfused skinny step and the hipBLASLt step, through a
    hipGraph replay too."""
    from aliyun_gpushare_device_plugin_amd.models.llama import LlamaConfig, LlamaModel
    from aliyun_gpushare_device_plugin_amd.models.llama_serve import LlamaServer

    cfg = LlamaConfig.tiny(d_model=1024, n_heads=8, n_kv_heads=2, head_dim=128, d_ff=2048, vocab=2048)
    model = LlamaModel(cfg, "cuda", seed=3)
    prompt = torch.randint(0, cfg.vocab, (8, 40), device="cuda")
    a = LlamaServer(model, 8, 128, gemm="skinny")
    assert a.fold_norm and a.fuse_rope
    b = LlamaServer(model, 8, 128, gemm="skinny")
    b.fold_norm = b.fuse_rope = False
    c = LlamaServer(model, 8, 128, gemm="hipblaslt")
    for s in (a, b, c):
        s.prefill(prompt)
    la, lb, lc = a.step(use_graph=False).float(), b.step(use_graph=False).float(), c.step(use_graph=False).float()
    scale = lc.abs().max().item()
    assert (la - lb).abs().max().item() < 2e-2 * scale
    assert (la - lc).abs().max().item() < 3e-2 * scale
    if torch.equal(a.tok, b.tok):              # same greedy tokens: the next steps are comparable
        a.capture()
        b.capture()
        ga, gb = a.step().float(), b.step().float()
        assert (ga - gb).abs().max().item() < 2e-2 * scale



@pytest.fixture
def skinny_prefetch():
    """Set the 4-wave LDS kernel's schedule (0 auto, 1 / 2 k-slices in flight, 3 wave-level K split,
    4 non-temporal W) for one test; restore the previous one."""
    from aliyun_gpushare_device_plugin_amd.ops import _lib

    lib = _lib.lib()
    before = lib.gs_skinny_get_prefetch()
    yield lambda pf: _lib.check(lib.gs_skinny_set_prefetch(pf), "gs_skinny_set_prefetch")
    lib.gs_skinny_set_prefetch(before)


@pytest.mark.parametrize("M,N,K", [(32, 4096, 4096), (33, 6144, 4096), (64, 256, 14336), (7, 512, 4096),
                                   (32, 16384, 1024), (1, 4096, 14336)])
def test_skinny_prefetch_depths_agree_bitwise(M, N, K, skinny_prefetch):
    """Two k-slices in flight (register ring, zero-size descriptors past the K range) change only
    when bytes arrive, not the arithmetic: outputs equal the one-slice kernel bit for bit, and both
    match fp32."""
    torch.manual_seed(M + N + K)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
    r = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    outs = []
    for pf in (1, 2, 3, 4, 0):
        skinny_prefetch(pf)
        outs.append((ops.skinny_linear(x, w), ops.skinny_linear(x, w, residual=r.clone())))
    for o in (outs[1], outs[3], outs[4]):      # 2 / 4 / auto: same arithmetic, other loads
        assert torch.equal(outs[0][0], o[0]) and torch.equal(outs[0][1], o[1])
    ref = x.float() @ w.float().t()
    for y, yr in (outs[1], outs[2]):           # 3 = wave-level K split: same sums, another order
        assert (y.float() - ref).abs().max().item() < 2e-2 * ref.abs().max().item() + 1e-2
        assert (yr.float() - ref - r.float()).abs().max().item() < 2e-2 * ref.abs().max().item() + 2e-2


@pytest.mark.parametrize("M", [1, 32, 64])
def test_skinny_swiglu_prefetch_depths_agree_bitwise(M, skinny_prefetch):
    from aliyun_gpushare_device_plugin_amd.ops.gemm import interleave_gate_up
    torch.manual_seed(100 + M)
    F, K = 8192, 2048
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = interleave_gate_up(torch.randn(2 * F, K, device="cuda", dtype=torch.bfloat16) * 0.05)
    ys = []
    for pf in (1, 2, 3, 4, 0):
        skinny_prefetch(pf)
        ys.append(ops.skinny_swiglu(x, w))
    assert ys[0] is not None and all(torch.equal(ys[0], ys[i]) for i in (1, 3, 4))
    scale = ys[0].float().abs().max().item()
    assert (ys[2].float() - ys[0].float()).abs().max().item() < 1e-2 * scale + 1e-3


def test_decode_step_prefetch_depths_agree_bitwise(skinny_prefetch):
    """Folded RMSNorm staging (norm weight through its own descriptor), the RoPE/KV-append
    reduction and the residual projections, one decode step per depth: identical logits."""
    from aliyun_gpushare_device_plugin_amd.models.llama import LlamaConfig, LlamaModel
    from aliyun_gpushare_device_plugin_amd.models.llama_serve import LlamaServer

    cfg = LlamaConfig.tiny(d_model=1024, n_heads=8, n_kv_heads=2, head_dim=128, d_ff=2048, vocab=2048)
    model = LlamaModel(cfg, "cuda", seed=5)
    prompt = torch.randint(0, cfg.vocab, (8, 40), device="cuda")
    logits = []
    for pf in (1, 2, 3, 4, 0):
        skinny_prefetch(pf)
        s = LlamaServer(model, 8, 128, gemm="skinny")
        assert s.fold_norm and s.fuse_rope
        s.prefill(prompt)
        logits.append(s.step(use_graph=False))
    assert all(torch.equal(logits[0], logits[i]) for i in (1, 3, 4))
    scale = logits[0].float().abs().max().item()
    assert (logits[2].float() - logits[0].float()).abs().max().item() < 2e-2 * scale


@pytest.mark.parametrize("K,rope", [(4096, False), (14336, False), (4096, True)])
def test_static_split_reductions_equal_the_loop(K, rope):
    """The split reductions with compile-time split counts (all partial loads issued at once) add
    the splits in the same order as the runtime loop: bit-identical outputs, plain and RoPE/KV."""
    from aliyun_gpushare_device_plugin_amd.ops import _lib

    torch.manual_seed(K)
    M, Hq, Hkv = 32, 32, 8
    N = (Hq + 2 * Hkv) * 128 if rope else 4096
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.03
    assert _lib.lib().gs_skinny_splits(N, K) > 1
    r0 = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    cos, sin = torch.randn(512, 64, device="cuda"), torch.randn(512, 64, device="cuda")
    pos = torch.arange(M, dtype=torch.int32, device="cuda") * 3
    outs = []
    try:
        for st in (0, 1):
            _lib.check(_lib.lib().gs_skinny_set_reduce_static(st), "gs_skinny_set_reduce_static")
            if rope:
                kc, vc = ops.kv_cache(M, Hkv, 256, 128)
                y = ops.skinny_linear(x, w, rope=(cos, sin, pos, kc, vc, Hq))
                outs.append((y, kc, vc))
            else:
                r = r0.clone()
                ssq = torch.zeros(N // 1024, M, device="cuda")
                y = ops.skinny_linear(x, w, residual=r, out=r, ssq_out=ssq)
                outs.append((y, ssq))
    finally:
        _lib.lib().gs_skinny_set_reduce_static(1)
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("B,V", [(32, 128256), (3, 1001), (1, 7), (64, 4096)])
def test_argmax_rows_matches_torch(B, V):
    """Greedy sampling kernel vs torch.argmax: bf16 ties resolved to the first index, strided rows,
    a V that is not a multiple of 8, -inf rows and NaN (counted as the maximum, as torch does)."""
    torch.manual_seed(V)
    ld = -(-V // 8) * 8 + 16                                    # 16-B aligned rows wider than V
    wide = (torch.randn(B, ld, device="cuda") * 4).round().to(torch.bfloat16)   # many exact ties
    x = wide[:, 8:8 + V]
    assert torch.equal(ops.argmax_rows(x), torch.argmax(x, -1))
    y = wide.clone()[:, 8:8 + V]
    y[0] = float("-inf")
    if B > 1:
        y[1, V // 2] = float("nan")
        y[1, V - 1] = float("nan")
    assert torch.equal(ops.argmax_rows(y), torch.argmax(y, -1))


def test_refused_skinny_options_leave_no_armed_state():
    """ADVICE (round 2): when the native side refuses a call's options after RoPE was armed, the
    wrapper must clear them, or the next unrelated skinny_linear on this thread would rotate its
    output and write into the stale cache pointers."""
    from aliyun_gpushare_device_plugin_amd.ops.gemm import _SkinnyOpts

    torch.manual_seed(7)
    M, Hq, Hkv, K, Smax = 8, 8, 2, 1024, 64
    N = (Hq + 2 * Hkv) * 128
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
    cos, sin = ops.rope_tables(128, 128, 500000.0, "cuda")
    pos = torch.arange(M, device="cuda", dtype=torch.int32)
    kc, vc = ops.kv_cache(M, Hkv, Smax, 128, "cuda")
    kc0, vc0 = kc.clone(), vc.clone()
    bad_norm = (torch.empty(0, M, device="cuda"), torch.ones(K, device="cuda", dtype=torch.bfloat16), 1e-5)
    with pytest.raises(Exception):
        with _SkinnyOpts(None, bad_norm, (cos, sin, pos, kc, vc, Hq)):   # nch = 0: refused after RoPE armed
            pass
    y = ops.skinny_linear(x, w)
    assert torch.equal(y, ops.skinny_linear(x, w))
    want = x.float() @ w.float().T
    assert (y.float() - want).abs().max().item() < 2e-2 * want.abs().max().item() + 1e-2
    torch.cuda.synchronize()
    assert torch.equal(kc, kc0) and torch.equal(vc, vc0)
