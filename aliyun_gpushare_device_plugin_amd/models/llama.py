"""Llama-3-8B-shaped decoder (random init, bf16) — the co-location demo workload (BASELINE
config 4: two such pods on one MI355X under the HIP quota shim).

Architecture = Llama-3-8B: 32 layers, d_model 4096, 32 query / 8 KV heads of 128, SwiGLU MLP
14336, RMSNorm eps 1e-5, RoPE theta 500000, vocab 128256 (weights random: no checkpoints
offline). Compute path per layer, all on hand-written gfx950 kernels except attention:
  rmsnorm(+residual, fused)  ->  QKV GEMM (one fused [6144, 4096] weight)
  ->  RoPE in place on the q/k slices of the QKV buffer (no copies)
  ->  causal GQA attention (ops.attention: flash-style HIP kernel when built, else SDPA)
  ->  O-proj GEMM with the residual add fused into its epilogue
  ->  rmsnorm  ->  gate|up GEMM (one [28672, 4096] weight, gate/up rows interleaved by 16) with
      SiLU(gate)*up computed in its epilogue (no [T, 28672] activation round trip)
  ->  down GEMM with the residual add fused
"""
from __future__ import annotations

import dataclasses
import math

import torch

from .. import ops


@dataclasses.dataclass
class LlamaConfig:
    vocab: int = 128256
    d_model: int = 4096
    n_layers: int = 32
    n_heads: int = 32
    n_kv_heads: int = 8
    head_dim: int = 128
    d_ff: int = 14336
    eps: float = 1e-5
    rope_theta: float = 500000.0
    max_seq: int = 8192

    @classmethod
    def llama3_8b(cls, **kw):
        return cls(**kw)

    @classmethod
    def tiny(cls, **kw):
        base = dict(vocab=1024, d_model=256, n_layers=2, n_heads=4, n_kv_heads=2, head_dim=64, d_ff=512,
                    max_seq=512)
        base.update(kw)
        return cls(**base)

    def n_params(self) -> int:
        qkv = self.d_model * (self.n_heads + 2 * self.n_kv_heads) * self.head_dim
        o = self.n_heads * self.head_dim * self.d_model
        mlp = 3 * self.d_model * self.d_ff
        return self.n_layers * (qkv + o + mlp + 2 * self.d_model) + 2 * self.vocab * self.d_model + self.d_model


class LlamaModel:
    """Inference-only model (weights are plain tensors; no nn.Module overhead in the hot loop)."""

    def __init__(self, cfg: LlamaConfig, device="cuda", seed: int = 0):
        self.cfg = c = cfg
        self.device = torch.device(device)
        g = torch.Generator(device=self.device).manual_seed(seed)

        def w(*shape, std=0.02):
            return (torch.randn(*shape, device=self.device, dtype=torch.bfloat16, generator=g) * std)

        self.embed = w(c.vocab, c.d_model)
        self.layers = []
        nq = (c.n_heads + 2 * c.n_kv_heads) * c.head_dim
        for _ in range(c.n_layers):
            self.layers.append({
                "attn_norm": torch.ones(c.d_model, device=self.device, dtype=torch.bfloat16),
                "wqkv": w(nq, c.d_model),
                "wo": w(c.d_model, c.n_heads * c.head_dim, std=0.02 / math.sqrt(2 * c.n_layers)),
                "mlp_norm": torch.ones(c.d_model, device=self.device, dtype=torch.bfloat16),
                "wgu": ops.interleave_gate_up(w(2 * c.d_ff, c.d_model)),   # epilogue-SwiGLU layout
                "wd": w(c.d_model, c.d_ff, std=0.02 / math.sqrt(2 * c.n_layers)),
            })
        self.final_norm = torch.ones(c.d_model, device=self.device, dtype=torch.bfloat16)
        self.lm_head = w(c.vocab, c.d_model)
        self.cos, self.sin = ops.rope_tables(c.max_seq, c.head_dim, c.rope_theta, self.device)

    def weight_bytes(self) -> int:
        n = self.embed.numel() + self.lm_head.numel() + self.final_norm.numel()
        for L in self.layers:
            n += sum(t.numel() for t in L.values())
        return 2 * n

    @torch.no_grad()
    def forward(self, tokens: torch.Tensor, logits: str = "last", kv_sink=None) -> torch.Tensor:
        """Prefill forward. ``tokens`` [B, S] int64. Returns logits [B, vocab] for the last
        position (``logits="last"``) or [B, S, vocab] (``"all"``). ``kv_sink(layer, k, v)`` receives
        each layer's post-RoPE K and V as [B, S, Hkv, D] views (the serving path fills its KV
        cache from them)."""
        c = self.cfg
        B, S = tokens.shape
        if S > c.max_seq:
            raise ValueError("sequence longer than max_seq")
        T = B * S
        h = self.embed[tokens.reshape(-1)]                      # residual stream [T, d]
        x = None
        hq, hk = c.n_heads * c.head_dim, c.n_kv_heads * c.head_dim
        for i, L in enumerate(self.layers):
            if i == 0:
                x = ops.rmsnorm(h, L["attn_norm"], c.eps)
            qkv = ops.linear(x, L["wqkv"])                       # [T, hq + 2 hk]
            q, k, v = qkv[:, :hq], qkv[:, hq:hq + hk], qkv[:, hq + hk:]
            ops.rope_(q, self.cos, self.sin, c.n_heads, c.head_dim, S)
            ops.rope_(k, self.cos, self.sin, c.n_kv_heads, c.head_dim, S)
            if kv_sink is not None:
                kv_sink(i, k.view(B, S, c.n_kv_heads, c.head_dim), v.view(B, S, c.n_kv_heads, c.head_dim))
            a = ops.attention(q.view(B, S, c.n_heads, c.head_dim), k.view(B, S, c.n_kv_heads, c.head_dim),
                              v.view(B, S, c.n_kv_heads, c.head_dim), causal=True)
            h = ops.linear(a.reshape(T, hq), L["wo"], residual=h)   # fused residual add
            x = ops.rmsnorm(h, L["mlp_norm"], c.eps)
            h = ops.linear(ops.linear_swiglu(x, L["wgu"]), L["wd"], residual=h)
            nxt = self.layers[i + 1]["attn_norm"] if i + 1 < len(self.layers) else self.final_norm
            x = ops.rmsnorm(h, nxt, c.eps)
        if logits == "last":
            last = x.view(B, S, c.d_model)[:, -1].contiguous()
            return ops.linear(last, self.lm_head)
        return ops.linear(x, self.lm_head).view(B, S, c.vocab)

    def flops_per_token(self, S: int) -> float:
        c = self.cfg
        dense = 2 * (self.cfg.n_params() - 2 * c.vocab * c.d_model)
        attn = 2 * 2 * c.n_layers * c.n_heads * c.head_dim * S / 2     # causal QK^T + PV
        return dense + attn


def reference_forward(model: LlamaModel, tokens: torch.Tensor) -> torch.Tensor:
    """Plain-PyTorch fp32 reference of the same network (numerics tests)."""
    c = model.cfg
    B, S = tokens.shape
    f = torch.float32

    def rms(x, w):
        return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + c.eps) * w.to(f)

    h = model.embed[tokens].to(f)
    pos = torch.arange(S, device=tokens.device)
    cos, sin = model.cos[pos].to(f), model.sin[pos].to(f)

    def rope(t):   # [B, S, H, D]
        d = t.shape[-1] // 2
        x1, x2 = t[..., :d], t[..., d:]
        cc, ss = cos[None, :, None, :], sin[None, :, None, :]
        return torch.cat([x1 * cc - x2 * ss, x2 * cc + x1 * ss], -1)

    hq, hk = c.n_heads * c.head_dim, c.n_kv_heads * c.head_dim
    for L in model.layers:
        x = rms(h, L["attn_norm"])
        qkv = x @ L["wqkv"].to(f).t()
        q = rope(qkv[..., :hq].reshape(B, S, c.n_heads, c.head_dim))
        k = rope(qkv[..., hq:hq + hk].reshape(B, S, c.n_kv_heads, c.head_dim))
        v = qkv[..., hq + hk:].reshape(B, S, c.n_kv_heads, c.head_dim)
        rep = c.n_heads // c.n_kv_heads
        k, v = k.repeat_interleave(rep, 2), v.repeat_interleave(rep, 2)
        a = torch.nn.functional.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2),
                                                             v.transpose(1, 2), is_causal=True)
        h = h + a.transpose(1, 2).reshape(B, S, hq) @ L["wo"].to(f).t()
        x = rms(h, L["mlp_norm"])
        gu = x @ ops.deinterleave_gate_up(L["wgu"]).to(f).t()
        g_, u_ = gu[..., :c.d_ff], gu[..., c.d_ff:]
        h = h + (torch.nn.functional.silu(g_) * u_) @ L["wd"].to(f).t()
    x = rms(h, model.final_norm)
    return x[:, -1] @ model.lm_head.to(f).t()
