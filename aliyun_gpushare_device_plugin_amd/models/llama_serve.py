"""Serving pod workload: Llama-3-8B prefill into a KV cache, then greedy decode, one hipGraph per step.

A GPU-sharing node mostly hosts inference servers, and their decode loop is the workload that
suffers most from a noisy neighbour: every step is ~35 small launches per layer's worth of
memory-bound work. The decode step here is built for that:

* KV cache ``[B, Hkv, Smax, 128]`` per layer (``ops.kv_cache``), filled by the prefill through
  ``LlamaModel.forward(kv_sink=...)`` and appended to by ``ops.kv_append``;
* attention = ``ops.decode_attention`` (split-K over the cache, ``native/kernels/decode_attention.hip``);
  the projections (M = batch <= 64) on the LDS-staged skinny MFMA GEMM (``ops.skinny_linear``,
  residual add fused in place), with the rest folded into it: RMSNorm into the next projection's
  X staging, SwiGLU into the gate/up epilogue, RoPE(q, k) + KV append into the QKV projection's
  split reduction. 5.08 ms per batch-32 step against 5.75 ms with hipBLASLt projections
  (``profiles/decode/README.md``); ``gemm="hipblaslt"`` runs them on ``torch.matmul`` /
  ``torch.addmm`` for A/B measurement;
* positions / lengths live in device tensors, so the whole 32-layer step is captured once in a
  hipGraph (``torch.cuda.CUDAGraph``) and replayed: one launch per step instead of ~450.
"""
from __future__ import annotations

import torch

from .. import ops
from .llama import LlamaModel


class LlamaServer:
    def __init__(self, model: LlamaModel, batch: int, max_ctx: int, gemm: str = "skinny",
                 priority: str = "normal"):
        c = self.cfg = model.cfg
        # "high": decode steps (eager or graph replay) go to a high-priority stream, so the
        # hardware queue scheduler dispatches their workgroups ahead of a co-located pod's
        # normal-priority work as CUs free up (a decode step is hundreds of small kernels, each
        # of which otherwise waits behind the neighbour's in-flight GEMM)
        if priority not in ("normal", "high"):
            raise ValueError("priority must be 'normal' or 'high'")
        self.stream = (torch.cuda.Stream(model.device, priority=torch.cuda.Stream.priority_range()[1])
                       if priority == "high" and str(model.device).startswith("cuda") else None)
        if gemm not in ("skinny", "hipblaslt") or (gemm == "skinny" and batch > 64):
            raise ValueError("gemm must be 'skinny' (batch <= 64) or 'hipblaslt'")
        self.gemm = gemm
        self.fuse_norm = False
        # RMSNorm folded across the projections (skinny path): the o / down projections' split
        # reduction emits row sums of squares and the next projection normalises while staging
        # its input, so no norm kernel runs between them
        self.fold_norm = (gemm == "skinny" and ops.skinny_ssq_ok(c.d_model, c.n_heads * c.head_dim)
                          and ops.skinny_ssq_ok(c.d_model, c.d_ff))
        self.ssq = (torch.zeros((c.d_model // 1024, batch), dtype=torch.float32, device=model.device)
                    if self.fold_norm else None)
        # RoPE(q, k) + KV append in the QKV projection's split reduction (no rope_kv_append launch)
        self.fuse_rope = gemm == "skinny" and ops.skinny_rope_ok((c.n_heads + 2 * c.n_kv_heads) * c.head_dim,
                                                                 c.d_model) and c.head_dim == 128
        if max_ctx > c.max_seq:
            raise ValueError("max_ctx exceeds the RoPE table (cfg.max_seq)")
        self.model, self.B = model, batch
        dev = model.device
        self.kc, self.vc = [], []
        for _ in range(c.n_layers):
            k, v = ops.kv_cache(batch, c.n_kv_heads, max_ctx, c.head_dim, dev)
            self.kc.append(k)
            self.vc.append(v)
        self.smax = self.kc[0].shape[2]
        self.max_ctx = max_ctx
        self.ws = ops.DecodeWorkspace(batch, c.n_heads, self.smax, c.head_dim, dev)
        self.tok = torch.zeros(batch, dtype=torch.long, device=dev)      # next input token per sequence
        self.pos = torch.zeros(batch, dtype=torch.int32, device=dev)     # its position (= cached length)
        self.lens = torch.zeros(batch, dtype=torch.int32, device=dev)    # cached length incl. the new token
        self.host_len = 0                                                # same, tracked on the host
        self.graph = None
        self.logits = None

    def kv_bytes(self) -> int:
        return 2 * sum(t.numel() for t in self.kc)

    @torch.no_grad()
    def prefill(self, tokens: torch.Tensor) -> torch.Tensor:
        """Run the prompt ``tokens`` [B, S] through the model, fill the caches, return the last
        logits and set up the first decode input (greedy)."""
        B, S = tokens.shape
        if B != self.B or S >= self.max_ctx:
            raise ValueError("prompt does not fit the server's batch / context")

        def sink(i, k, v):
            self.kc[i][:, :, :S].copy_(k.transpose(1, 2))
            self.vc[i][:, :, :S].copy_(v.transpose(1, 2))

        logits = self.model.forward(tokens, kv_sink=sink)
        self.tok.copy_(logits.argmax(-1))
        self.pos.fill_(S)
        self.host_len = S
        return logits

    def _mm(self, x, w, residual=None):
        if self.gemm == "skinny":
            return ops.skinny_linear(x, w, residual=residual, out=residual)
        return torch.matmul(x, w.t()) if residual is None else torch.addmm(residual, x, w.t())

    def _mm_in(self, x, w, rope=None):
        """Projection of a layer input that may be a deferred norm ``(h, norm_w)``; ``rope`` (skinny
        path) = ``ops.skinny_linear``'s RoPE + KV-append epilogue."""
        if isinstance(x, tuple):
            h, nw = x
            return ops.skinny_linear(h, w, norm=(self.ssq, nw, self.cfg.eps), rope=rope)
        if rope is not None:
            return ops.skinny_linear(x, w, rope=rope)
        return self._mm(x, w)

    def _mm_norm(self, x, w, residual, norm_w):
        """``h = residual + x @ w.T`` (in place) and ``rmsnorm(h) * norm_w``. ``fuse_norm`` folds the
        norm into the skinny GEMM's split reduction; measured on MI355X it saves nothing at batch
        32 (5.62 vs 5.57 ms per step: the fused pass runs one workgroup per row), so it is off."""
        if self.fold_norm:
            h = ops.skinny_linear(x, w, residual=residual, out=residual, ssq_out=self.ssq)
            return h, (h, norm_w)                      # the norm is applied by the consumer
        if self.gemm == "skinny" and self.fuse_norm:
            return ops.skinny_linear(x, w, residual=residual, out=residual, norm_weight=norm_w, eps=self.cfg.eps)
        h = self._mm(x, w, residual)
        return h, ops.rmsnorm(h, norm_w, self.cfg.eps)

    @torch.no_grad()
    def _step(self) -> torch.Tensor:
        c, m = self.cfg, self.model
        hq = c.n_heads * c.head_dim
        torch.add(self.pos, 1, out=self.lens)
        h = m.embed.index_select(0, self.tok)                          # residual stream [B, d]
        x = ops.rmsnorm(h, m.layers[0]["attn_norm"], c.eps)
        for i, L in enumerate(m.layers):
            rope = (m.cos, m.sin, self.pos, self.kc[i], self.vc[i], c.n_heads) if self.fuse_rope else None
            qkv = self._mm_in(x, L["wqkv"], rope=rope)
            if rope is None:
                ops.rope_kv_append(qkv, m.cos, m.sin, self.pos, self.kc[i], self.vc[i], c.n_heads)
            a = ops.decode_attention(qkv[:, :hq], self.kc[i], self.vc[i], self.lens, self.ws)
            h, x = self._mm_norm(a, L["wo"], h, L["mlp_norm"])
            act = None
            if self.gemm == "skinny":                                   # SwiGLU in the epilogue
                act = (ops.skinny_swiglu(x[0], L["wgu"], norm=(self.ssq, x[1], c.eps)) if isinstance(x, tuple)
                       else ops.skinny_swiglu(x, L["wgu"]))
            if act is None:
                gu = self._mm_in(x, L["wgu"])                           # gate/up rows interleaved by 16
                act = ops.silu_mul(gu, interleaved=True)
            nxt = m.layers[i + 1]["attn_norm"] if i + 1 < len(m.layers) else m.final_norm
            h, x = self._mm_norm(act, L["wd"], h, nxt)
        logits = self._mm_in(x, m.lm_head)
        ops.argmax_rows(logits, out=self.tok)                          # greedy, one launch
        self.pos.add_(1)
        return logits

    def capture(self) -> None:
        """Capture one decode step in a hipGraph (after a warm-up step on a side stream). The
        warm-up and the capture advance nothing: positions are restored afterwards."""
        save = (self.tok.clone(), self.pos.clone())
        s = torch.cuda.Stream(self.model.device)
        s.wait_stream(torch.cuda.current_stream(self.model.device))
        with torch.cuda.stream(s):
            self._step()
        torch.cuda.current_stream(self.model.device).wait_stream(s)
        self.tok.copy_(save[0])
        self.pos.copy_(save[1])
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=self.stream):
            self.logits = self._step()
        self.tok.copy_(save[0])
        self.pos.copy_(save[1])
        self.graph = g

    def rewind(self, length: int) -> None:
        """Continue decoding from position ``length`` (the cache beyond it is overwritten)."""
        if not 0 < length < self.max_ctx:
            raise ValueError("rewind length outside the cache")
        self.pos.fill_(length)
        self.host_len = length

    def step(self, use_graph: bool = True) -> torch.Tensor:
        """One greedy decode step for every sequence; returns the step's logits [B, vocab]."""
        if self.host_len + 1 > self.max_ctx:
            raise RuntimeError("context full")
        self.host_len += 1
        if self.stream is not None and torch.cuda.current_stream(self.model.device) != self.stream:
            # (a caller that made self.stream its current stream pays no hand-off per step)
            cur = torch.cuda.current_stream(self.model.device)
            self.stream.wait_stream(cur)
            with torch.cuda.stream(self.stream):
                out = self._replay_or_step(use_graph)
            cur.wait_stream(self.stream)
            return out
        return self._replay_or_step(use_graph)

    def _replay_or_step(self, use_graph: bool) -> torch.Tensor:
        if use_graph:
            if self.graph is None:
                self.capture()
            self.graph.replay()
            return self.logits
        return self._step()
