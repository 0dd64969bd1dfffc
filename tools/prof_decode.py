#!/usr/bin/env python3
"""Decode-only workload for rocprofv3: Llama-3-8B, batch 32, 1024-token prompt, N graph-replayed
decode steps (run under `rocprofv3 --kernel-trace --stats`; the prefill shows up too)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from aliyun_gpushare_device_plugin_amd.models.llama import LlamaConfig, LlamaModel  # noqa: E402
from aliyun_gpushare_device_plugin_amd.models.llama_serve import LlamaServer  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--batch", type=int, default=32)
ap.add_argument("--gemm", default="skinny")
a = ap.parse_args()
model = LlamaModel(LlamaConfig.llama3_8b(), "cuda", seed=1)
srv = LlamaServer(model, a.batch, 2048, gemm=a.gemm)
srv.prefill(torch.randint(0, model.cfg.vocab, (a.batch, 1024), device="cuda"))
srv.capture()
for _ in range(a.steps):
    srv.step()
torch.cuda.synchronize()
print("done", srv.host_len)
