#!/usr/bin/env python3
"""Run a few Llama-3-8B prefill forwards (random weights, batch x seq tokens) for rocprofv3.

python tools/prof_llama.py [--batch 4] [--seq 2048] [--iters 3] [--layers 32]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from aliyun_gpushare_device_plugin_amd.models.llama import LlamaConfig, LlamaModel  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--seq", type=int, default=2048)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--layers", type=int, default=32)
    a = ap.parse_args()
    m = LlamaModel(LlamaConfig.llama3_8b(n_layers=a.layers))
    tok = torch.randint(0, m.cfg.vocab, (a.batch, a.seq), device="cuda")
    m.forward(tok)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        m.forward(tok)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.iters
    print(f"forward {dt * 1e3:.2f} ms, {a.batch * a.seq / dt:.0f} tokens/s", flush=True)


if __name__ == "__main__":
    main()
