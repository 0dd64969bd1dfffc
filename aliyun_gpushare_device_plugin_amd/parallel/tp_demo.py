"""RCCL tensor-parallel pair validation (BASELINE config 5, "xGMI-aware TP-pair placement").

Two ranks (one per GPU of a TP pair placed by the topology-aware extender) run a
Megatron-style column/row-parallel MLP block: each rank holds half of the gate|up and down
weights (sharded on d_ff), computes its partial down-projection on the MFMA GEMM kernel and
the pair all-reduces it over RCCL (``torch.distributed`` backend ``nccl`` = RCCL on ROCm).
It reports the all-reduce bus bandwidth, which on a direct xGMI link is ≈ link speed and on
a PCIe-routed pair far lower — the observable the placement is for. On CPU (tests) it runs
with ``gloo`` and the torch reference GEMM, checking numerics only.

torchrun --nproc-per-node 2 -m aliyun_gpushare_device_plugin_amd.parallel.tp_demo
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=4096)
    ap.add_argument("--d-model", type=int, default=4096)
    ap.add_argument("--d-ff", type=int, default=14336)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--allreduce-mib", type=int, default=256)
    a = ap.parse_args(argv)

    import torch
    import torch.distributed as dist

    rank, world = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    gpu = torch.cuda.is_available()
    if gpu:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local) if gpu else torch.device("cpu")
    dist.init_process_group("nccl" if gpu else "gloo", device_id=dev if gpu else None)
    dt = torch.bfloat16 if gpu else torch.float32
    g = torch.Generator(device="cpu").manual_seed(0)
    T, D, F = a.tokens, a.d_model, a.d_ff
    if not gpu:
        T, D, F = 64, 128, 256
    x = torch.randn(T, D, generator=g).to(dev, dt)
    w_gu = (torch.randn(2 * F, D, generator=g) * 0.02).to(dev, dt)   # full weights, same on every rank
    w_d = (torch.randn(D, F, generator=g) * 0.02).to(dev, dt)
    shard = F // world
    gu_local = torch.cat([w_gu[rank * shard:(rank + 1) * shard], w_gu[F + rank * shard:F + (rank + 1) * shard]])
    d_local = w_d[:, rank * shard:(rank + 1) * shard].contiguous()

    def block():
        if gpu:
            from ..ops import linear, silu_mul
            h = silu_mul(linear(x, gu_local))
            y = linear(h, d_local)
        else:
            gu = x @ gu_local.t()
            h = torch.nn.functional.silu(gu[:, :shard]) * gu[:, shard:]
            y = h @ d_local.t()
        dist.all_reduce(y)
        return y

    y = block()
    gu = x.float() @ w_gu.float().t()
    ref = (torch.nn.functional.silu(gu[:, :F]) * gu[:, F:]) @ w_d.float().t()
    rel = ((y.float() - ref).norm() / ref.norm()).item()

    buf = torch.ones(a.allreduce_mib * (1 << 20) // 2, dtype=dt, device=dev) if gpu else torch.ones(1 << 16)
    for _ in range(3):
        dist.all_reduce(buf)
    if gpu:
        torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        dist.all_reduce(buf)
    if gpu:
        torch.cuda.synchronize()
    dt_s = (time.perf_counter() - t0) / a.iters
    size = buf.numel() * buf.element_size()
    busbw = size * 2 * (world - 1) / world / dt_s / 1e9
    if rank == 0:
        print(json.dumps({"world": world, "tp_block_rel_err": rel, "allreduce_bytes": size,
                          "allreduce_ms": dt_s * 1e3, "busbw_GBps": busbw, "backend": dist.get_backend()}))
    dist.destroy_process_group()
    return 0 if rel < 5e-2 else 1


if __name__ == "__main__":
    sys.exit(main())
