"""``gpu-player`` for MI355X: the bin-pack demo workload (reference demo image
``cheyang/gpu-player:v2``, ``demo/binpack-1/binpack-1.yaml:39``).

A player owns an HBM share (the pod's ``aliyun.com/gpu-mem`` grant) and generates real
matrix-core traffic in it: bf16 GEMMs on the hand-written gfx950 MFMA kernel, operands
carved out of the share, on the player's own HIP stream so co-located players genuinely
share the GPU. Inside a container the share is enforced by the quota shim; in the bench the
players of one GPU run in one process and the share is allocated explicitly.
"""
from __future__ import annotations

import torch

from ..ops import gemm_nt, gemm_nt_repeat

GIB = 1 << 30


class GemmPlayer:
    def __init__(self, share_bytes: int, device: torch.device | int = 0, m: int = 4096, n: int = 4096,
                 k: int = 4096, touch_fraction: float = 0.9, seed: int = 0, pool: torch.Tensor | None = None,
                 fused_burst: bool = False):
        # fused_burst: a burst is ONE dispatch of `iters` identical GEMMs (ops.gemm_nt_repeat)
        # instead of `iters` launches, so the CUs never drain at kernel boundaries
        self.fused_burst = fused_burst
        self.device = torch.device("cuda", device) if isinstance(device, int) else device
        self.m, self.n, self.k = m, n, k
        self.stream = torch.cuda.Stream(self.device)
        need = (m * k + n * k + m * n) * 2
        self.share_bytes = int(share_bytes * touch_fraction) if pool is None else pool.numel() * 2
        if self.share_bytes < need:
            raise ValueError(f"share of {share_bytes} bytes cannot hold a {m}x{n}x{k} GEMM working set")
        # The pod's HBM share, in one piece like a framework's memory pool: either a slice of a
        # caller-owned arena (``pool``, see HBMArena) or its own allocation. An own allocation is
        # made on the device's default stream and recorded onto the pod stream: PyTorch's
        # caching allocator pools blocks per allocating stream, so a share freed by a retired
        # pod is then reusable by its replacement instead of forcing free-all + hipMalloc.
        self.pool = pool if pool is not None else torch.empty(self.share_bytes // 2, dtype=torch.bfloat16,
                                                               device=self.device)
        self.pool.record_stream(self.stream)
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.stream):
            off = 0

            def carve(r, c):
                nonlocal off
                t = self.pool[off: off + r * c].view(r, c)
                off += r * c
                return t

            self.a, self.b, self.c = carve(m, k), carve(n, k), carve(m, n)
            g = torch.Generator(device=self.device).manual_seed(seed)
            self.a.uniform_(-1, 1, generator=g)
            self.b.uniform_(-1, 1, generator=g)
        self.flops = 0.0

    def run(self, iters: int):
        with torch.cuda.stream(self.stream):
            if self.fused_burst:
                gemm_nt_repeat(self.a, self.b, self.c, iters)
            else:
                for _ in range(iters):
                    gemm_nt(self.a, self.b, out=self.c)
        self.flops += 2.0 * self.m * self.n * self.k * iters

    def synchronize(self):
        self.stream.synchronize()

    def release(self):
        self.synchronize()
        self.a = self.b = self.c = self.pool = None


class HBMArena:
    """A GPU's shareable HBM allocated once and handed out in gpu-mem units (first fit).

    Mirrors what the node really looks like — pods' shares are disjoint ranges of one device's
    memory — without a multi-GB hipMalloc/hipFree each time a pod lands on the GPU (a pod that
    replaces one of a different size would otherwise miss PyTorch's block cache and force
    free-all + re-map of tens of GB). ``alloc`` returns None when no contiguous run of units
    is free; callers then fall back to an own allocation.
    """

    def __init__(self, device: torch.device, units: int, touch_fraction: float = 0.9):
        total = torch.cuda.get_device_properties(device).total_memory
        self.units = units
        self.unit_elems = int(total * touch_fraction) // units // 2
        self.buf = torch.empty(self.unit_elems * units, dtype=torch.bfloat16, device=device)
        self.owner: list[str | None] = [None] * units

    def alloc(self, key: str, n_units: int) -> torch.Tensor | None:
        run = 0
        for i, o in enumerate(self.owner):
            run = run + 1 if o is None else 0
            if run == n_units:
                start = i - n_units + 1
                for j in range(start, i + 1):
                    self.owner[j] = key
                return self.buf[start * self.unit_elems: (i + 1) * self.unit_elems]
        return None

    def free(self, key: str) -> None:
        self.owner = [None if o == key else o for o in self.owner]
