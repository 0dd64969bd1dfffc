"""Where a pod's state allocation time goes on MI355X: ``hipMalloc`` cost per GiB, by chunk size,
on fresh HBM and on HBM that amdgpu has just wiped after a free (``bench.py`` pod cycle, phase
``hold``). One process, no shim. Prints one JSON line per measurement.

    python tools/alloc_probe.py --gib 64
"""
from __future__ import annotations

import argparse
import json
import time

import torch


def used() -> int:
    free, total = torch.cuda.mem_get_info()
    return total - free


def alloc(gib: int, chunk_mib: int):
    t0 = time.perf_counter()
    n = (gib << 30) // (chunk_mib << 20)
    bufs = [torch.empty((chunk_mib << 20) // 2, dtype=torch.bfloat16, device="cuda") for _ in range(n)]
    torch.cuda.synchronize()
    return bufs, time.perf_counter() - t0


def free_all(bufs) -> tuple[float, float]:
    base = used() - sum(b.numel() * 2 for b in bufs)
    t0 = time.perf_counter()
    bufs.clear()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    t1 = time.perf_counter()
    while used() > base + (1 << 30) and time.perf_counter() - t1 < 30:
        time.sleep(0.002)
    return t1 - t0, time.perf_counter() - t1


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=int, default=64)
    ap.add_argument("--chunks", default="2048,256,8192,256,2048,64")
    ap.add_argument("--settle", type=float, default=8.0)
    a = ap.parse_args()
    torch.empty(1, device="cuda")
    for chunk in (int(c) for c in a.chunks.split(",")):
        bufs, t_alloc = alloc(a.gib, chunk)
        t_free, t_back = free_all(bufs)
        bufs, t_realloc = alloc(a.gib, chunk)            # HBM that amdgpu is still wiping
        t = time.perf_counter()
        bufs[0].fill_(1)
        torch.cuda.synchronize()
        t_touch = time.perf_counter() - t
        free_all(bufs)
        time.sleep(a.settle)                              # wipes done
        bufs, t_settled = alloc(a.gib, chunk)
        free_all(bufs)
        time.sleep(a.settle)
        print(json.dumps({"probe": "alloc", "gib": a.gib, "chunk_mib": chunk,
                          "alloc_ms": round(t_alloc * 1e3, 1), "alloc_GBps": round((a.gib << 30) / t_alloc / 1e9, 1),
                          "free_ms": round(t_free * 1e3, 1), "returned_after_ms": round(t_back * 1e3, 1),
                          "realloc_ms": round(t_realloc * 1e3, 1),
                          "realloc_GBps": round((a.gib << 30) / t_realloc / 1e9, 1),
                          "settled_alloc_ms": round(t_settled * 1e3, 1),
                          "first_fill_ms": round(t_touch * 1e3, 2)}), flush=True)
    # allocate while the previous free is still being wiped
    bufs, _ = alloc(a.gib, 2048)
    bufs.clear()
    torch.cuda.empty_cache()
    t0 = time.perf_counter()
    bufs, t_alloc = alloc(a.gib // 4, 2048)
    print(json.dumps({"probe": "alloc_during_wipe", "gib": a.gib // 4, "alloc_ms": round(t_alloc * 1e3, 1),
                      "alloc_GBps": round((a.gib // 4 << 30) / t_alloc / 1e9, 1)}), flush=True)
    free_all(bufs)


if __name__ == "__main__":
    main()
