"""Feasibility probe for the per-GPU HBM broker (docs/HBM_TURNOVER.md).

A long-lived "broker" process holds a large HBM block. It hands the block to a short-lived
"tenant" process through HIP IPC (torch CUDA-tensor sharing: dma-buf on this pool). The tenant
writes it and exits. The broker zeroes the block with a memset kernel and hands it to the next
tenant. For comparison, the same tenant allocates a fresh block right after another process
freed one of the same size, which is the path the bench's churn takes and which waits for the
amdgpu wipe.

Prints one JSON line: times to import, write and zero the block, and for the fresh allocation
after a free.

    python tools/diag/hbm_broker_probe.py --gib 48
"""
from __future__ import annotations

import argparse
import json
import time

import torch
import torch.multiprocessing as mp


def tenant(q_in, q_out):
    t0 = time.perf_counter()
    blk = q_in.get()                              # the broker's block, imported through IPC
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    blk.fill_(7)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    q_out.put({"import_ms": (t1 - t0) * 1e3, "write_ms": (t2 - t1) * 1e3, "first_byte": int(blk[0].item())})
    del blk
    q_in.get()                                    # the broker's "done": exit only then (IPC rule)


def fresh(gib, q_out, hold_s):
    # another tenant: allocate, hold, free and exit; the next one allocates right after
    t0 = time.perf_counter()
    x = torch.empty(gib << 30, dtype=torch.uint8, device="cuda")
    x.fill_(1)
    torch.cuda.synchronize()
    q_out.put({"alloc_ms": (time.perf_counter() - t0) * 1e3})
    time.sleep(hold_s)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gib", type=int, default=48)
    a = ap.parse_args(argv)
    ctx = mp.get_context("spawn")
    out = {"gib": a.gib}

    # --- broker path ------------------------------------------------------------------------
    blk = torch.empty(a.gib << 30, dtype=torch.uint8, device="cuda")
    blk.zero_()
    torch.cuda.synchronize()
    for k in range(2):
        q_in, q_out = ctx.Queue(), ctx.Queue()
        p = ctx.Process(target=tenant, args=(q_in, q_out))
        p.start()
        q_in.put(blk)
        r = q_out.get(timeout=120)
        q_in.put("done")
        p.join(60)
        t0 = time.perf_counter()
        blk.zero_()                               # the broker's scrub before the next tenant
        torch.cuda.synchronize()
        r["zero_ms"] = (time.perf_counter() - t0) * 1e3
        r["zero_GBps"] = (a.gib << 30) / (r["zero_ms"] / 1e3) / 1e9
        out[f"broker_tenant_{k}"] = {x: round(v, 2) if isinstance(v, float) else v for x, v in r.items()}
    del blk
    torch.cuda.empty_cache()
    time.sleep(5)                                 # let amdgpu finish returning it

    # --- fresh allocation right after a free (the churn's path) -----------------------------------
    # fill the GPU so that only the tenant's block (plus a little) is free: the next tenant's
    # allocation must reuse exactly the memory the previous one freed, as in the full node
    free, _ = torch.cuda.mem_get_info()
    filler = torch.empty(max(0, free - ((a.gib + 4) << 30)), dtype=torch.uint8, device="cuda")
    out["filler_gib"] = round(filler.numel() / (1 << 30), 1)
    q = ctx.Queue()
    p = ctx.Process(target=fresh, args=(a.gib, q, 0.5))
    p.start()
    first = q.get(timeout=120)
    p.join(60)                                    # exits: its VRAM goes back through the wipe
    t0 = time.perf_counter()
    p2 = ctx.Process(target=fresh, args=(a.gib, q, 0.0))
    p2.start()
    second = q.get(timeout=300)
    p2.join(60)
    out["fresh_after_free"] = {"first_alloc_ms": round(first["alloc_ms"], 1),
                               "alloc_after_free_ms": round(second["alloc_ms"], 1),
                               "spawn_to_ready_ms": round((time.perf_counter() - t0) * 1e3, 1)}
    del filler
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
