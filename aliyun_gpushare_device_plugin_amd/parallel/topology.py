"""xGMI topology export and TP-group placement (new capability; no reference counterpart).

The reference has no topology at all (``Device.Topology`` left nil, ``nvidia.go:79-81``).
MI355X nodes connect their 8 GPUs with point-to-point xGMI (7 links per GPU, ≈153 GB/s
each), so on a healthy UBB every pair is one hop — but a downed link, a CPX/NPS partition
mode or a missing GPU breaks that symmetry, and an RCCL tensor-parallel pod group placed
across a non-xGMI pair falls back to PCIe. The plugin exports the link matrix as a node
annotation (``gpushare.amd.com/xgmi-topology``); ``best_group`` is the placement rule a
TP-aware extender (and ``extender/core.py``) applies to it.
"""
from __future__ import annotations

import itertools

from ..device import smi as S


def build_topology(smi: S.SMI, indices: list[int] | None = None) -> dict:
    from ..device.model import partition_layout

    devs = smi.devices()
    sel = [d for d in devs if indices is None or d.index in set(indices)]
    m = smi.link_matrix()
    idx = [d.index for d in sel]
    sockets, parts, _ = partition_layout(devs)
    return {
        "version": 1,
        "hive_id": format(sel[0].hive_id, "x") if sel else "0",
        "gpus": [{"index": k, "uuid": d.uuid, "bdf": d.bdf, "numa": d.numa_node,
                  "partition": d.compute_partition, "nps": d.memory_partition,
                  "socket": sockets[d.index], "partition_index": parts[d.index]} for k, d in enumerate(sel)],
        "link_type": [[m[i][j].type_name for j in idx] for i in idx],
        "hops": [[m[i][j].hops for j in idx] for i in idx],
        "weight": [[m[i][j].weight for j in idx] for i in idx],
    }


def xgmi_connected(topo: dict, a: int, b: int) -> bool:
    if a == b:
        return True
    lt = topo.get("link_type") or []
    try:
        return lt[a][b] == "xgmi" and topo["hops"][a][b] == 1
    except (IndexError, KeyError):
        return False


def best_group(topo: dict | None, free: list[int], size: int, request: int,
               exclude: set[int] | None = None) -> list[int] | None:
    """Pick ``size`` distinct GPUs, each with ``free[i] >= request``, pairwise one-hop xGMI.

    Tie-break for bin-packing density: minimise the summed leftover capacity (best fit),
    then the summed hop count (for partially connected graphs), then indices.
    Returns None when no such group exists.
    """
    exclude = exclude or set()
    ok = [i for i, f in enumerate(free) if f >= request and i not in exclude]
    if len(ok) < size:
        return None
    best, best_key = None, None
    n = len(free)
    for combo in itertools.combinations(ok, size):
        if topo is not None and n == len(topo.get("link_type") or []):
            if not all(xgmi_connected(topo, a, b) for a, b in itertools.combinations(combo, 2)):
                continue
            hops = sum(topo["hops"][a][b] for a, b in itertools.combinations(combo, 2))
        else:
            hops = 0
        key = (sum(free[i] - request for i in combo), hops, combo)
        if best_key is None or key < best_key:
            best, best_key = list(combo), key
    return best


def verdict(topo: dict | None, n: int, healthy: list | None = None) -> tuple[bool, list[str]]:
    """Pass/fail of the topology the plugin exported for an ``n``-GPU node: present, ``n × n``,
    and — on a healthy UBB (every GPU healthy) — every pair one-hop xGMI. Returns (ok, reasons)."""
    why = []
    lt = (topo or {}).get("link_type")
    if not lt:
        return False, ["no xGMI topology annotation on the node"]
    if len(lt) != n or any(len(r) != n for r in lt) or len((topo or {}).get("hops") or []) != n:
        return False, [f"topology matrix is {len(lt)}x{len(lt[0]) if lt else 0}, expected {n}x{n}"]
    if healthy is None or all(healthy):
        bad = [(a, b, lt[a][b], topo["hops"][a][b]) for a, b in itertools.combinations(range(n), 2)
               if not xgmi_connected(topo, a, b)]
        why += [f"GPU pair {a}-{b}: {t}, {h} hop(s) (healthy UBB: one-hop xGMI expected)" for a, b, t, h in bad]
    return not why, why


def bench_report(rank: int, world: int, use_gpu: bool, topo: dict | None, device=None, mib: int = 256,
                 iters: int = 10) -> dict | None:
    """Multi-GPU bench section (collective: every rank calls it). Rank 0 brings the topology
    the plugin exported from SMI; the TP pair a topology-aware extender would choose for a
    2-GPU pod group (``best_group``) runs an RCCL all-reduce (``torch.distributed`` backend
    ``nccl`` = RCCL) over its link and reports bus bandwidth — one xGMI hop is ≈ link speed,
    a PCIe-routed pair far lower. Returns the report on rank 0, None elsewhere."""
    import time

    import torch
    import torch.distributed as dist

    pair = None
    if rank == 0:
        n = len((topo or {}).get("link_type") or [])
        pair = best_group(topo, [1] * n, 2, 1) if n >= 2 else None
        pair = pair or [0, 1]
    box = [pair]
    dist.broadcast_object_list(box, src=0)
    pair = box[0]
    grp = dist.new_group(pair)
    busbw = None
    if rank in pair:
        if use_gpu:
            buf = torch.ones(mib * (1 << 20) // 2, dtype=torch.bfloat16, device=device)
        else:
            buf = torch.ones(1 << 16, dtype=torch.float32)
        for _ in range(3):
            dist.all_reduce(buf, group=grp)
        if use_gpu:
            torch.cuda.synchronize()
        dist.barrier(group=grp)
        t0 = time.perf_counter()
        for _ in range(iters):
            dist.all_reduce(buf, group=grp)
        if use_gpu:
            torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / iters
        size = buf.numel() * buf.element_size()
        busbw = {"bytes": size, "ms": round(dt * 1e3, 3), "busbw_GBps": round(size * 2 * (len(pair) - 1) / len(pair)
                                                                              / dt / 1e9, 2)}
    out = [None] * world
    dist.all_gather_object(out, busbw)
    dist.destroy_process_group(grp)
    if rank != 0:
        return None
    a, b = pair
    rep = {"tp_pair": pair, "tp_pair_allreduce": out[a], "backend": dist.get_backend()}
    if topo:
        rep.update(hive_id=topo.get("hive_id"), link_type=topo.get("link_type"), hops=topo.get("hops"),
                   pair_link=topo["link_type"][a][b], pair_hops=topo["hops"][a][b])
    return rep
