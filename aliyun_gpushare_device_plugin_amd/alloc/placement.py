"""Placement truth: the extender's per-pod GPU annotations follow where containers really run.

The problem (reference ``allocate.go:43-152``, inherited by every gpushare plugin): an
``AllocateRequest`` carries fake device IDs and nothing else (``allocate.go:55-57``), so the
plugin answers "the oldest assumed pod of this size" (``allocate.go:79-89``). When the kubelet
admits two equal-size pods A (``IDX=0``) and B (``IDX=1``) in the other order, B's container is
handed GPU 0 and A's GPU 1, while the annotations keep saying A→0, B→1. Per-GPU sums agree while
both live; once A is deleted, the extender (which rebuilds its ledger from ``IDX`` /
``scheduler.framework.gpushare.allocation``, like ``cmd/inspect/nodeinfo.go:169-197``) frees GPU
0 — which physically still holds B — and over-commits it with the next pod.

The kubelet knows which pod got which fake IDs: it checkpoints them and publishes them on the
pod-resources API (``api/podresources.py``). The plugin keeps a **grant book** — for every
container it answered, the fake-ID set → (GPU, units, the pod it matched, CU slots, ledger
key) — and this module joins the two:

* a pod whose every gpu container holds a known grant is **allocated**; its truthful
  annotations are the grants' GPUs (``IDX``, plus the per-container allocation JSON when it has
  one or its containers landed on different GPUs) and ``ASSIGNED=true``;
* a grant answered recently whose IDs no pod holds yet is **in flight**: it is assumed to be
  where it was answered (the pod it matched keeps its annotation);
* every other live gpu pod is **unallocated**: it still needs its reservation. The extender's
  per-GPU total (Σ annotations of live pods) must not change, so the budget left per GPU is
  that total minus what allocated and in-flight pods physically use there. Unallocated pods
  that fit their current ``IDX`` keep it; the others (their reservation was consumed by
  another pod) move to a GPU with budget left — for an equal-size swap that is exactly the
  reservation the other pod did not use — and are reset to ``ASSIGNED=false`` so their own
  admission matches them again.

``plan`` is pure (tested with hypothesis in ``tests/test_properties.py``); the engine applies
its fixes through the same ordered patch queue as its ASSIGNED patches (``alloc/engine.py``).
"""
from __future__ import annotations

import collections
import dataclasses
import hashlib
import json
import threading

from .. import const
from ..cluster import objects as O
from . import annotations as A


def ids_key(ids) -> str:
    """Key of one container's fake-ID set (equals ``journal.request_key`` for a one-container
    request, the only shape the kubelet sends)."""
    return hashlib.sha1("\x1f".join(sorted(ids)).encode()).hexdigest()


@dataclasses.dataclass
class Grant:
    gpu: int
    units: int
    claimed: str            # uid of the pod the answer was matched to ("" = single-GPU fallback)
    t: float                # wall time of the answer
    cu: str | None = None   # CU-slot run answered (alloc/cuslots.py annotation form)
    ledger: str = ""        # ledger key of the container (quota/ledger.py)


class GrantBook:
    """Answered containers by fake-ID set. Bounded: a grant is needed only until the
    kubelet's pod-resources shows who holds it (seconds), and grants of pods that are gone are
    dropped by ``prune``."""

    def __init__(self, max_entries: int = 65536):
        self._g: collections.OrderedDict[str, Grant] = collections.OrderedDict()
        self._mu = threading.Lock()
        self.max_entries = max_entries

    def record(self, key: str, g: Grant) -> None:
        with self._mu:
            self._g[key] = g
            self._g.move_to_end(key)
            while len(self._g) > self.max_entries:
                self._g.popitem(last=False)

    def get(self, key: str) -> Grant | None:
        with self._mu:
            return self._g.get(key)

    def items(self) -> list[tuple[str, Grant]]:
        with self._mu:
            return list(self._g.items())

    def prune(self, keep_keys: set, live_uids: set, now: float, in_flight_s: float) -> None:
        """Drop grants no pod holds (``keep_keys``), whose matched pod is gone, and that are
        too old to still be in flight."""
        with self._mu:
            for k in [k for k, g in self._g.items()
                      if k not in keep_keys and g.claimed not in live_uids and now - g.t > in_flight_s]:
                del self._g[k]

    def __len__(self):
        return len(self._g)


@dataclasses.dataclass
class Fix:
    uid: str
    ns: str
    name: str
    ann: dict                   # annotation values to write (None = delete the key)
    assigned: bool | None       # True: the pod now holds a grant; False: reservation re-armed
    holder_of: list = dataclasses.field(default_factory=list)   # grants (keys) this pod holds
    reason: str = ""


def annotated_usage(pod: dict) -> dict[int, int]:
    """Per-GPU units the extender attributes to ``pod`` (allocation JSON, else IDX × total)."""
    alloc = A.allocation_from_annotation(pod)
    if alloc:
        return alloc
    g = _idx(pod)
    total = O.gpu_mem_of_pod(pod)
    return {g: total} if g >= 0 and total > 0 else {}


def _idx(pod: dict) -> int:
    try:
        return int(O.annotations(pod).get(const.ENV_RESOURCE_INDEX, "-1"))
    except ValueError:
        return -1


def _gpu_containers(pod: dict) -> list[tuple[int, str, int]]:
    """(index in spec.containers, name, gpu-mem units) of each container with a gpu-mem limit."""
    out = []
    for i, c in enumerate(O.containers(pod)):
        n = O.container_limit(c, const.RESOURCE_NAME)
        if n > 0:
            out.append((i, c.get("name", ""), n))
    return out


def _alloc_json(per_ctr: dict[int, tuple[int, int]]) -> str:
    return json.dumps({str(ci): {str(g): u} for ci, (g, u) in sorted(per_ctr.items())}, separators=(",", ":"))


def plan(pods: list[dict], held, book: GrantBook, now: float, in_flight_s: float = 30.0) -> list[Fix]:
    """Fixes that make the annotations of ``pods`` (this node's live pods) match physical
    placement. ``held`` = ``podresources.PodDevices`` of this node (the kubelet's view)."""
    live = [p for p in pods if not O.deleting(p) and not O.is_terminated(p) and O.gpu_mem_of_pod(p) > 0]
    by_name = {(O.namespace(p), O.name(p)): p for p in live}
    held_keys: set[str] = set()
    phys: dict[str, dict[int, tuple[int, int]]] = {}    # uid -> ctr index -> (gpu, units)
    holds: dict[str, list[str]] = {}
    cu_of: dict[str, str | None] = {}
    unknown: set[str] = set()                           # holds devices we cannot attribute
    seen_uids: set[str] = set()
    for pd in held:
        for _, ids in pd.containers:
            held_keys.add(ids_key(ids))
        p = by_name.get((pd.namespace, pd.name))
        if p is None:
            continue
        u = O.uid(p)
        seen_uids.add(u)
        idx_of = {name: (ci, n) for ci, name, n in _gpu_containers(p)}
        per = {}
        for cname, ids in pd.containers:
            k = ids_key(ids)
            g = book.get(k)
            ci = idx_of.get(cname)
            if g is None or ci is None or g.gpu < 0:
                unknown.add(u)
                continue
            per[ci[0]] = (g.gpu, len(ids))
            holds.setdefault(u, []).append(k)
            if cu_of.get(u) is None:
                cu_of[u] = g.cu
        if u not in unknown and len(per) == len(idx_of):
            phys[u] = per
        elif u not in unknown:
            unknown.add(u)                              # mid-admission (multi-container pod)
    # answers whose IDs nobody holds yet: assumed to sit where they were answered
    in_flight: dict[str, list[Grant]] = {}
    for k, g in book.items():
        if k not in held_keys and g.claimed and now - g.t <= in_flight_s:
            in_flight.setdefault(g.claimed, []).append(g)

    fixes: list[Fix] = []
    annotated: collections.Counter = collections.Counter()
    used: collections.Counter = collections.Counter()
    unallocated = []
    for p in live:
        u = O.uid(p)
        ann_use = annotated_usage(p)
        annotated.update(ann_use)
        if u in phys:
            for g, n in phys[u].values():
                used[g] += n
            want = collections.Counter()
            for g, n in phys[u].values():
                want[g] += n
            split = len(want) > 1
            cur = O.annotations(p)
            fix_ann = {}
            main = max(sorted(want), key=lambda g: want[g])
            if str(main) != cur.get(const.ENV_RESOURCE_INDEX):
                fix_ann[const.ENV_RESOURCE_INDEX] = str(main)
            if split or const.GPUSHARE_ALLOCATION_FLAG in cur:
                aj = _alloc_json(phys[u])
                if A.allocation_from_annotation(p) != dict(want) or cur.get(const.GPUSHARE_ALLOCATION_FLAG) != aj:
                    fix_ann[const.GPUSHARE_ALLOCATION_FLAG] = aj
            cu = cu_of.get(u)
            if cu and cur.get(const.POD_ANNOTATION_CU_SLOTS) != cu and fix_ann:
                fix_ann[const.POD_ANNOTATION_CU_SLOTS] = cu
            assigned = None if A.is_assigned_pod(p) else True
            if fix_ann or assigned:
                fixes.append(Fix(u, O.namespace(p), O.name(p), fix_ann, assigned, holds.get(u, []), "holder"))
        elif u in unknown or u in in_flight or (u in seen_uids):
            if u in in_flight and u not in unknown:
                for g in in_flight[u]:
                    used[g.gpu] += g.units
            else:
                used.update(ann_use)
        else:
            unallocated.append(p)

    budget = collections.Counter({g: annotated[g] - used[g] for g in set(annotated) | set(used)})
    overflow = []
    for p in A.order_by_assume_time(unallocated):
        need = annotated_usage(p)
        if need and all(budget[g] >= n for g, n in need.items()):
            for g, n in need.items():
                budget[g] -= n
        else:
            overflow.append(p)
    for p in overflow:
        total = O.gpu_mem_of_pod(p)
        fits = [g for g in sorted(budget) if budget[g] >= total]
        if not fits:
            continue                                    # nothing exact left: leave it to the extender
        g = min(fits, key=lambda x: (budget[x] - total, x))
        budget[g] -= total
        ann = {const.ENV_RESOURCE_INDEX: str(g)}
        if const.GPUSHARE_ALLOCATION_FLAG in O.annotations(p):
            ann[const.GPUSHARE_ALLOCATION_FLAG] = _alloc_json({ci: (g, n) for ci, _, n in _gpu_containers(p)})
        if const.POD_ANNOTATION_CU_SLOTS in O.annotations(p):
            ann[const.POD_ANNOTATION_CU_SLOTS] = None
        fixes.append(Fix(O.uid(p), O.namespace(p), O.name(p), ann,
                         False if A.is_assigned_pod(p) else None, [], "rehomed"))
    return fixes


def physical_usage(held, book: GrantBook) -> dict[int, int]:
    """Per-GPU units held by containers according to the kubelet and the grant book."""
    out: collections.Counter = collections.Counter()
    for pd in held:
        for _, ids in pd.containers:
            g = book.get(ids_key(ids))
            if g is not None:
                out[g.gpu] += len(ids)
    return dict(out)
