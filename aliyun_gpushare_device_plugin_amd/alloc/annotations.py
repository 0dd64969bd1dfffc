"""Plugin side of the gpushare-scheduler-extender annotation handshake (component C7).

Reference ``pkg/gpu/nvidia/podutils.go``:
* ``isGPUMemoryAssumedPod`` (``:78-119``): has a ``gpu-mem`` limit, an ``ASSUME_TIME``
  annotation, and ``ASSIGNED == "false"``;
* ``getGPUIDFromPodAnnotation`` (``:37-61``): ``ALIYUN_COM_GPU_MEM_IDX`` → int, -1 on error;
* ``getAssumeTimeFromPodAnnotation`` (``:64-75``): unix-ns uint64, 0 on error;
* ``patchPodAnnotationSpecAssigned`` (``:27-35``): ``{ASSIGNED:"true", ASSUME_TIME:<now ns>}``;
* ordering by assume time ascending (``podmanager.go:326-347``).
"""
from __future__ import annotations

import json
import time

from .. import const
from ..cluster import objects as O
from ..utils import log


def gpu_id_from_annotation(pod: dict) -> int:
    v = O.annotations(pod).get(const.ENV_RESOURCE_INDEX)
    if v is None:
        log.warning("Failed to get dev id for pod %s in ns %s", O.name(pod), O.namespace(pod))
        return -1
    try:
        return int(v)
    except ValueError:
        log.warning("Failed to parse dev id %s for pod %s in ns %s", v, O.name(pod), O.namespace(pod))
        return -1


def assume_time(pod: dict) -> int:
    v = O.annotations(pod).get(const.ENV_RESOURCE_ASSUME_TIME)
    if v is None:
        return 0
    try:
        t = int(v)
        return t if t >= 0 else 0
    except ValueError:
        log.warning("Failed to parse assume Timestamp %s", v)
        return 0


def is_assumed_pod(pod: dict) -> bool:
    if O.gpu_mem_of_pod(pod) <= 0:
        return False
    ann = O.annotations(pod)
    if const.ENV_RESOURCE_ASSUME_TIME not in ann:
        return False
    return ann.get(const.ENV_ASSIGNED_FLAG) == "false"


def is_assigned_pod(pod: dict) -> bool:
    return O.annotations(pod).get(const.ENV_ASSIGNED_FLAG) == "true"


def assigned_patch(now_ns: int | None = None) -> dict:
    now = time.time_ns() if now_ns is None else now_ns
    return {"metadata": {"annotations": {const.ENV_ASSIGNED_FLAG: "true",
                                         const.ENV_RESOURCE_ASSUME_TIME: str(now)}}}


def order_by_assume_time(pods: list[dict]) -> list[dict]:
    # stable sort; the reference's Less uses <= which is not a strict order, so ties keep
    # whatever order LIST returned — we keep arrival order deterministically.
    return sorted(pods, key=assume_time)


def dedupe_by_uid(pods: list[dict], node: str) -> list[dict]:
    """``getPendingPodsInNode`` (``podmanager.go:273-291``): drop other nodes' pods, dedupe."""
    seen, out = set(), []
    for p in pods:
        md = p.get("metadata") or {}
        if (p.get("spec") or {}).get("nodeName") != node:
            log.warning("Pod %s in ns %s is not assigned to node %s as expected, it's placed on node %s",
                        md.get("name"), md.get("namespace"), node, O.node_name(p))
            continue
        u = md.get("uid")
        if u in seen:
            continue
        seen.add(u)
        out.append(p)
    return out


def allocation_from_annotation(pod: dict) -> dict[int, int]:
    """``scheduler.framework.gpushare.allocation`` = ``{"<ctr>": {"<gpu>": mem}}`` summed per
    GPU (``cmd/inspect/nodeinfo.go:245-272``). Empty dict when absent or malformed."""
    raw = O.annotations(pod).get(const.GPUSHARE_ALLOCATION_FLAG)
    if not raw:
        return {}
    try:
        alloc = json.loads(raw)
        out: dict[int, int] = {}
        for per_ctr in alloc.values():
            for gpu, mem in per_ctr.items():
                out[int(gpu)] = out.get(int(gpu), 0) + int(mem)
        return out
    except (ValueError, AttributeError, TypeError):
        return {}
