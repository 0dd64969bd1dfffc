"""Helpers over Kubernetes objects kept as plain JSON dicts (no client-go equivalent here)."""
from __future__ import annotations

from .. import const
from ..utils.units import parse_quantity


def meta(o: dict) -> dict:
    return o.setdefault("metadata", {}) if isinstance(o, dict) else {}


def name(o: dict) -> str:
    return (o.get("metadata") or {}).get("name", "")


def namespace(o: dict) -> str:
    return (o.get("metadata") or {}).get("namespace", "default")


def uid(o: dict) -> str:
    return (o.get("metadata") or {}).get("uid", "")


def resource_version(o: dict) -> str:
    return (o.get("metadata") or {}).get("resourceVersion", "")


def annotations(o: dict) -> dict:
    return (o.get("metadata") or {}).get("annotations") or {}


def labels(o: dict) -> dict:
    return (o.get("metadata") or {}).get("labels") or {}


def node_name(pod: dict) -> str:
    return (pod.get("spec") or {}).get("nodeName", "") or ""


def phase(pod: dict) -> str:
    return (pod.get("status") or {}).get("phase", "") or ""


def containers(pod: dict) -> list:
    return (pod.get("spec") or {}).get("containers") or []


def container_limit(c: dict, resource: str = const.RESOURCE_NAME) -> int:
    lim = ((c.get("resources") or {}).get("limits") or {})
    if resource not in lim:
        return 0
    try:
        return parse_quantity(lim[resource])
    except (ValueError, ArithmeticError):
        return 0


def gpu_mem_of_pod(pod: dict) -> int:
    """Σ containers' ``aliyun.com/gpu-mem`` limits; init containers ignored
    (``podutils.go:122-131``, ``inspect/podinfo.go:125-135``)."""
    return sum(container_limit(c) for c in containers(pod))


def gpu_mem_per_container(pod: dict) -> list[int]:
    return [container_limit(c) for c in containers(pod)]


def rv_int(rv: str) -> int:
    try:
        return int(rv)
    except (TypeError, ValueError):
        return -1


def node_allocatable(node: dict, resource: str) -> int:
    v = ((node.get("status") or {}).get("allocatable") or {}).get(resource)
    if v is None:
        return 0
    try:
        return parse_quantity(v)
    except (ValueError, ArithmeticError):
        return 0


def node_capacity(node: dict, resource: str) -> int | None:
    v = ((node.get("status") or {}).get("capacity") or {}).get(resource)
    if v is None:
        return None
    try:
        return parse_quantity(v)
    except (ValueError, ArithmeticError):
        return None


def node_internal_ip(node: dict) -> str:
    for a in (node.get("status") or {}).get("addresses") or []:
        if a.get("type") == "InternalIP":
            return a.get("address", "unknown")
    return "unknown"


def deleting(pod: dict) -> bool:
    """Graceful deletion started (``metadata.deletionTimestamp`` set)."""
    return bool((pod.get("metadata") or {}).get("deletionTimestamp"))


def is_terminated(pod: dict) -> bool:
    return phase(pod) in ("Succeeded", "Failed")
