"""Node-level state the plugin writes or reads.

* ``patch_gpu_count`` — ``aliyun.com/gpu-count`` capacity/allocatable via a node-status
  strategic-merge PATCH; skipped when already equal (``podmanager.go:160-185``). The
  reference computes a two-way merge diff of the whole node (``:77-158``); the only field
  it changes is this one, so the patch is built directly and never touches addresses.
* ``cgpu_isolation_disabled`` — node label ``cgpu.disable.isolation=true``
  (``podmanager.go:62-75``).
* ``export_topology`` / ``export_health`` — AMD additions: the xGMI link matrix and per-GPU
  health as node annotations, consumed by a TP-aware extender and by the inspect CLI.
"""
from __future__ import annotations

import json

from .. import const
from ..utils import log
from . import objects as O
from .client import APIClient


def patch_gpu_count(client: APIClient, node_name: str, gpu_count: int) -> bool:
    """Returns True when a PATCH was sent."""
    node = client.get_node(node_name)
    cur = O.node_capacity(node, const.RESOURCE_COUNT)
    if cur == gpu_count:
        log.info("No need to update Capacity %s", const.RESOURCE_COUNT)
        return False
    q = str(int(gpu_count))
    client.patch_node_status(node_name, {"status": {"capacity": {const.RESOURCE_COUNT: q},
                                                    "allocatable": {const.RESOURCE_COUNT: q}}})
    log.info("Updated Capacity %s=%s successfully.", const.RESOURCE_COUNT, q)
    return True


def cgpu_isolation_disabled(client: APIClient, node_name: str, quiet: bool = False) -> bool:
    node = client.get_node(node_name)
    if O.labels(node).get(const.NODE_LABEL_DISABLE_CGPU) == "true":
        if not quiet:
            log.info("enable gpusharing mode and disable cgpu mode")
        return True
    return False


def export_annotation(client: APIClient, node_name: str, key: str, value: dict) -> None:
    client.patch_node(node_name, {"metadata": {"annotations": {key: json.dumps(value, sort_keys=True,
                                                                               separators=(",", ":"))}}})


def export_memory_unit(client: APIClient, node_name: str, unit: str) -> None:
    """Record the unit of ``aliyun.com/gpu-mem`` on the node (read by kubectl-inspect-gpushare)."""
    node = client.get_node(node_name)
    if O.annotations(node).get(const.NODE_ANNOTATION_MEMORY_UNIT) != unit:
        client.patch_node(node_name, {"metadata": {"annotations": {const.NODE_ANNOTATION_MEMORY_UNIT: unit}}})


def export_topology(client: APIClient, node_name: str, topology: dict) -> None:
    export_annotation(client, node_name, const.NODE_ANNOTATION_TOPOLOGY, topology)


def export_health(client: APIClient, node_name: str, health: dict) -> None:
    export_annotation(client, node_name, const.NODE_ANNOTATION_HEALTH, health)


def read_topology(node: dict) -> dict | None:
    raw = O.annotations(node).get(const.NODE_ANNOTATION_TOPOLOGY)
    if not raw:
        return None
    try:
        return json.loads(raw)
    except ValueError:
        return None
