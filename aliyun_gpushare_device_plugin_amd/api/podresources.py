"""kubelet pod-resources API ``v1`` — which pod/container holds which device IDs.

An ``AllocateRequest`` names no pod (reference ``allocate.go:55-57`` only counts fake IDs), so
the plugin cannot tell from Allocate alone which of two equal-size pods the kubelet is
admitting. The kubelet publishes the answer after the fact on
``/var/lib/kubelet/pod-resources/kubelet.sock`` (``PodResourcesLister``, GA since 1.20): every
active pod's containers with the device IDs the device manager checkpointed for them. The
plugin reads it to make the extender's placement annotations follow where containers actually
run (``alloc/placement.py``).

Field numbers, types and method paths are those of upstream
``k8s.io/kubelet/pkg/apis/podresources/v1/api.proto``; ``dynamic_resources`` (DRA, field 5 of
``ContainerResources``) is left out — proto3 parsers skip unknown fields, and the plugin never
reads it. Golden-byte tests: ``tests/test_api_wire.py``.
"""
from __future__ import annotations

import dataclasses

from . import _proto
from ._proto import I64, MSG, OPT, REP, STR, U64

PACKAGE = "v1"
SOCKET = "/var/lib/kubelet/pod-resources/kubelet.sock"

_MESSAGES = [
    ("AllocatableResourcesRequest", []),
    ("AllocatableResourcesResponse", [("devices", 1, REP, MSG, "ContainerDevices"),
                                      ("cpu_ids", 2, REP, I64, None),
                                      ("memory", 3, REP, MSG, "ContainerMemory")]),
    ("ListPodResourcesRequest", []),
    ("ListPodResourcesResponse", [("pod_resources", 1, REP, MSG, "PodResources")]),
    ("PodResources", [("name", 1, OPT, STR, None),
                      ("namespace", 2, OPT, STR, None),
                      ("containers", 3, REP, MSG, "ContainerResources")]),
    ("ContainerResources", [("name", 1, OPT, STR, None),
                            ("devices", 2, REP, MSG, "ContainerDevices"),
                            ("cpu_ids", 3, REP, I64, None),
                            ("memory", 4, REP, MSG, "ContainerMemory")]),
    ("ContainerMemory", [("memory_type", 1, OPT, STR, None),
                         ("size", 2, OPT, U64, None),
                         ("topology", 3, OPT, MSG, "TopologyInfo")]),
    ("ContainerDevices", [("resource_name", 1, OPT, STR, None),
                          ("device_ids", 2, REP, STR, None),
                          ("topology", 3, OPT, MSG, "TopologyInfo")]),
    ("TopologyInfo", [("nodes", 1, REP, MSG, "NUMANode")]),
    ("NUMANode", [("ID", 1, OPT, I64, None)]),
    ("GetPodResourcesRequest", [("pod_name", 1, OPT, STR, None),
                                ("pod_namespace", 2, OPT, STR, None)]),
    ("GetPodResourcesResponse", [("pod_resources", 1, OPT, MSG, "PodResources")]),
]

SERVICES = {
    "PodResourcesLister": [
        ("List", "ListPodResourcesRequest", "ListPodResourcesResponse", False),
        ("GetAllocatableResources", "AllocatableResourcesRequest", "AllocatableResourcesResponse", False),
        ("Get", "GetPodResourcesRequest", "GetPodResourcesResponse", False),
    ],
}

PROTO = _proto.ProtoFile("podresources/v1/api.proto", PACKAGE, _MESSAGES, SERVICES)
FILE_DESCRIPTOR = PROTO.descriptor

ListPodResourcesRequest = PROTO["ListPodResourcesRequest"]
ListPodResourcesResponse = PROTO["ListPodResourcesResponse"]
PodResources = PROTO["PodResources"]
ContainerResources = PROTO["ContainerResources"]
ContainerDevices = PROTO["ContainerDevices"]
GetPodResourcesRequest = PROTO["GetPodResourcesRequest"]
GetPodResourcesResponse = PROTO["GetPodResourcesResponse"]
AllocatableResourcesRequest = PROTO["AllocatableResourcesRequest"]
AllocatableResourcesResponse = PROTO["AllocatableResourcesResponse"]


@dataclasses.dataclass(frozen=True)
class PodDevices:
    """One pod's holdings of one resource: ``containers`` = ((container name, device IDs), ...)
    in the order the kubelet lists them. The kubelet reports one ``ContainerDevices`` per device
    (each with its own topology), so the IDs of a container are the union over entries."""
    namespace: str
    name: str
    containers: tuple


def pod_devices(resp, resource: str, include_empty: bool = False) -> list[PodDevices]:
    """Per pod, its containers' IDs of ``resource``. ``include_empty``: also list pods and
    containers holding none yet — the kubelet adds a pod to its pod manager right before
    admitting it, so a Pending pod whose gpu containers hold no (or only some) IDs is the one
    whose ``Allocate`` calls are in progress (``alloc/engine.py`` admission identity)."""
    out = []
    for pr in resp.pod_resources:
        ctrs = []
        for c in pr.containers:
            ids = [i for d in c.devices if d.resource_name == resource for i in d.device_ids]
            if ids or include_empty:
                ctrs.append((c.name, tuple(ids)))
        if ctrs:
            out.append(PodDevices(pr.namespace, pr.name, tuple(ctrs)))
    return out


class PodResourcesClient:
    """``PodResourcesLister`` client over the kubelet's pod-resources socket. The channel is
    kept open (a local UDS); ``list`` costs one RPC."""

    def __init__(self, socket_path: str = SOCKET, resource: str | None = None, timeout: float = 2.0):
        from .. import const

        self.socket, self.timeout = socket_path, timeout
        self.resource = resource or const.RESOURCE_NAME
        self._ch = None
        self._stub = None

    def _connect(self):
        import grpc

        if self._stub is None:
            self._ch = grpc.insecure_channel(_proto.unix_target(self.socket))
            self._stub = PROTO.stub(self._ch, "PodResourcesLister")
        return self._stub

    def list(self, include_empty: bool = False, timeout: float | None = None) -> list[PodDevices]:
        import grpc

        try:
            resp = self._connect().List(ListPodResourcesRequest(), timeout=timeout or self.timeout)
        except grpc.RpcError:
            self.close()        # the kubelet restarted: re-dial on the next call
            raise
        return pod_devices(resp, self.resource, include_empty)

    def available(self) -> bool:
        import os

        return os.path.exists(self.socket)

    def close(self):
        if self._ch is not None:
            self._ch.close()
        self._ch = self._stub = None
