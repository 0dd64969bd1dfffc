"""kubelet device-plugin API ``v1beta1`` — messages and gRPC service plumbing.

The reference links the generated Go package ``k8s.io/kubelet/pkg/apis/deviceplugin/v1beta1``
(``go.mod:14``; used at ``server.go:126,165-172`` and ``allocate.go:43``). There is no protoc
gRPC plugin in this environment, so the ``.proto`` is expressed here as a
``FileDescriptorProto`` built at import time; message classes come from protobuf's message
factory and the services are wired with grpcio generic handlers. Field numbers, types and
full method names are exactly those of upstream ``api.proto`` so the bytes on the wire are
identical (golden-byte tests in ``tests/test_api_wire.py``).
"""
from __future__ import annotations

from . import _proto
from ._proto import BOOL as _BOOL, I32 as _I32, I64 as _I64, MSG as _MSG, OPT as _OPT, REP as _REP, STR as _STR

PACKAGE = "v1beta1"
VERSION = "v1beta1"

# (message name, [(field name, number, label, type, type_name or None, json_name or None)])
_MESSAGES = [
    ("DevicePluginOptions", [("pre_start_required", 1, _OPT, _BOOL, None),
                             ("get_preferred_allocation_available", 2, _OPT, _BOOL, None)]),
    ("RegisterRequest", [("version", 1, _OPT, _STR, None),
                         ("endpoint", 2, _OPT, _STR, None),
                         ("resource_name", 3, _OPT, _STR, None),
                         ("options", 4, _OPT, _MSG, "DevicePluginOptions")]),
    ("Empty", []),
    ("ListAndWatchResponse", [("devices", 1, _REP, _MSG, "Device")]),
    ("TopologyInfo", [("nodes", 1, _REP, _MSG, "NUMANode")]),
    ("NUMANode", [("ID", 1, _OPT, _I64, None)]),
    ("Device", [("ID", 1, _OPT, _STR, None),
                ("health", 2, _OPT, _STR, None),
                ("topology", 3, _OPT, _MSG, "TopologyInfo")]),
    ("PreStartContainerRequest", [("devices_ids", 1, _REP, _STR, None)]),
    ("PreStartContainerResponse", []),
    ("PreferredAllocationRequest", [("container_requests", 1, _REP, _MSG,
                                     "ContainerPreferredAllocationRequest")]),
    ("ContainerPreferredAllocationRequest", [("available_deviceIDs", 1, _REP, _STR, None),
                                             ("must_include_deviceIDs", 2, _REP, _STR, None),
                                             ("allocation_size", 3, _OPT, _I32, None)]),
    ("PreferredAllocationResponse", [("container_responses", 1, _REP, _MSG,
                                      "ContainerPreferredAllocationResponse")]),
    ("ContainerPreferredAllocationResponse", [("deviceIDs", 1, _REP, _STR, None)]),
    ("AllocateRequest", [("container_requests", 1, _REP, _MSG, "ContainerAllocateRequest")]),
    ("ContainerAllocateRequest", [("devices_ids", 1, _REP, _STR, None)]),
    ("CDIDevice", [("name", 1, _OPT, _STR, None)]),
    ("AllocateResponse", [("container_responses", 1, _REP, _MSG, "ContainerAllocateResponse")]),
    ("ContainerAllocateResponse", [("envs", 1, _REP, _MSG, "ContainerAllocateResponse.EnvsEntry"),
                                   ("mounts", 2, _REP, _MSG, "Mount"),
                                   ("devices", 3, _REP, _MSG, "DeviceSpec"),
                                   ("annotations", 4, _REP, _MSG,
                                    "ContainerAllocateResponse.AnnotationsEntry"),
                                   ("cdi_devices", 5, _REP, _MSG, "CDIDevice")]),
    ("Mount", [("container_path", 1, _OPT, _STR, None),
               ("host_path", 2, _OPT, _STR, None),
               ("read_only", 3, _OPT, _BOOL, None)]),
    ("DeviceSpec", [("container_path", 1, _OPT, _STR, None),
                    ("host_path", 2, _OPT, _STR, None),
                    ("permissions", 3, _OPT, _STR, None)]),
]

# map<string,string> fields are repeated nested *Entry messages with map_entry=true.
_MAP_ENTRIES = {"ContainerAllocateResponse": ["EnvsEntry", "AnnotationsEntry"]}

# service -> [(method, input, output, server_streaming)]
SERVICES = {
    "Registration": [("Register", "RegisterRequest", "Empty", False)],
    "DevicePlugin": [
        ("GetDevicePluginOptions", "Empty", "DevicePluginOptions", False),
        ("ListAndWatch", "Empty", "ListAndWatchResponse", True),
        ("GetPreferredAllocation", "PreferredAllocationRequest", "PreferredAllocationResponse", False),
        ("Allocate", "AllocateRequest", "AllocateResponse", False),
        ("PreStartContainer", "PreStartContainerRequest", "PreStartContainerResponse", False),
    ],
}


PROTO = _proto.ProtoFile("deviceplugin/v1beta1/api.proto", PACKAGE, _MESSAGES, SERVICES, _MAP_ENTRIES)
FILE_DESCRIPTOR = PROTO.descriptor
_BY_NAME = PROTO.by_name
_CLASSES = {f"{PACKAGE}.{k}": v for k, v in _BY_NAME.items()}

DevicePluginOptions = _CLASSES["v1beta1.DevicePluginOptions"]
RegisterRequest = _CLASSES["v1beta1.RegisterRequest"]
Empty = _CLASSES["v1beta1.Empty"]
ListAndWatchResponse = _CLASSES["v1beta1.ListAndWatchResponse"]
TopologyInfo = _CLASSES["v1beta1.TopologyInfo"]
NUMANode = _CLASSES["v1beta1.NUMANode"]
Device = _CLASSES["v1beta1.Device"]
PreStartContainerRequest = _CLASSES["v1beta1.PreStartContainerRequest"]
PreStartContainerResponse = _CLASSES["v1beta1.PreStartContainerResponse"]
PreferredAllocationRequest = _CLASSES["v1beta1.PreferredAllocationRequest"]
ContainerPreferredAllocationRequest = _CLASSES["v1beta1.ContainerPreferredAllocationRequest"]
PreferredAllocationResponse = _CLASSES["v1beta1.PreferredAllocationResponse"]
ContainerPreferredAllocationResponse = _CLASSES["v1beta1.ContainerPreferredAllocationResponse"]
AllocateRequest = _CLASSES["v1beta1.AllocateRequest"]
ContainerAllocateRequest = _CLASSES["v1beta1.ContainerAllocateRequest"]
CDIDevice = _CLASSES["v1beta1.CDIDevice"]
AllocateResponse = _CLASSES["v1beta1.AllocateResponse"]
ContainerAllocateResponse = _CLASSES["v1beta1.ContainerAllocateResponse"]
Mount = _CLASSES["v1beta1.Mount"]
DeviceSpec = _CLASSES["v1beta1.DeviceSpec"]


def message_class(name: str):
    return _BY_NAME[name]


def method_path(service: str, method: str) -> str:
    """Full gRPC method path, e.g. ``/v1beta1.DevicePlugin/Allocate``."""
    return f"/{PACKAGE}.{service}/{method}"


# ------------------------------------------------------------------------------------------
# grpcio glue
# ------------------------------------------------------------------------------------------

def add_servicer(server, service: str, impl) -> None:
    """Register ``impl`` (an object with one method per RPC) on a ``grpc.Server``.

    Equivalent of the generated ``RegisterDevicePluginServer`` / ``RegisterRegistrationServer``
    (``server.go:125-126``).
    """
    PROTO.add_servicer(server, service, impl)


def Stub(channel, service: str):
    """Client stub for one service over an existing ``grpc.Channel``.

    ``Stub(channel, "DevicePlugin").Allocate(req)`` mirrors the generated Go client.
    """
    return PROTO.stub(channel, service)


unix_target = _proto.unix_target
