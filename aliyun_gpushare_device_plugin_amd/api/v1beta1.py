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

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

PACKAGE = "v1beta1"
VERSION = "v1beta1"

_F = descriptor_pb2.FieldDescriptorProto
_OPT, _REP = _F.LABEL_OPTIONAL, _F.LABEL_REPEATED
_STR, _BOOL, _I64, _I32, _MSG = _F.TYPE_STRING, _F.TYPE_BOOL, _F.TYPE_INT64, _F.TYPE_INT32, _F.TYPE_MESSAGE

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


def _build_file() -> descriptor_pb2.FileDescriptorProto:
    fdp = descriptor_pb2.FileDescriptorProto(name="deviceplugin/v1beta1/api.proto",
                                             package=PACKAGE, syntax="proto3")
    for name, fields in _MESSAGES:
        m = fdp.message_type.add(name=name)
        for entry in _MAP_ENTRIES.get(name, []):
            e = m.nested_type.add(name=entry)
            e.options.map_entry = True
            e.field.add(name="key", number=1, label=_OPT, type=_STR, json_name="key")
            e.field.add(name="value", number=2, label=_OPT, type=_STR, json_name="value")
        for fname, num, label, ftype, tname in fields:
            f = m.field.add(name=fname, number=num, label=label, type=ftype)
            if tname:
                f.type_name = f".{PACKAGE}.{tname}"
    for svc, methods in SERVICES.items():
        s = fdp.service.add(name=svc)
        for meth, inp, out, stream in methods:
            s.method.add(name=meth, input_type=f".{PACKAGE}.{inp}", output_type=f".{PACKAGE}.{out}",
                         server_streaming=stream)
    return fdp


_POOL = descriptor_pool.DescriptorPool()
_CLASSES = message_factory.GetMessages([_build_file()], pool=_POOL)
FILE_DESCRIPTOR = _POOL.FindFileByName("deviceplugin/v1beta1/api.proto")

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

_BY_NAME = {k.split(".", 1)[1]: v for k, v in _CLASSES.items() if k.count(".") == 1}


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
    import grpc

    handlers = {}
    for meth, inp, out, stream in SERVICES[service]:
        fn = getattr(impl, meth)
        req_cls, resp_cls = _BY_NAME[inp], _BY_NAME[out]
        factory = grpc.unary_stream_rpc_method_handler if stream else grpc.unary_unary_rpc_method_handler
        handlers[meth] = factory(fn, request_deserializer=req_cls.FromString,
                                 response_serializer=resp_cls.SerializeToString)
    server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(f"{PACKAGE}.{service}", handlers),))


class Stub:
    """Client stub for one service over an existing ``grpc.Channel``.

    ``Stub(channel, "DevicePlugin").Allocate(req)`` mirrors the generated Go client.
    """

    def __init__(self, channel, service: str):
        for meth, inp, out, stream in SERVICES[service]:
            make = channel.unary_stream if stream else channel.unary_unary
            setattr(self, meth, make(method_path(service, meth),
                                     request_serializer=_BY_NAME[inp].SerializeToString,
                                     response_deserializer=_BY_NAME[out].FromString))


def unix_target(path: str) -> str:
    return "unix://" + path if not path.startswith("unix:") else path
