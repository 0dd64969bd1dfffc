"""Runtime ``.proto`` → message classes + grpcio service glue (no protoc gRPC plugin offline).

A kubelet API file is described as plain tables — messages with (name, number, label, type,
type name) fields, map entries, and services — turned into a ``FileDescriptorProto`` at import
time. Message classes come from protobuf's message factory; services are wired with grpcio
generic handlers, so method paths and bytes on the wire are those of the upstream ``.proto``.
Used by ``api/v1beta1.py`` (device plugin) and ``api/podresources.py`` (pod-resources v1).
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

F = descriptor_pb2.FieldDescriptorProto
OPT, REP = F.LABEL_OPTIONAL, F.LABEL_REPEATED
STR, BOOL, I64, U64, I32, MSG = (F.TYPE_STRING, F.TYPE_BOOL, F.TYPE_INT64, F.TYPE_UINT64, F.TYPE_INT32,
                                 F.TYPE_MESSAGE)


class ProtoFile:
    """One ``.proto`` file: ``messages`` = [(name, [(field, number, label, type, type_name)])],
    ``map_entries`` = {message: [EntryName]} (string→string maps), ``services`` =
    {service: [(method, input, output, server_streaming)]}."""

    def __init__(self, file_name: str, package: str, messages, services, map_entries=None):
        self.package, self.services = package, services
        fdp = descriptor_pb2.FileDescriptorProto(name=file_name, package=package, syntax="proto3")
        for name, fields in messages:
            m = fdp.message_type.add(name=name)
            for entry in (map_entries or {}).get(name, []):
                e = m.nested_type.add(name=entry)
                e.options.map_entry = True
                e.field.add(name="key", number=1, label=OPT, type=STR, json_name="key")
                e.field.add(name="value", number=2, label=OPT, type=STR, json_name="value")
            for fname, num, label, ftype, tname in fields:
                f = m.field.add(name=fname, number=num, label=label, type=ftype)
                if tname:
                    f.type_name = f".{package}.{tname}"
        for svc, methods in services.items():
            s = fdp.service.add(name=svc)
            for meth, inp, out, stream in methods:
                s.method.add(name=meth, input_type=f".{package}.{inp}", output_type=f".{package}.{out}",
                             server_streaming=stream)
        pool = descriptor_pool.DescriptorPool()
        classes = message_factory.GetMessages([fdp], pool=pool)
        self.descriptor = pool.FindFileByName(file_name)
        self.by_name = {k.split(".", 1)[1]: v for k, v in classes.items() if k.count(".") == 1}

    def __getitem__(self, name: str):
        return self.by_name[name]

    def method_path(self, service: str, method: str) -> str:
        return f"/{self.package}.{service}/{method}"

    def add_servicer(self, server, service: str, impl) -> None:
        """Register ``impl`` (one method per RPC) on a ``grpc.Server`` — the generated
        ``Register<Service>Server`` equivalent."""
        import grpc

        handlers = {}
        for meth, inp, out, stream in self.services[service]:
            fn = getattr(impl, meth)
            factory = grpc.unary_stream_rpc_method_handler if stream else grpc.unary_unary_rpc_method_handler
            handlers[meth] = factory(fn, request_deserializer=self.by_name[inp].FromString,
                                     response_serializer=_serializer(self.by_name[out]))
        server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(f"{self.package}.{service}",
                                                                              handlers),))

    def stub(self, channel, service: str):
        """Client stub over an existing ``grpc.Channel`` (generated Go client equivalent)."""
        return _Stub(self, channel, service)


def _serializer(cls):
    """A handler may return the message or its wire bytes already serialized (the Allocate
    fast path answers with bytes prepared before the request arrived)."""
    ser = cls.SerializeToString

    def f(r):
        return r if isinstance(r, bytes) else ser(r)
    return f


class _Stub:
    def __init__(self, pf: ProtoFile, channel, service: str):
        for meth, inp, out, stream in pf.services[service]:
            make = channel.unary_stream if stream else channel.unary_unary
            setattr(self, meth, make(pf.method_path(service, meth),
                                     request_serializer=pf.by_name[inp].SerializeToString,
                                     response_deserializer=pf.by_name[out].FromString))


def unix_target(path: str) -> str:
    return "unix://" + path if not path.startswith("unix:") else path
