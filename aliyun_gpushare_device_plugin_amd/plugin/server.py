"""kubelet ``DevicePlugin`` gRPC server over a Unix socket (component C4).

Reference ``pkg/gpu/nvidia/server.go``: serves on ``/var/lib/kubelet/device-plugins/
aliyungpushare.sock``, self-dials to confirm (5 s), registers ``aliyun.com/gpu-mem`` with the
kubelet, streams the fake-device list in ``ListAndWatch`` and re-sends it on health changes.

Fixed here:
* ``ListAndWatch`` streams read an immutable snapshot and wake on a generation counter, so
  several streams never race on shared ``Device.Health`` (quirk 12) and no health update
  blocks when no stream is attached;
* devices can go back to Healthy (``server.go:188`` FIXME);
* ``GetPreferredAllocation`` is implemented and advertised when enabled (it panicked);
* ``PreStartContainer`` (a no-op there, ``:199-201``) is requested when the kubelet's
  pod-resources API is available: before each container starts, the plugin makes the pod's
  placement annotations match the GPU the container was really given (alloc/placement.py);
* the Allocate RPC is not serialized behind one plugin-wide lock (see alloc/engine.py).
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import threading
import time

import grpc

from .. import const
from ..alloc.engine import AllocationError, Allocator
from ..api import v1beta1 as api
from ..device.model import DeviceModel
from ..utils import log
from ..utils.metrics import PluginMetrics


def dial(socket_path: str, timeout: float = 5.0) -> grpc.Channel:
    """Blocking dial with timeout (``server.go:98-111``)."""
    ch = grpc.insecure_channel(api.unix_target(socket_path))
    try:
        grpc.channel_ready_future(ch).result(timeout=timeout)
    except grpc.FutureTimeoutError:
        ch.close()
        raise TimeoutError(f"timed out dialing {socket_path}")
    return ch


class _Servicer:
    def __init__(self, plugin: "DevicePluginServer"):
        self.p = plugin

    def GetDevicePluginOptions(self, request, context):
        return self.p.options()

    def ListAndWatch(self, request, context):
        p = self.p
        gen = p.model.generation
        yield api.ListAndWatchResponse(devices=p.model.device_list())
        p.metrics.listandwatch_sends.inc()
        while not p.stopped.is_set() and context.is_active():
            new = p.model.wait_change(gen, timeout=0.5)
            if new != gen and not p.stopped.is_set():
                gen = new
                yield api.ListAndWatchResponse(devices=p.model.device_list())
                p.metrics.listandwatch_sends.inc()

    def Allocate(self, request, context):
        t_in = time.monotonic_ns()
        try:
            # message, or prepared wire bytes; follow-up work runs after the reply is sent
            out = self.p.allocator.allocate_raw(request, defer=context.add_callback)
        except AllocationError as e:
            context.abort(grpc.StatusCode.FAILED_PRECONDITION, str(e))
        # handler entry/exit (CLOCK_MONOTONIC, ns) in the trailing metadata: a caller splits its
        # round trip into transport-in, handler and transport-out (bench.py); the kubelet ignores it
        context.set_trailing_metadata(((const.HANDLER_STAMP_KEY, f"{t_in},{time.monotonic_ns()}"),))
        return out

    def GetPreferredAllocation(self, request, context):
        return self.p.allocator.preferred(request)

    def PreStartContainer(self, request, context):
        self.p.allocator.prestart(request)
        return api.PreStartContainerResponse()


class DevicePluginServer:
    def __init__(self, model: DeviceModel, allocator: Allocator, socket_path: str | None = None,
                 resource_name: str = const.RESOURCE_NAME, preferred_allocation: bool = False,
                 metrics: PluginMetrics | None = None, max_workers: int = 16):
        self.model, self.allocator = model, allocator
        self.socket = socket_path or const.plugin_socket()
        self.resource_name = resource_name
        self.preferred_allocation = preferred_allocation
        self.metrics = metrics or allocator.metrics
        self.max_workers = max_workers
        self.server: grpc.Server | None = None
        self.stopped = threading.Event()

    def options(self) -> api.DevicePluginOptions:
        return api.DevicePluginOptions(pre_start_required=self.allocator.podres is not None
                                       or bool(self.allocator.prestart_hooks),
                                       get_preferred_allocation_available=self.preferred_allocation)

    def _cleanup(self):
        try:
            os.remove(self.socket)
        except FileNotFoundError:
            pass

    def start(self):
        self._cleanup()
        os.makedirs(os.path.dirname(self.socket), exist_ok=True)
        self.server = grpc.server(cf.ThreadPoolExecutor(max_workers=self.max_workers,
                                                        thread_name_prefix="dp-rpc"),
                                  options=[("grpc.max_send_message_length", 64 << 20)])
        api.add_servicer(self.server, "DevicePlugin", _Servicer(self))
        port = self.server.add_insecure_port(api.unix_target(self.socket))
        if port == 0:
            raise RuntimeError(f"failed to listen on {self.socket}")
        self.server.start()
        dial(self.socket, 5.0).close()      # confirm the server answers (server.go:130-135)
        log.info("Starting to serve on %s", self.socket)

    def stop(self, grace: float = 0.5):
        self.stopped.set()
        self.model.notify_all()
        if self.server is not None:
            self.server.stop(grace).wait(grace + 1.0)
            self.server = None
        self._cleanup()

    def register(self, kubelet_socket: str | None = None, timeout: float = 5.0):
        ks = kubelet_socket or const.kubelet_socket()
        ch = dial(ks, timeout)
        try:
            stub = api.Stub(ch, "Registration")
            req = api.RegisterRequest(version=api.VERSION, endpoint=os.path.basename(self.socket),
                                      resource_name=self.resource_name)
            opts = self.options()
            if opts.pre_start_required or opts.get_preferred_allocation_available:
                req.options.CopyFrom(opts)     # the kubelet reads the options from Register
            stub.Register(req, timeout=timeout)
        finally:
            ch.close()
        log.info("Registered device plugin for %s with Kubelet", self.resource_name)

    def serve(self, kubelet_socket: str | None = None):
        """``Serve`` (``server.go:232-249``): start, then register; stop on register failure."""
        self.start()
        try:
            self.register(kubelet_socket)
        except Exception:
            self.stop()
            raise


def wait_for_socket(path: str, timeout: float = 10.0) -> bool:
    t = time.monotonic() + timeout
    while time.monotonic() < t:
        if os.path.exists(path):
            return True
        time.sleep(0.01)
    return False
