"""Fake kubelet device manager (test and bench stand-in).

Plays the kubelet's side of the device-plugin API over real gRPC-on-UDS:
* serves ``v1beta1.Registration`` on ``<dir>/kubelet.sock``;
* on ``Register`` dials the plugin's endpoint, reads ``GetDevicePluginOptions`` and keeps a
  ``ListAndWatch`` stream, mirroring the advertised healthy-device count into the node's
  ``aliyun.com/gpu-mem`` capacity/allocatable (what the real kubelet reports);
* ``admit(pod)`` does what pod admission does: for each container with a ``gpu-mem`` limit,
  pick that many free healthy fake IDs (asking ``GetPreferredAllocation`` when offered),
  call ``Allocate`` once per container, and remember the IDs until ``release``;
* ``restart()`` re-creates ``kubelet.sock`` like a kubelet restart (the plugin must notice
  and re-register, ``gpumanager.go:82-87``);
* serves the pod-resources API (``v1.PodResourcesLister``) on ``<dir>/pod-resources.sock``:
  every admitted pod's containers with the fake IDs checkpointed for them, exactly what the
  real kubelet publishes on ``/var/lib/kubelet/pod-resources/kubelet.sock``;
* when the plugin registered with ``pre_start_required``, calls ``PreStartContainer`` for each
  gpu container after the pod's admission, before "starting" it.
"""
from __future__ import annotations

import concurrent.futures as cf
import dataclasses
import os
import threading
import time

import grpc

from .. import const
from ..api import podresources as podres
from ..api import v1beta1 as api
from ..cluster import objects as O
from ..cluster.client import APIClient
from ..utils import log
from .h2client import NativeUnaryClient, UnaryError

_STATUS = {s.value[0]: s for s in grpc.StatusCode}


@dataclasses.dataclass
class Admission:
    pod_uid: str
    responses: list          # ContainerAllocateResponse per gpu container
    latencies: list          # seconds per Allocate RPC
    device_ids: list
    error: str | None = None
    # per Allocate RPC: (kubelet -> handler entry, handler, handler exit -> kubelet) seconds,
    # from the handler's own timestamps in the reply's trailing metadata (one system-wide
    # CLOCK_MONOTONIC for both processes)
    splits: list = dataclasses.field(default_factory=list)


class FakeKubelet:
    def __init__(self, plugin_dir: str, client: APIClient | None = None, node: str | None = None,
                 resource: str = const.RESOURCE_NAME):
        self.dir, self.client, self.node, self.resource = plugin_dir, client, node, resource
        os.makedirs(plugin_dir, exist_ok=True)
        self.sock = os.path.join(plugin_dir, const.KUBELET_SOCKET_NAME)
        self.server = None
        self.registrations: list = []
        self.registered = threading.Event()
        self.devices: dict[str, str] = {}
        self.devices_updated = threading.Condition()
        self.list_updates = 0
        self.options = None
        self._channel = None
        self._stub = None
        self._law_thread = None
        self._allocated: dict[str, set] = {}
        self._used: set = set()                 # union of _allocated, kept incrementally
        self._healthy: list[str] = []           # healthy IDs in advertised order, per device update
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._holdings: dict[str, tuple] = {}    # uid -> (ns, name, [(container, ids)])
        self._specs: dict[str, list] = {}        # uid -> container names (all listed, like the kubelet)
        self.podres_sock = os.path.join(plugin_dir, "pod-resources.sock")
        self._h2 = None                           # NativeUnaryClient for Allocate (see _connect)
        self._watch = None                        # this node's pods, as the kubelet's own watch sees them
        self.prestart_calls = 0
        self.reg_options = None

    # -- read-only /pods endpoint (--pod-source=kubelet / --query-kubelet) ------------------
    def serve_pods(self, token: str = "sim-kubelet-token") -> int:
        """The kubelet's ``GET /pods/`` (``client.go:119-134``): this node's pods as a PodList,
        bearer-token checked. Plain HTTP on 127.0.0.1 (``--kubelet-scheme http``). Returns the port."""
        import http.server
        import json as _json

        kl = self

        class H(http.server.BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def log_message(self, *a):
                pass

            def do_GET(self):
                if self.headers.get("Authorization") != f"Bearer {kl.pods_token}":   # rotatable
                    code, body = 401, b'{"message":"Unauthorized"}'
                elif self.path.rstrip("/") != "/pods":
                    code, body = 404, b"{}"
                else:
                    items, _ = kl.client.list_pods(field_selector=f"spec.nodeName={kl.node}")
                    code, body = 200, _json.dumps({"kind": "PodList", "apiVersion": "v1", "items": items}).encode()
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

        self.pods_token = token
        self._pods_srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
        self._pods_srv.daemon_threads = True
        threading.Thread(target=self._pods_srv.serve_forever, name="kubelet-pods", daemon=True).start()
        self.pods_port = self._pods_srv.server_address[1]
        return self.pods_port

    # -- Registration service -------------------------------------------------------------
    # -- pod-resources service (v1.PodResourcesLister) ----------------------------------
    def _pod_resources(self, uid_filter=None) -> list:
        with self._lock:
            items = list(self._holdings.items())
            specs = dict(self._specs)
        out = []
        for uid, (ns, name, ctrs) in items:
            if uid_filter is not None and not uid_filter(ns, name):
                continue
            got = dict(ctrs)
            names = specs.get(uid) or [cn for cn, _ in ctrs]
            out.append(podres.PodResources(name=name, namespace=ns, containers=[
                podres.ContainerResources(name=cn, devices=[
                    podres.ContainerDevices(resource_name=self.resource, device_ids=[i]) for i in got.get(cn, ())])
                for cn in names]))
        return out

    def List(self, request, context):
        return podres.ListPodResourcesResponse(pod_resources=self._pod_resources())

    def Get(self, request, context):
        got = self._pod_resources(lambda ns, n: (ns, n) == (request.pod_namespace, request.pod_name))
        if not got:
            context.abort(grpc.StatusCode.NOT_FOUND, "pod not found")
        return podres.GetPodResourcesResponse(pod_resources=got[0])

    def GetAllocatableResources(self, request, context):
        with self.devices_updated:
            healthy = list(self._healthy)
        return podres.AllocatableResourcesResponse(devices=[
            podres.ContainerDevices(resource_name=self.resource, device_ids=[i]) for i in healthy])

    def Register(self, request, context):
        self.registrations.append((request.version, request.endpoint, request.resource_name))
        self.reg_options = request.options if request.HasField("options") else None
        if request.version != api.VERSION:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, f"unsupported version {request.version}")
        threading.Thread(target=self._connect, args=(request.endpoint,), daemon=True).start()
        return api.Empty()

    def start(self):
        self._stop.clear()
        try:
            os.remove(self.sock)
        except FileNotFoundError:
            pass
        try:
            os.remove(self.podres_sock)
        except FileNotFoundError:
            pass
        self.server = grpc.server(cf.ThreadPoolExecutor(max_workers=4, thread_name_prefix="kubelet"))
        api.add_servicer(self.server, "Registration", self)
        podres.PROTO.add_servicer(self.server, "PodResourcesLister", self)
        self.server.add_insecure_port(api.unix_target(self.sock))
        self.server.add_insecure_port(api.unix_target(self.podres_sock))
        self.server.start()
        if self.client is not None and self.node and self._watch is None:
            from ..cluster.podcache import WatchCache

            self._watch = WatchCache(self.client, self.node).start()
        return self

    def stop(self):
        self._stop.set()
        if self._watch is not None:
            self._watch.stop()
            self._watch = None
        if self.server is not None:
            self.server.stop(0.2).wait(1.0)
            self.server = None
        if self._channel is not None:
            self._channel.close()
            self._channel = None
        if self._h2 is not None:
            self._h2.close()
            self._h2 = None

    def restart(self):
        self.stop()
        self.registered.clear()
        self.start()

    # -- plugin connection ----------------------------------------------------------------
    def _connect(self, endpoint: str):
        path = os.path.join(self.dir, endpoint)
        if self._channel is not None:
            self._channel.close()
        ch = grpc.insecure_channel(api.unix_target(path))
        grpc.channel_ready_future(ch).result(timeout=5)
        self._channel = ch
        self._stub = api.Stub(ch, "DevicePlugin")
        self.options = self._stub.GetDevicePluginOptions(api.Empty(), timeout=5)
        if self._h2 is not None:
            self._h2.close()
            self._h2 = None
        if NativeUnaryClient.wanted():
            # Allocate the way the real kubelet calls it: compiled client code (sim/h2client.py)
            self._h2 = NativeUnaryClient(path)
        self._law_thread = threading.Thread(target=self._list_and_watch, args=(self._stub,), daemon=True)
        self._law_thread.start()

    def _list_and_watch(self, stub):
        try:
            for resp in stub.ListAndWatch(api.Empty()):
                devs = {d.ID: d.health for d in resp.devices}
                healthy = [d for d, h in devs.items() if h == const.HEALTHY]
                with self.devices_updated:
                    self.devices = devs
                    self._healthy = healthy
                    self.list_updates += 1
                    self.devices_updated.notify_all()
                self.registered.set()
                self._report_capacity()
                if self._stop.is_set():
                    break
        except grpc.RpcError as e:
            if not self._stop.is_set():
                log.V(2).info("fake kubelet ListAndWatch ended: %s", e.code())

    def _report_capacity(self):
        if self.client is None or not self.node:
            return
        healthy = sum(1 for h in self.devices.values() if h == const.HEALTHY)
        total = len(self.devices)
        try:
            self.client.patch_node_status(self.node, {"status": {"capacity": {self.resource: str(total)},
                                                                 "allocatable": {self.resource: str(healthy)}}})
        except Exception as e:  # noqa: BLE001
            log.warning("fake kubelet capacity report failed: %s", e)

    def wait_devices(self, pred, timeout: float = 10.0) -> bool:
        t = time.monotonic() + timeout
        with self.devices_updated:
            while not pred(self.devices):
                left = t - time.monotonic()
                if left <= 0:
                    return False
                self.devices_updated.wait(left)
        return True

    # -- device manager -------------------------------------------------------------------
    def _free_healthy(self) -> list[str]:
        used = self._used
        return [d for d in self._healthy if d not in used]

    def _await_watch(self, uid: str, limit: float = 2.0) -> None:
        """The kubelet admits a pod its own apiserver watch delivered (bound to this node) —
        the event the plugin's informer reads too; a harness handing it the bind response
        directly would always outrun the plugin's cache."""
        w = self._watch
        if w is None or not w.wait_synced(limit):
            return
        t = time.monotonic() + limit
        while time.monotonic() < t:
            if w.get(uid) is not None:
                return
            time.sleep(0.0002)

    def admit(self, pod: dict, timeout: float = 10.0) -> Admission:
        uid = O.uid(pod)
        self._await_watch(uid)
        adm = Admission(uid, [], [], [])
        started = []
        # like the kubelet's HandlePodAdditions: the pod joins the pod manager (and so the
        # pod-resources List, holding nothing yet) right before it is admitted
        with self._lock:
            self._holdings[uid] = (O.namespace(pod), O.name(pod), [])
            self._specs[uid] = [c.get("name", "") for c in O.containers(pod)]
        for c in O.containers(pod):
            n = O.container_limit(c, self.resource)
            if n <= 0:
                continue
            with self._lock:
                free = self._free_healthy()
                if len(free) < n:
                    adm.error = f"insufficient {self.resource}: want {n}, free {len(free)}"
                    self._holdings.pop(uid, None)      # rejected: no longer an active pod
                    self._specs.pop(uid, None)
                    self._used.difference_update(self._allocated.pop(uid, ()))
                    return adm
                ids = free[:n]
                if self.options is not None and self.options.get_preferred_allocation_available:
                    pr = self._stub.GetPreferredAllocation(api.PreferredAllocationRequest(container_requests=[
                        api.ContainerPreferredAllocationRequest(available_deviceIDs=free, allocation_size=n)]),
                        timeout=timeout)
                    pref = list(pr.container_responses[0].deviceIDs) if pr.container_responses else []
                    if len(pref) == n and set(pref) <= set(free):
                        ids = pref
                self._allocated.setdefault(uid, set()).update(ids)
                self._used.update(ids)
            areq = api.AllocateRequest(container_requests=[api.ContainerAllocateRequest(devices_ids=ids)])
            h2 = self._h2
            if h2 is not None:
                try:
                    raw, stamp, t0n, t1n = h2.unary("/v1beta1.DevicePlugin/Allocate", areq.SerializeToString(),
                                                    timeout)
                except UnaryError as e:
                    adm.error = f"Allocate failed: {_STATUS.get(e.status, e.status)} {e.message}"
                    self.release(uid)
                    return adm
                except ConnectionError as e:
                    adm.error = f"Allocate failed: {e}"
                    self.release(uid)
                    return adm
                resp = api.AllocateResponse.FromString(raw)
                adm.latencies.append((t1n - t0n) / 1e9)
            else:
                t0n = time.monotonic_ns()
                t0 = time.perf_counter()
                try:
                    resp, call = self._stub.Allocate.with_call(areq, timeout=timeout)
                except grpc.RpcError as e:
                    adm.latencies.append(time.perf_counter() - t0)
                    adm.error = f"Allocate failed: {e.code()} {e.details()}"
                    self.release(uid)
                    return adm
                adm.latencies.append(time.perf_counter() - t0)
                t1n = time.monotonic_ns()
                stamp = dict(call.trailing_metadata() or ()).get(const.HANDLER_STAMP_KEY)
            if stamp:
                a, b = (int(x) for x in stamp.split(","))
                adm.splits.append(((a - t0n) / 1e9, (b - a) / 1e9, (t1n - b) / 1e9))
            adm.responses.append(resp.container_responses[0])
            adm.device_ids.append(ids)
            # the device manager checkpoints the container's IDs (pod-resources shows them)
            started.append((c.get("name", ""), tuple(ids)))
            with self._lock:
                self._holdings[uid] = (O.namespace(pod), O.name(pod), list(started))
        if self._pre_start_required():
            for _, ids in started:     # container start: PreStartContainer per gpu container
                self.prestart_calls += 1
                try:
                    self._stub.PreStartContainer(api.PreStartContainerRequest(devices_ids=list(ids)),
                                                 timeout=timeout)
                except grpc.RpcError as e:
                    adm.error = f"PreStartContainer failed: {e.code()} {e.details()}"
        return adm

    def _pre_start_required(self) -> bool:
        o = self.reg_options if self.reg_options is not None else self.options
        return bool(o is not None and o.pre_start_required)

    def release(self, pod_uid: str):
        with self._lock:
            self._used.difference_update(self._allocated.pop(pod_uid, ()))
            self._holdings.pop(pod_uid, None)
            self._specs.pop(pod_uid, None)

    def allocated_ids(self) -> set:
        with self._lock:
            return set(self._used)
