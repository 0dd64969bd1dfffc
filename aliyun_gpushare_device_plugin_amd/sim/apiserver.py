"""In-memory fake kube-apiserver (test and bench stand-in; SURVEY §4 "fakes to build").

Implements the REST subset the plugin, the extender simulator, the kubelet simulator and
``kubectl-inspect-gpushare`` use, with real HTTP/1.1 keep-alive semantics so client code is
exercised end to end:

* nodes: GET/LIST/POST, PATCH (metadata) and PATCH ``/status`` (strategic merge subset);
* pods: LIST (``fieldSelector`` on ``spec.nodeName``/``status.phase``/``metadata.*``,
  simple ``labelSelector``), GET, POST, PATCH (+``/status``), DELETE, POST ``/binding``;
* WATCH ``/api/v1/pods?watch=1`` as a chunked JSON-lines stream, replaying from
  ``resourceVersion`` (410 Gone when the history window has moved past it) and emitting
  DELETED when an object stops matching the watch's selector (watch-cache semantics);
* optimistic concurrency: a PATCH carrying a stale ``metadata.resourceVersion`` gets 409;
* ``coordination.k8s.io/v1`` Leases: GET, POST, PUT (compare-and-swap on ``resourceVersion``,
  409 on a stale one) — the extender's leader election.

Run standalone: ``python -m aliyun_gpushare_device_plugin_amd.sim.apiserver --port 0``.
"""
from __future__ import annotations

import argparse
import collections
import copy
import json
import queue
import re
import sys
import threading
import time
import urllib.parse
import uuid as uuidlib

from .. import const

_CONFLICT_MSG = const.OPTIMISTIC_LOCK_ERROR_MSG


def strategic_merge(dst, patch):
    """Subset of strategic-merge / JSON-merge patch: maps merge recursively, ``null``
    deletes, lists are replaced."""
    if not isinstance(patch, dict) or not isinstance(dst, dict):
        return copy.deepcopy(patch)
    out = dict(dst)
    for k, v in patch.items():
        if k.startswith("$"):
            continue
        if v is None:
            out.pop(k, None)
        elif isinstance(v, dict) and isinstance(out.get(k), dict):
            out[k] = strategic_merge(out[k], v)
        else:
            out[k] = copy.deepcopy(v)
    return out


def _get_field(obj, path):
    cur = obj
    for p in path.split("."):
        if not isinstance(cur, dict):
            return ""
        cur = cur.get(p)
    return "" if cur is None else str(cur)


def parse_field_selector(sel: str | None):
    reqs = []
    for part in (sel or "").split(","):
        part = part.strip()
        if not part:
            continue
        if "!=" in part:
            k, v = part.split("!=", 1)
            reqs.append((k.strip(), v.strip(), False))
        else:
            k, _, v = part.partition("==" if "==" in part else "=")
            reqs.append((k.strip(), v.strip(), True))
    return reqs


def parse_label_selector(sel: str | None):
    reqs = []
    for part in (sel or "").split(","):
        part = part.strip()
        if not part:
            continue
        if "!=" in part:
            k, v = part.split("!=", 1)
            reqs.append((k.strip(), v.strip(), "ne"))
        elif "=" in part:
            k, _, v = part.partition("==" if "==" in part else "=")
            reqs.append((k.strip(), v.strip(), "eq"))
        else:
            reqs.append((part, None, "exists"))
    return reqs


def matches(obj, fsel, lsel) -> bool:
    for k, v, eq in fsel:
        if (_get_field(obj, k) == v) != eq:
            return False
    labels = (obj.get("metadata") or {}).get("labels") or {}
    for k, v, op in lsel:
        if op == "exists" and k not in labels:
            return False
        if op == "eq" and labels.get(k) != v:
            return False
        if op == "ne" and labels.get(k) == v:
            return False
    return True


class _Watcher:
    """A watch's selectors and its sink: ``push(event)`` when given (the asyncio front end),
    else a thread-safe queue ``q`` (direct Store users)."""

    def __init__(self, fsel, lsel, push=None):
        self.fsel, self.lsel = fsel, lsel
        self.q: "queue.Queue" = queue.Queue()
        self.put = push or self.q.put


class Store:
    def __init__(self, history: int = 20000):
        self.lock = threading.RLock()
        self.rv = 1
        self.pods: dict[tuple, dict] = {}
        self.nodes: dict[str, dict] = {}
        self.leases: dict[tuple, dict] = {}
        self.history: collections.deque = collections.deque(maxlen=history)  # (rv, type, old, new)
        self.watchers: list[_Watcher] = []
        self.requests = collections.Counter()
        # fault injection: kind -> (monotonic deadline, HTTP status). "pod_patch" fails every
        # metadata PATCH of a pod (not the kubelet's /status), "assign_patch" only the plugin's
        # ASSIGNED=true patch
        self.faults: dict[str, tuple[float, int]] = {}
        # bearer-token authentication: None = anonymous allowed; a set = only these tokens
        self.valid_tokens: set | None = None

    def inject(self, kind: str, seconds: float, code: int = 503):
        with self.lock:
            if seconds <= 0:
                self.faults.pop(kind, None)
            else:
                self.faults[kind] = (time.monotonic() + seconds, code)

    def fault(self, kind: str) -> int | None:
        f = self.faults.get(kind)
        if f is None:
            return None
        if time.monotonic() >= f[0]:
            self.faults.pop(kind, None)
            return None
        return f[1]

    def _bump(self, obj):
        self.rv += 1
        obj.setdefault("metadata", {})["resourceVersion"] = str(self.rv)
        return self.rv

    def _notify(self, typ, old, new):
        rv = self.rv
        self.history.append((rv, typ, old, new))
        for w in list(self.watchers):
            self._deliver(w, typ, old, new)

    @staticmethod
    def _deliver(w, typ, old, new):
        was = old is not None and matches(old, w.fsel, w.lsel)
        now = new is not None and matches(new, w.fsel, w.lsel)
        if typ == "DELETED":
            if was:
                w.put({"type": "DELETED", "object": old})
        elif now:
            w.put({"type": "ADDED" if (typ == "ADDED" or not was) else "MODIFIED", "object": new})
        elif was:
            w.put({"type": "DELETED", "object": new})

    # -- pods -----------------------------------------------------------------------------
    def create_pod(self, ns, pod):
        with self.lock:
            pod = copy.deepcopy(pod)
            md = pod.setdefault("metadata", {})
            md["namespace"] = ns
            if not md.get("name"):
                if md.get("generateName"):
                    md["name"] = md["generateName"] + uuidlib.uuid4().hex[:5]
                else:
                    raise KeyError("name required")
            key = (ns, md["name"])
            if key in self.pods:
                return None
            md.setdefault("uid", str(uuidlib.uuid4()))
            md.setdefault("creationTimestamp", time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()))
            pod.setdefault("spec", {})
            st = pod.setdefault("status", {})
            st.setdefault("phase", "Pending")
            self._bump(pod)
            self.pods[key] = pod
            self._notify("ADDED", None, pod)
            return pod

    def patch_pod(self, ns, name, patch, status_only=False):
        with self.lock:
            cur = self.pods.get((ns, name))
            if cur is None:
                return None
            want_rv = ((patch or {}).get("metadata") or {}).get("resourceVersion")
            if want_rv and want_rv != cur["metadata"]["resourceVersion"]:
                raise ValueError("conflict")
            want_uid = ((patch or {}).get("metadata") or {}).get("uid")
            if want_uid and want_uid != cur["metadata"].get("uid"):
                # kube-apiserver: "Precondition failed: UID in precondition: …" (409)
                raise ValueError("uid precondition")
            if status_only:
                patch = {"status": (patch or {}).get("status", {})}
            new = strategic_merge(cur, patch)
            new["metadata"] = dict(new["metadata"])   # never mutate the stored/history version
            new["metadata"]["uid"] = cur["metadata"]["uid"]
            new["metadata"]["name"], new["metadata"]["namespace"] = name, ns
            self._bump(new)
            self.pods[(ns, name)] = new
            self._notify("MODIFIED", cur, new)
            return new

    def delete_pod(self, ns, name):
        with self.lock:
            cur = self.pods.pop((ns, name), None)
            if cur is None:
                return None
            gone = dict(cur)
            gone["metadata"] = dict(cur["metadata"])
            self._bump(gone)
            self._notify("DELETED", gone, None)   # DELETED carries the deletion's resourceVersion
            return gone

    def bind_pod(self, ns, name, node):
        with self.lock:
            cur = self.pods.get((ns, name))
            if cur is None:
                return None
            if (cur.get("spec") or {}).get("nodeName"):
                raise ValueError("already bound")
            conds = list((cur.get("status") or {}).get("conditions") or [])
            conds.append({"type": "PodScheduled", "status": "True"})
            return self.patch_pod(ns, name, {"spec": {"nodeName": node}, "status": {"conditions": conds}})

    def list_pods(self, ns=None, fsel=None, lsel=None):
        with self.lock:
            items = [p for (pns, _), p in self.pods.items()
                     if (ns is None or pns == ns) and matches(p, fsel or [], lsel or [])]
            return items, str(self.rv)

    # -- nodes ----------------------------------------------------------------------------
    def create_node(self, node):
        with self.lock:
            node = copy.deepcopy(node)
            md = node.setdefault("metadata", {})
            if md["name"] in self.nodes:
                return None
            md.setdefault("uid", str(uuidlib.uuid4()))
            node.setdefault("status", {}).setdefault("capacity", {})
            node["status"].setdefault("allocatable", {})
            self._bump(node)
            self.nodes[md["name"]] = node
            return node

    def patch_node(self, name, patch, status_only=False):
        with self.lock:
            cur = self.nodes.get(name)
            if cur is None:
                return None
            if status_only:
                patch = {"status": (patch or {}).get("status", {})}
            else:
                patch = {k: v for k, v in (patch or {}).items() if k != "status"}
            new = strategic_merge(cur, patch)
            new["metadata"] = dict(new["metadata"])
            self._bump(new)
            self.nodes[name] = new
            return new

    # -- leases ---------------------------------------------------------------------------
    def create_lease(self, ns, obj):
        with self.lock:
            obj = copy.deepcopy(obj)
            md = obj.setdefault("metadata", {})
            md["namespace"] = ns
            key = (ns, md.get("name"))
            if key in self.leases:
                return None
            md.setdefault("uid", str(uuidlib.uuid4()))
            self._bump(obj)
            self.leases[key] = obj
            return copy.deepcopy(obj)

    def replace_lease(self, ns, name, obj):
        """PUT: the stored object's ``resourceVersion`` must match the one sent (ValueError)."""
        with self.lock:
            cur = self.leases.get((ns, name))
            if cur is None:
                return None
            if (obj.get("metadata") or {}).get("resourceVersion") != cur["metadata"]["resourceVersion"]:
                raise ValueError("conflict")
            new = copy.deepcopy(obj)
            new["metadata"] = dict(new.get("metadata") or {}, name=name, namespace=ns, uid=cur["metadata"]["uid"])
            self._bump(new)
            self.leases[(ns, name)] = new
            return copy.deepcopy(new)

    # -- watch ----------------------------------------------------------------------------
    def add_watcher(self, fsel, lsel, since_rv, push=None):
        with self.lock:
            w = _Watcher(fsel, lsel, push)
            if since_rv:
                since = int(since_rv)
                if self.history and since < self.history[0][0] - 1 and since < self.rv:
                    return None  # too old
                for rv, typ, old, new in self.history:
                    if rv > since:
                        self._deliver(w, typ, old, new)
            self.watchers.append(w)
            return w

    def remove_watcher(self, w):
        with self.lock:
            if w in self.watchers:
                self.watchers.remove(w)


_POD_RE = re.compile(r"^/api/v1/namespaces/([^/]+)/pods(?:/([^/]+))?(?:/(status|binding))?$")
_NODE_RE = re.compile(r"^/api/v1/nodes(?:/([^/]+))?(?:/(status))?$")
_LEASE_RE = re.compile(r"^/apis/coordination\.k8s\.io/v1/namespaces/([^/]+)/leases(?:/([^/]+))?$")


_REASONS = {200: "OK", 201: "Created", 404: "Not Found", 409: "Conflict", 410: "Gone", 400: "Bad Request",
            405: "Method Not Allowed", 401: "Unauthorized", 503: "Service Unavailable"}


def _status(code, reason, msg):
    return code, {"kind": "Status", "apiVersion": "v1", "status": "Failure", "message": msg, "reason": reason,
                  "code": code}


def _lease_route(store: Store, method: str, m, body: bytes):
    store.requests[f"{method} lease"] += 1
    code = store.fault("lease")
    if code:
        return _status(code, "ServiceUnavailable", "injected fault")
    ns, name = m.group(1), m.group(2)
    if method == "GET" and name:
        with store.lock:
            obj = copy.deepcopy(store.leases.get((ns, name)))
        return (200, obj) if obj else _status(404, "NotFound", f'leases.coordination.k8s.io "{name}" not found')
    obj = json.loads(body) if body else {}
    if method == "POST" and not name:
        made = store.create_lease(ns, obj)
        return (201, made) if made else _status(409, "AlreadyExists", "lease already exists")
    if method == "PUT" and name:
        try:
            new = store.replace_lease(ns, name, obj)
        except ValueError:
            return _status(409, "Conflict", _CONFLICT_MSG)
        return (200, new) if new else _status(404, "NotFound", f'leases.coordination.k8s.io "{name}" not found')
    return _status(405, "MethodNotAllowed", method)


def route(store: Store, method: str, target: str, body: bytes):
    """One REST request against ``store``. Returns ``(code, obj)``, or ``("watch", fsel, lsel, rv,
    timeout)`` for a watch (the caller streams it)."""
    u = urllib.parse.urlsplit(target)
    path = u.path.rstrip("/")
    m = _LEASE_RE.match(path)
    if m:
        return _lease_route(store, method, m, body)
    if method == "GET":
        q = dict(urllib.parse.parse_qsl(u.query)) if u.query else {}
        if path == "/debug/requests":      # simulator introspection: request counts by verb/kind
            with store.lock:
                return 200, dict(store.requests)
        store.requests["GET " + ("watch" if q.get("watch") else path.split("/")[-1])] += 1
        fsel, lsel = parse_field_selector(q.get("fieldSelector")), parse_label_selector(q.get("labelSelector"))
        if path == "/api/v1/pods" or re.fullmatch(r"/api/v1/namespaces/[^/]+/pods", path):
            ns = None if path == "/api/v1/pods" else path.split("/")[4]
            if q.get("watch") in ("1", "true"):
                return "watch", fsel, lsel, q.get("resourceVersion"), float(q.get("timeoutSeconds") or 300)
            items, rv = store.list_pods(ns, fsel, lsel)
            return 200, {"kind": "PodList", "apiVersion": "v1", "metadata": {"resourceVersion": rv}, "items": items}
        m = _POD_RE.match(path)
        if m and m.group(2) and not m.group(3):
            with store.lock:
                p = store.pods.get((m.group(1), m.group(2)))
            return (200, p) if p else _status(404, "NotFound", f'pods "{m.group(2)}" not found')
        m = _NODE_RE.match(path)
        if m:
            with store.lock:
                if m.group(1):
                    n = store.nodes.get(m.group(1))
                    return (200, n) if n else _status(404, "NotFound", f'nodes "{m.group(1)}" not found')
                items = [n for n in store.nodes.values() if matches(n, fsel, lsel)]
            return 200, {"kind": "NodeList", "apiVersion": "v1", "metadata": {"resourceVersion": str(store.rv)},
                         "items": items}
        return _status(404, "NotFound", path)
    obj = json.loads(body) if body else {}
    if method == "POST":
        if path == "/debug/faults":        # simulator fault injection: {"kind", "seconds", "code"}
            store.inject(obj["kind"], float(obj.get("seconds", 0)), int(obj.get("code", 503)))
            return 200, {"faults": {k: v[1] for k, v in store.faults.items()}}
        store.requests["POST " + path.split("/")[-1]] += 1
        m = _POD_RE.match(path)
        if m and not m.group(2):
            p = store.create_pod(m.group(1), obj)
            return (201, p) if p else _status(409, "AlreadyExists", "pod already exists")
        if m and m.group(3) == "binding":
            try:
                p = store.bind_pod(m.group(1), m.group(2), obj["target"]["name"])
            except ValueError:
                return _status(409, "Conflict", "pod is already assigned to a node")
            return (201, {"kind": "Status", "status": "Success"}) if p else _status(404, "NotFound", "pod not found")
        if path == "/api/v1/nodes":
            n = store.create_node(obj)
            return (201, n) if n else _status(409, "AlreadyExists", "node already exists")
        return _status(404, "NotFound", path)
    if method == "PATCH":
        store.requests["PATCH " + ("status" if path.endswith("/status") else path.split("/")[3])] += 1
        m = _POD_RE.match(path)
        if m and m.group(2) and not m.group(3):
            assigning = ((obj.get("metadata") or {}).get("annotations") or {}).get(const.ENV_ASSIGNED_FLAG) == "true"
            code = store.fault("pod_patch") or (store.fault("assign_patch") if assigning else None)
            if code:
                store.requests["PATCH dropped"] += 1
                return _status(code, "ServiceUnavailable", "injected fault")
        if m and m.group(2):
            try:
                p = store.patch_pod(m.group(1), m.group(2), obj, status_only=m.group(3) == "status")
            except ValueError:
                return _status(409, "Conflict", _CONFLICT_MSG)
            return (200, p) if p else _status(404, "NotFound", f'pods "{m.group(2)}" not found')
        m = _NODE_RE.match(path)
        if m and m.group(1):
            n = store.patch_node(m.group(1), obj, status_only=m.group(2) == "status")
            return (200, n) if n else _status(404, "NotFound", f'nodes "{m.group(1)}" not found')
        return _status(404, "NotFound", path)
    if method == "DELETE":
        store.requests["DELETE"] += 1
        m = _POD_RE.match(path)
        if m and m.group(2):
            p = store.delete_pod(m.group(1), m.group(2))
            return (200, p) if p else _status(404, "NotFound", "pod not found")
        return _status(404, "NotFound", path)
    return _status(405, "MethodNotAllowed", method)


def _response(code: int, obj) -> bytes:
    body = json.dumps(obj, separators=(",", ":")).encode()
    return (b"HTTP/1.1 %d %s\r\nServer: fake-apiserver/2\r\nContent-Type: application/json\r\n"
            b"Content-Length: %d\r\n\r\n" % (code, _REASONS.get(code, "Error").encode(), len(body))) + body


class FakeAPIServer:
    """HTTP/1.1 front end on one asyncio event loop (its own thread, or the caller's with
    ``serve_forever``): keep-alive request/response, chunked watch streams. Every request is
    handled inline on the loop — no thread per connection, no ``http.server`` parsing — which
    keeps the fake's per-request cost well below the plugin's (the N=8 bench churns ~50 requests
    per step through it)."""

    def __init__(self, host: str = "127.0.0.1", port: int = 0, latency_s: float = 0.0, store: Store | None = None):
        import asyncio
        import socket

        self.store = store or Store()
        self.latency_s = latency_s
        self.stopping = threading.Event()
        self._sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self._sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self._sock.bind((host, port))
        self._sock.listen(256)
        self.loop = asyncio.new_event_loop()
        self.thread = None
        self._server = None

    @property
    def url(self) -> str:
        h, p = self._sock.getsockname()[:2]
        return f"http://{h}:{p}"

    # -- connection handling ------------------------------------------------------------------
    async def _conn(self, reader, writer):
        import asyncio
        import socket

        sock = writer.get_extra_info("socket")
        if sock is not None:
            sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        try:
            while not self.stopping.is_set():
                try:
                    head = await reader.readuntil(b"\r\n\r\n")
                except (asyncio.IncompleteReadError, asyncio.LimitOverrunError, ConnectionError):
                    return
                lines = head.split(b"\r\n")
                try:
                    method, target, _ = lines[0].decode("latin-1").split(" ", 2)
                except ValueError:
                    return
                n = 0
                token = None
                for ln in lines[1:]:
                    low = ln[:22].lower()
                    if low[:15] == b"content-length:":
                        n = int(ln[15:].strip() or 0)
                    elif low[:21] == b"authorization: bearer":
                        token = ln[21:].strip().decode("latin-1")
                body = await reader.readexactly(n) if n else b""
                if self.latency_s > 0:
                    # injected network RTT: a thread sleep is accurate to ~0.1 ms, where the event
                    # loop's own timers round up to epoll's 1 ms granularity (+~1 ms per request)
                    await asyncio.get_running_loop().run_in_executor(None, time.sleep, self.latency_s)
                valid = self.store.valid_tokens
                if valid is not None and token not in valid:
                    self.store.requests["401"] += 1
                    writer.write(_response(*_status(401, "Unauthorized", "Unauthorized")))
                    continue
                try:
                    res = route(self.store, method, target, body)
                except Exception as e:  # noqa: BLE001 - a malformed request must not kill the fake
                    res = _status(400, "BadRequest", repr(e))
                if res[0] == "watch":
                    await self._watch(writer, *res[1:])
                    return
                writer.write(_response(*res))
                if writer.transport.get_write_buffer_size() > 1 << 20:
                    await writer.drain()
        finally:
            writer.close()

    async def _watch(self, writer, fsel, lsel, rv, timeout):
        import asyncio

        loop = asyncio.get_running_loop()
        aq: asyncio.Queue = asyncio.Queue()
        loop_tid = threading.get_ident()

        def push(ev):   # called under the store lock, from the loop thread or a direct Store user
            if threading.get_ident() == loop_tid:
                aq.put_nowait(ev)
            else:
                loop.call_soon_threadsafe(aq.put_nowait, ev)

        w = self.store.add_watcher(fsel, lsel, rv, push=push)
        if w is None:
            writer.write(_response(*_status(410, "Expired", "too old resource version")))
            return
        writer.write(b"HTTP/1.1 200 OK\r\nContent-Type: application/json\r\nTransfer-Encoding: chunked\r\n\r\n")
        deadline = loop.time() + timeout
        try:
            while not self.stopping.is_set():
                left = deadline - loop.time()
                if left <= 0:
                    break
                try:
                    ev = await asyncio.wait_for(aq.get(), min(left, 0.5))
                except asyncio.TimeoutError:
                    continue
                evs = [ev]
                while not aq.empty():
                    evs.append(aq.get_nowait())
                data = b"".join(json.dumps(e, separators=(",", ":")).encode() + b"\n" for e in evs)
                writer.write(b"%x\r\n%s\r\n" % (len(data), data))
                await writer.drain()
        except (ConnectionError, OSError):
            return
        finally:
            self.store.remove_watcher(w)
            if not writer.is_closing():   # end the chunked stream (also on shutdown/cancel)
                writer.write(b"0\r\n\r\n")

    # -- lifecycle ---------------------------------------------------------------------------------
    async def _start_server(self):
        import asyncio

        self._server = await asyncio.start_server(self._conn, sock=self._sock, limit=1 << 22)

    def serve_forever(self):
        import asyncio

        asyncio.set_event_loop(self.loop)
        self.loop.run_until_complete(self._start_server())
        try:
            self.loop.run_forever()
        finally:   # cancel the connection / watch tasks and let them unwind before closing
            if self._server is not None:
                self._server.close()
            tasks = [t for t in asyncio.all_tasks(self.loop) if not t.done()]
            for t in tasks:
                t.cancel()
            if tasks:
                self.loop.run_until_complete(asyncio.gather(*tasks, return_exceptions=True))
            self.loop.run_until_complete(self.loop.shutdown_asyncgens())
            self.loop.close()

    def start(self):
        self.thread = threading.Thread(target=self.serve_forever, name="fake-apiserver", daemon=True)
        self.thread.start()
        import time as _t

        t_end = _t.monotonic() + 10
        while self._server is None and _t.monotonic() < t_end:
            _t.sleep(0.001)
        return self

    def stop(self):
        self.stopping.set()

        if self.loop.is_running():
            try:
                self.loop.call_soon_threadsafe(self.loop.stop)
            except RuntimeError:   # loop already closed
                pass
        if self.thread is not None:
            self.thread.join(timeout=5)
        try:
            self._sock.close()
        except OSError:
            pass

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()


def make_node(name: str, labels: dict | None = None, ip: str = "10.0.0.1") -> dict:
    return {"apiVersion": "v1", "kind": "Node",
            "metadata": {"name": name, "labels": dict(labels or {"gpushare": "true"})},
            "status": {"capacity": {"cpu": "128", "memory": "1536Gi"},
                       "allocatable": {"cpu": "128", "memory": "1536Gi"},
                       "addresses": [{"type": "InternalIP", "address": ip}, {"type": "Hostname", "address": name}]}}


def main(argv=None):
    ap = argparse.ArgumentParser(description="fake kube-apiserver")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--latency-ms", type=float, default=0.0)
    a = ap.parse_args(argv)
    s = FakeAPIServer(a.host, a.port, a.latency_ms / 1000.0)
    print(s.url, flush=True)
    try:
        s.serve_forever()
    except KeyboardInterrupt:
        pass
    return 0


if __name__ == "__main__":
    sys.exit(main())
