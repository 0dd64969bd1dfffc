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
* optimistic concurrency: a PATCH carrying a stale ``metadata.resourceVersion`` gets 409.

Run standalone: ``python -m aliyun_gpushare_device_plugin_amd.sim.apiserver --port 0``.
"""
from __future__ import annotations

import argparse
import collections
import copy
import http.server
import json
import queue
import re
import socketserver
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
    def __init__(self, fsel, lsel):
        self.fsel, self.lsel = fsel, lsel
        self.q: "queue.Queue" = queue.Queue()


class Store:
    def __init__(self, history: int = 20000):
        self.lock = threading.RLock()
        self.rv = 1
        self.pods: dict[tuple, dict] = {}
        self.nodes: dict[str, dict] = {}
        self.history: collections.deque = collections.deque(maxlen=history)  # (rv, type, old, new)
        self.watchers: list[_Watcher] = []
        self.requests = collections.Counter()

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
                w.q.put({"type": "DELETED", "object": old})
        elif now:
            w.q.put({"type": "ADDED" if (typ == "ADDED" or not was) else "MODIFIED", "object": new})
        elif was:
            w.q.put({"type": "DELETED", "object": new})

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

    # -- watch ----------------------------------------------------------------------------
    def add_watcher(self, fsel, lsel, since_rv):
        with self.lock:
            w = _Watcher(fsel, lsel)
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


class _Handler(http.server.BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"
    server_version = "fake-apiserver/1"
    disable_nagle_algorithm = True   # header and body leave in one segment, no delayed-ACK stall

    def log_message(self, *a):
        pass

    @property
    def store(self) -> Store:
        return self.server.store

    def _send(self, code, obj):
        body = json.dumps(obj, separators=(",", ":")).encode()
        self.send_response(code)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(body)))
        self._headers_buffer.append(b"\r\n" + body)   # one write for headers + body
        self.flush_headers()

    def _status(self, code, reason, msg):
        self._send(code, {"kind": "Status", "apiVersion": "v1", "status": "Failure", "message": msg,
                          "reason": reason, "code": code})

    def _body(self):
        n = int(self.headers.get("Content-Length") or 0)
        return json.loads(self.rfile.read(n)) if n else {}

    def _delay(self):
        d = self.server.latency_s
        if d > 0:
            time.sleep(d)

    def do_GET(self):
        self._delay()
        u = urllib.parse.urlsplit(self.path)
        q = dict(urllib.parse.parse_qsl(u.query))
        path = u.path.rstrip("/")
        if path == "/debug/requests":      # simulator introspection: request counts by verb/kind
            with self.store.lock:
                return self._send(200, dict(self.store.requests))
        self.store.requests["GET " + ("watch" if q.get("watch") else path.split("/")[-1])] += 1
        fsel, lsel = parse_field_selector(q.get("fieldSelector")), parse_label_selector(q.get("labelSelector"))
        if path == "/api/v1/pods" or re.fullmatch(r"/api/v1/namespaces/[^/]+/pods", path):
            ns = None if path == "/api/v1/pods" else path.split("/")[4]
            if q.get("watch") in ("1", "true"):
                return self._watch(fsel, lsel, q.get("resourceVersion"), float(q.get("timeoutSeconds") or 300))
            items, rv = self.store.list_pods(ns, fsel, lsel)
            return self._send(200, {"kind": "PodList", "apiVersion": "v1", "metadata": {"resourceVersion": rv},
                                    "items": items})
        m = _POD_RE.match(path)
        if m and m.group(2) and not m.group(3):
            with self.store.lock:
                p = self.store.pods.get((m.group(1), m.group(2)))
            return self._send(200, p) if p else self._status(404, "NotFound", f'pods "{m.group(2)}" not found')
        m = _NODE_RE.match(path)
        if m:
            with self.store.lock:
                if m.group(1):
                    n = self.store.nodes.get(m.group(1))
                    return self._send(200, n) if n else self._status(404, "NotFound",
                                                                     f'nodes "{m.group(1)}" not found')
                items = [n for n in self.store.nodes.values() if matches(n, fsel, lsel)]
            return self._send(200, {"kind": "NodeList", "apiVersion": "v1",
                                    "metadata": {"resourceVersion": str(self.store.rv)}, "items": items})
        return self._status(404, "NotFound", path)

    def _watch(self, fsel, lsel, rv, timeout):
        w = self.store.add_watcher(fsel, lsel, rv)
        if w is None:
            return self._status(410, "Expired", "too old resource version")
        self.send_response(200)
        self.send_header("Content-Type", "application/json")
        self.send_header("Transfer-Encoding", "chunked")
        self.end_headers()
        deadline = time.monotonic() + timeout
        try:
            while time.monotonic() < deadline and not self.server.stopping.is_set():
                try:
                    ev = w.q.get(timeout=0.2)
                except queue.Empty:
                    continue
                data = json.dumps(ev, separators=(",", ":")).encode() + b"\n"
                self.wfile.write(b"%x\r\n%s\r\n" % (len(data), data))
                self.wfile.flush()
            self.wfile.write(b"0\r\n\r\n")
        except (BrokenPipeError, ConnectionResetError, OSError):
            pass
        finally:
            self.store.remove_watcher(w)
            self.close_connection = True

    def do_POST(self):
        self._delay()
        path = urllib.parse.urlsplit(self.path).path.rstrip("/")
        body = self._body()
        self.store.requests["POST " + path.split("/")[-1]] += 1
        m = _POD_RE.match(path)
        if m and not m.group(2):
            p = self.store.create_pod(m.group(1), body)
            return self._send(201, p) if p else self._status(409, "AlreadyExists", "pod already exists")
        if m and m.group(3) == "binding":
            try:
                p = self.store.bind_pod(m.group(1), m.group(2), body["target"]["name"])
            except ValueError:
                return self._status(409, "Conflict", "pod is already assigned to a node")
            return self._send(201, {"kind": "Status", "status": "Success"}) if p else \
                self._status(404, "NotFound", "pod not found")
        if path == "/api/v1/nodes":
            n = self.store.create_node(body)
            return self._send(201, n) if n else self._status(409, "AlreadyExists", "node already exists")
        return self._status(404, "NotFound", path)

    def do_PATCH(self):
        self._delay()
        path = urllib.parse.urlsplit(self.path).path.rstrip("/")
        body = self._body()
        self.store.requests["PATCH " + ("status" if path.endswith("/status") else path.split("/")[3])] += 1
        m = _POD_RE.match(path)
        if m and m.group(2):
            try:
                p = self.store.patch_pod(m.group(1), m.group(2), body, status_only=m.group(3) == "status")
            except ValueError:
                return self._status(409, "Conflict", _CONFLICT_MSG)
            return self._send(200, p) if p else self._status(404, "NotFound", f'pods "{m.group(2)}" not found')
        m = _NODE_RE.match(path)
        if m and m.group(1):
            n = self.store.patch_node(m.group(1), body, status_only=m.group(2) == "status")
            return self._send(200, n) if n else self._status(404, "NotFound", f'nodes "{m.group(1)}" not found')
        return self._status(404, "NotFound", path)

    def do_DELETE(self):
        self._delay()
        path = urllib.parse.urlsplit(self.path).path.rstrip("/")
        self.store.requests["DELETE"] += 1
        m = _POD_RE.match(path)
        if m and m.group(2):
            p = self.store.delete_pod(m.group(1), m.group(2))
            return self._send(200, p) if p else self._status(404, "NotFound", "pod not found")
        return self._status(404, "NotFound", path)


class _Server(socketserver.ThreadingMixIn, http.server.HTTPServer):
    daemon_threads = True
    allow_reuse_address = True
    request_queue_size = 128


class FakeAPIServer:
    def __init__(self, host: str = "127.0.0.1", port: int = 0, latency_s: float = 0.0, store: Store | None = None):
        self.store = store or Store()
        self.httpd = _Server((host, port), _Handler)
        self.httpd.store = self.store
        self.httpd.latency_s = latency_s
        self.httpd.stopping = threading.Event()
        self.thread = None

    @property
    def url(self) -> str:
        h, p = self.httpd.server_address[:2]
        return f"http://{h}:{p}"

    def start(self):
        self.thread = threading.Thread(target=self.httpd.serve_forever, name="fake-apiserver", daemon=True)
        self.thread.start()
        return self

    def stop(self):
        self.httpd.stopping.set()
        self.httpd.shutdown()
        self.httpd.server_close()

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
        s.httpd.serve_forever()
    except KeyboardInterrupt:
        pass
    return 0


if __name__ == "__main__":
    sys.exit(main())
