"""Minimal kube-apiserver REST client (component C6's transport).

The reference uses client-go (``podmanager.go:32-60`` clientset from ``$KUBECONFIG`` or
in-cluster config). No Kubernetes Python client is installed offline, so this is a thin
keep-alive HTTP(S) client over ``http.client``: one persistent connection per thread, JSON
bodies, strategic-merge / merge patches, LIST with field/label selectors, and streaming
WATCH. Errors carry the HTTP status so optimistic-lock conflicts are detected by status
code (409), not by string comparison (reference quirk ``allocate.go:140``).
"""
from __future__ import annotations

import base64
import http.client
import json
import os
import socket
import ssl
import tempfile
import threading
import time
import urllib.parse

import yaml

from .. import const
from ..utils import log

STRATEGIC = "application/strategic-merge-patch+json"
MERGE = "application/merge-patch+json"


class APIError(Exception):
    def __init__(self, status: int, reason: str, message: str, body=None):
        super().__init__(f"{status} {reason}: {message}")
        self.status, self.reason, self.message, self.body = status, reason, message, body

    @property
    def conflict(self) -> bool:
        return self.status == 409

    @property
    def not_found(self) -> bool:
        return self.status == 404

    @property
    def gone(self) -> bool:
        return self.status == 410


class KubeConfig:
    """Connection settings. A bearer token read from a file (the projected service-account
    token in a pod, or a kubeconfig ``tokenFile``) is re-read every ``TOKEN_RELOAD_S`` and on a
    401, as client-go's in-cluster config does (``rest.InClusterConfig`` behind
    ``podmanager.go:37-48``): bound service-account tokens rotate (≈1 h) and a plugin that
    cached the first one would lose the apiserver after it expires."""

    TOKEN_RELOAD_S = 60.0

    def __init__(self, server: str, token: str | None = None, ca_file: str | None = None,
                 cert_file: str | None = None, key_file: str | None = None, insecure: bool = False,
                 token_file: str | None = None):
        self.server = server.rstrip("/")
        self.ca_file, self.cert_file, self.key_file = ca_file, cert_file, key_file
        self.insecure = insecure
        self.token_file = token_file
        self._token = token
        self._token_read = 0.0
        self._token_lock = threading.Lock()
        self.token_reloads = 0
        if token_file and token is None:
            self.reload_token(force=True)

    @property
    def token(self) -> str | None:
        if self.token_file and time.monotonic() - self._token_read >= self.TOKEN_RELOAD_S:
            self.reload_token()
        return self._token

    @token.setter
    def token(self, v: str | None):
        self._token = v

    def reload_token(self, force: bool = False) -> bool:
        """Re-read ``token_file``; True when the token changed."""
        if not self.token_file:
            return False
        with self._token_lock:
            if not force and time.monotonic() - self._token_read < self.TOKEN_RELOAD_S:
                return False
            try:
                with open(self.token_file) as f:
                    new = f.read().strip()
            except OSError as e:
                log.warning("cannot read token file %s: %s", self.token_file, e)
                self._token_read = time.monotonic()
                return False
            self._token_read = time.monotonic()
            changed = new != self._token
            if changed:
                self._token = new
                self.token_reloads += 1
            return changed

    @classmethod
    def in_cluster(cls) -> "KubeConfig":
        host, port = os.environ.get("KUBERNETES_SERVICE_HOST"), os.environ.get("KUBERNETES_SERVICE_PORT", "443")
        if not host:
            raise RuntimeError("not running in a cluster: KUBERNETES_SERVICE_HOST unset")
        if ":" in host:
            host = f"[{host}]"
        return cls(f"https://{host}:{port}", ca_file=const.SA_CA_FILE, token_file=const.SA_TOKEN_FILE)

    @classmethod
    def from_file(cls, path: str) -> "KubeConfig":
        with open(path) as f:
            cfg = yaml.safe_load(f) or {}
        ctx_name = cfg.get("current-context")
        ctxs = {c["name"]: c.get("context", {}) for c in cfg.get("contexts", [])}
        ctx = ctxs.get(ctx_name) or (next(iter(ctxs.values())) if ctxs else {})
        clusters = {c["name"]: c.get("cluster", {}) for c in cfg.get("clusters", [])}
        users = {u["name"]: u.get("user", {}) for u in cfg.get("users", [])}
        cl = clusters.get(ctx.get("cluster")) or (next(iter(clusters.values())) if clusters else {})
        us = users.get(ctx.get("user")) or (next(iter(users.values())) if users else {})

        def materialize(data_key, file_key, src):
            if src.get(file_key):
                return src[file_key]
            if src.get(data_key):
                fd, p = tempfile.mkstemp(prefix="gpushare-kube-")
                with os.fdopen(fd, "wb") as f:
                    f.write(base64.b64decode(src[data_key]))
                return p
            return None

        token = us.get("token")
        token_file = us.get("tokenFile") if not token else None
        return cls(cl.get("server", "http://127.0.0.1:8080"), token=token, token_file=token_file,
                   ca_file=materialize("certificate-authority-data", "certificate-authority", cl),
                   cert_file=materialize("client-certificate-data", "client-certificate", us),
                   key_file=materialize("client-key-data", "client-key", us),
                   insecure=bool(cl.get("insecure-skip-tls-verify")))

    @classmethod
    def load(cls, kubeconfig: str | None = None, server: str | None = None) -> "KubeConfig":
        """``--apiserver`` flag > ``$KUBECONFIG`` file (if it exists) > in-cluster
        (same precedence as ``podmanager.go:33-48``)."""
        if server:
            return cls(server)
        path = kubeconfig if kubeconfig is not None else os.environ.get(const.ENV_KUBECONFIG, "")
        if path and os.path.exists(path):
            return cls.from_file(path)
        return cls.in_cluster()


class APIClient:
    def __init__(self, cfg: KubeConfig, timeout: float = 10.0):
        self.cfg = cfg
        self.timeout = timeout
        u = urllib.parse.urlsplit(cfg.server)
        self._https = u.scheme == "https"
        self._host = u.hostname or "127.0.0.1"
        self._port = u.port or (443 if self._https else 80)
        self._prefix = u.path.rstrip("/")
        self._tls = None
        if self._https:
            ctx = ssl.create_default_context(cafile=cfg.ca_file) if cfg.ca_file else ssl.create_default_context()
            if cfg.insecure:
                ctx.check_hostname = False
                ctx.verify_mode = ssl.CERT_NONE
            if cfg.cert_file:
                ctx.load_cert_chain(cfg.cert_file, cfg.key_file)
            self._tls = ctx
        self._local = threading.local()
        self.requests = 0

    def thread_requests(self) -> int:
        """apiserver requests made so far by the calling thread (the Allocate handler counts
        the round trips on its own path with it)."""
        return getattr(self._local, "n", 0)

    # -- transport ----------------------------------------------------------------------
    def _new_conn(self, timeout=None):
        t = self.timeout if timeout is None else timeout
        if self._https:
            c = http.client.HTTPSConnection(self._host, self._port, timeout=t, context=self._tls)
        else:
            c = http.client.HTTPConnection(self._host, self._port, timeout=t)
        c.connect()
        try:
            c.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        except OSError:
            pass
        return c

    def _conn(self):
        c = getattr(self._local, "conn", None)
        if c is None:
            c = self._local.conn = self._new_conn()
        return c

    def _headers(self, content_type=None):
        h = {"Accept": "application/json", "User-Agent": "gpushare-device-plugin-amd/1"}
        if self.cfg.token:
            h["Authorization"] = f"Bearer {self.cfg.token}"
        if content_type:
            h["Content-Type"] = content_type
        return h

    def request(self, method: str, path: str, query: dict | None = None, body=None,
                content_type: str = "application/json", timeout: float | None = None):
        """One request; ``timeout`` bounds each socket operation of this call (default: the
        client's), e.g. a lease renewal that must give up before its renew deadline."""
        url = self._prefix + path
        if query:
            url += "?" + urllib.parse.urlencode({k: v for k, v in query.items() if v is not None})
        data = None if body is None else (body if isinstance(body, bytes) else json.dumps(body).encode())
        r, raw = self._roundtrip(method, url, data, content_type, timeout)
        if r.status == 401 and self.cfg.reload_token(force=True):
            # rotated service-account token: retry once with the new one
            log.info("apiserver answered 401; retrying with the reloaded token")
            r, raw = self._roundtrip(method, url, data, content_type, timeout)
        self.requests += 1
        self._local.n = getattr(self._local, "n", 0) + 1
        try:
            obj = json.loads(raw) if raw else {}
        except ValueError:
            obj = {"message": raw[:200].decode(errors="replace")}
        if r.status >= 400:
            raise APIError(r.status, obj.get("reason", r.reason) if isinstance(obj, dict) else r.reason,
                           obj.get("message", "") if isinstance(obj, dict) else str(obj), obj)
        return obj

    def _roundtrip(self, method, url, data, content_type, timeout=None):
        for attempt in (0, 1):
            c = self._conn()
            t = self.timeout if timeout is None else timeout
            c.timeout = t
            if c.sock is not None:
                c.sock.settimeout(t)
            try:
                c.request(method, url, body=data, headers=self._headers(content_type if data is not None else None))
                r = c.getresponse()
                return r, r.read()
            except (http.client.HTTPException, OSError):
                # stale keep-alive connection: reconnect once
                try:
                    c.close()
                finally:
                    self._local.conn = None
                if attempt:
                    raise
        raise AssertionError("unreachable")

    # -- nodes --------------------------------------------------------------------------
    def get_node(self, name: str) -> dict:
        return self.request("GET", f"/api/v1/nodes/{name}")

    def list_nodes(self, label_selector: str | None = None) -> list:
        return self.request("GET", "/api/v1/nodes", {"labelSelector": label_selector}).get("items", [])

    def patch_node_status(self, name: str, patch: dict) -> dict:
        return self.request("PATCH", f"/api/v1/nodes/{name}/status", body=patch, content_type=STRATEGIC)

    def patch_node(self, name: str, patch: dict) -> dict:
        return self.request("PATCH", f"/api/v1/nodes/{name}", body=patch, content_type=STRATEGIC)

    def create_node(self, node: dict) -> dict:
        return self.request("POST", "/api/v1/nodes", body=node)

    # -- pods ---------------------------------------------------------------------------
    def list_pods(self, namespace: str | None = None, field_selector: str | None = None,
                  label_selector: str | None = None) -> tuple[list, str]:
        path = f"/api/v1/namespaces/{namespace}/pods" if namespace else "/api/v1/pods"
        r = self.request("GET", path, {"fieldSelector": field_selector, "labelSelector": label_selector})
        return r.get("items", []), (r.get("metadata") or {}).get("resourceVersion", "")

    def get_pod(self, namespace: str, name: str) -> dict:
        return self.request("GET", f"/api/v1/namespaces/{namespace}/pods/{name}")

    def create_pod(self, namespace: str, pod: dict) -> dict:
        return self.request("POST", f"/api/v1/namespaces/{namespace}/pods", body=pod)

    def patch_pod(self, namespace: str, name: str, patch: dict, content_type: str = STRATEGIC) -> dict:
        return self.request("PATCH", f"/api/v1/namespaces/{namespace}/pods/{name}", body=patch,
                            content_type=content_type)

    def patch_pod_status(self, namespace: str, name: str, patch: dict) -> dict:
        return self.request("PATCH", f"/api/v1/namespaces/{namespace}/pods/{name}/status", body=patch,
                            content_type=STRATEGIC)

    def delete_pod(self, namespace: str, name: str) -> dict:
        return self.request("DELETE", f"/api/v1/namespaces/{namespace}/pods/{name}")

    def bind_pod(self, namespace: str, name: str, node: str, uid: str | None = None) -> dict:
        body = {"apiVersion": "v1", "kind": "Binding", "metadata": {"name": name, "namespace": namespace},
                "target": {"apiVersion": "v1", "kind": "Node", "name": node}}
        if uid:
            body["metadata"]["uid"] = uid
        return self.request("POST", f"/api/v1/namespaces/{namespace}/pods/{name}/binding", body=body)

    def watch_pods(self, field_selector: str | None = None, resource_version: str | None = None,
                   timeout_seconds: int = 300, stop: threading.Event | None = None, holder: list | None = None,
                   label_selector: str | None = None):
        """Yields watch events (dicts with ``type`` and ``object``) until the server ends the
        stream (``timeoutSeconds``), or ``stop`` is set and the socket is shut down by
        ``abort_watch(holder)``. Uses its own connection; reads block without a socket timeout
        (an idle watch is normal), so stopping works by shutting the socket down."""
        q = {"watch": "1", "fieldSelector": field_selector, "labelSelector": label_selector,
             "resourceVersion": resource_version,
             "timeoutSeconds": str(timeout_seconds), "allowWatchBookmarks": "true"}
        url = self._prefix + "/api/v1/pods?" + urllib.parse.urlencode({k: v for k, v in q.items() if v})
        c = self._new_conn()
        if holder is not None:
            holder[:] = [c]
        try:
            c.request("GET", url, headers=self._headers())
            r = c.getresponse()
            if r.status >= 400:
                raw = r.read()
                try:
                    obj = json.loads(raw)
                except ValueError:
                    obj = {}
                if r.status == 401:
                    self.cfg.reload_token(force=True)     # the informer's next attempt uses it
                raise APIError(r.status, obj.get("reason", r.reason), obj.get("message", ""), obj)
            c.sock.settimeout(None)
            buf = b""
            while not (stop and stop.is_set()):
                try:
                    chunk = r.read1(65536)
                except (ValueError, http.client.IncompleteRead):   # cut mid-chunk: stream over
                    break
                if not chunk:
                    break
                t_read = time.monotonic_ns()
                buf += chunk
                while b"\n" in buf:
                    line, buf = buf.split(b"\n", 1)
                    line = line.strip()
                    if line:
                        ev = json.loads(line)
                        ev["_read_ns"] = t_read            # when its bytes arrived (timelines)
                        yield ev
        finally:
            if holder is not None:
                holder[:] = []
            try:
                c.close()
            except Exception:
                pass

    @staticmethod
    def abort_watch(holder: list | None):
        for c in list(holder or []):
            try:
                c.sock.shutdown(socket.SHUT_RDWR)
            except (OSError, AttributeError):
                pass

    def close(self):
        c = getattr(self._local, "conn", None)
        if c is not None:
            c.close()
            self._local.conn = None


def build_client(kubeconfig: str | None = None, server: str | None = None, timeout: float = 10.0) -> APIClient:
    cfg = KubeConfig.load(kubeconfig, server)
    log.V(1).info("apiserver %s", cfg.server)
    return APIClient(cfg, timeout=timeout)
