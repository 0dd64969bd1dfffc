"""Kubelet read-only client: HTTPS GET ``https://<addr>:<port>/pods/`` (component C8).

Reference ``pkg/kubelet/client/client.go:16-134``: bearer token or client cert, TLS
verification always skipped, decodes a ``v1.PodList``. Fixed here: the
response body is always closed and non-2xx statuses raise instead of being decoded. A
service-account token read from its file is re-read on a timer and on a 401 (rotation), with
the same policy as the apiserver client (``cluster/client.py`` ``KubeConfig``).
"""
from __future__ import annotations

import http.client
import json
import os
import ssl
import time

from .. import const


class KubeletClient:
    def __init__(self, address: str = "127.0.0.1", port: int = 10250, token: str | None = None,
                 cert_file: str | None = None, key_file: str | None = None, timeout: float = 10.0,
                 scheme: str = "https", token_file: str | None = None):
        self.address, self.port, self.token, self.timeout = address, port, token, timeout
        self.scheme = scheme
        self.token_file = token_file
        self._token_read = time.monotonic()
        self._ctx = None
        if scheme == "https":
            ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_CLIENT)
            ctx.check_hostname = False
            ctx.verify_mode = ssl.CERT_NONE      # client.go:56-72: Insecure: true
            if cert_file:
                ctx.load_cert_chain(cert_file, key_file)
            self._ctx = ctx

    @classmethod
    def from_flags(cls, address, port, cert_file="", key_file="", token="", timeout=10.0, scheme="https"):
        """``buildKubeletClient`` (``cmd/nvidia/main.go:28-53``): with no cert/key/token, read the
        service-account token; unlike the reference a missing token is an error, not a panic."""
        token_file = None
        if not (cert_file or key_file or token):
            if os.path.exists(const.SA_TOKEN_FILE):
                with open(const.SA_TOKEN_FILE) as f:
                    token = f.read().strip()
                token_file = const.SA_TOKEN_FILE
            else:
                raise RuntimeError(f"in cluster mode, find token failed: {const.SA_TOKEN_FILE} missing")
        return cls(address, port, token or None, cert_file or None, key_file or None, timeout, scheme, token_file)

    def _reload_token(self, force: bool = False) -> bool:
        from .client import KubeConfig

        if not self.token_file or (not force and time.monotonic() - self._token_read < KubeConfig.TOKEN_RELOAD_S):
            return False
        self._token_read = time.monotonic()
        try:
            with open(self.token_file) as f:
                new = f.read().strip()
        except OSError:
            return False
        changed, self.token = new != self.token, new
        return changed

    def get_node_running_pods(self) -> list[dict]:
        self._reload_token()
        try:
            return self._get_pods()
        except PermissionError:
            if not self._reload_token(force=True):
                raise
            return self._get_pods()

    def _get_pods(self) -> list[dict]:
        if self.scheme == "https":
            c = http.client.HTTPSConnection(self.address, self.port, timeout=self.timeout, context=self._ctx)
        else:
            c = http.client.HTTPConnection(self.address, self.port, timeout=self.timeout)
        try:
            h = {"Accept": "application/json"}
            if self.token:
                h["Authorization"] = f"Bearer {self.token}"
            c.request("GET", "/pods/", headers=h)
            r = c.getresponse()
            body = r.read()
            if r.status == 401:
                raise PermissionError(f"kubelet /pods returned 401: {body[:200]!r}")
            if r.status != 200:
                raise RuntimeError(f"kubelet /pods returned {r.status}: {body[:200]!r}")
            return (json.loads(body) or {}).get("items", []) or []
        finally:
            c.close()
