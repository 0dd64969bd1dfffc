"""Control of the per-GPU HBM broker (``native/hbmbroker``, docs/HBM_TURNOVER.md).

The broker holds a GPU's shareable HBM as VMM granules and lends each pod its own granules,
zeroed between pods, so an admission never waits for amdgpu to wipe the HBM a retired pod freed.
The granter (the device plugin at Allocate, or the bench acting for it) grants a pod's bytes
under a one-time token on the broker's admin socket. The pod's quota shim takes the grant with
that token (``GPUSHARE_HBM_BROKER`` / ``GPUSHARE_HBM_TOKEN`` in its env) and serves the pod's
``hipMalloc`` from it.

No counterpart in the reference: there a pod's memory is whatever cGPU lets the driver hand out
(``pkg/gpu/nvidia/allocate.go:114-127``).
"""
from __future__ import annotations

import json
import os
import secrets
import socket
import subprocess
import threading

from ..utils.native import ensure_built

ENV_SOCKET = "GPUSHARE_HBM_BROKER"
ENV_TOKEN = "GPUSHARE_HBM_TOKEN"


def broker_exe() -> str:
    return ensure_built("hbmbroker")


def new_token() -> str:
    return secrets.token_hex(16)


def _request(path: str, line: str, timeout: float = 10.0) -> str:
    s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    s.settimeout(timeout)
    try:
        s.connect(path)
        s.sendall(line.encode() + b"\n")
        buf = b""
        while not buf.endswith(b"\n"):
            chunk = s.recv(4096)
            if not chunk:
                break
            buf += chunk
        return buf.decode().strip()
    finally:
        s.close()


class HBMBroker:
    """One broker process for one GPU (started and stopped here), or a handle on a running one
    (``attach``)."""

    def __init__(self, socket_path: str, device: int = 0, gib: float | None = None, reserve_gib: float = 16.0,
                 granule_mib: int = 1024, wait_s: float = 30.0, env: dict | None = None):
        self.socket_path = socket_path
        self.device, self.gib, self.reserve_gib = device, gib, reserve_gib
        self.granule_mib, self.wait_s = granule_mib, wait_s
        self.env = env
        self.proc: subprocess.Popen | None = None
        self.info: dict = {}

    @classmethod
    def attach(cls, socket_path: str) -> "HBMBroker":
        return cls(socket_path)

    @property
    def admin_path(self) -> str:
        return self.socket_path + ".admin"

    def start(self, timeout: float = 180.0) -> dict:
        cmd = [broker_exe(), "--socket", self.socket_path, "--device", str(self.device),
               "--granule-mib", str(self.granule_mib), "--wait-s", str(self.wait_s)]
        cmd += ["--gib", str(self.gib)] if self.gib else ["--reserve-gib", str(self.reserve_gib)]
        os.makedirs(os.path.dirname(self.socket_path) or ".", exist_ok=True)
        self.proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                                     env=self.env)
        got: dict = {}

        def first_line():
            ln = self.proc.stdout.readline()
            if ln.strip():
                got.update(json.loads(ln))

        t = threading.Thread(target=first_line, daemon=True)
        t.start()
        t.join(timeout)
        if not got.get("ready"):
            p = self.proc
            self.stop()
            err = p.stderr.read() if p.stderr else ""
            raise RuntimeError(f"hbm broker did not start (exit {p.returncode}): {err[-2000:]}")
        self.info = got
        return got

    def grant(self, token: str, nbytes: int) -> int:
        """Grant ``nbytes`` (rounded up to granules) to the pod holding ``token``; returns the
        number of granules."""
        r = _request(self.admin_path, f"GRANT {token} {int(nbytes)}")
        if not r.startswith("OK "):
            raise RuntimeError(f"hbm broker refused the grant: {r!r}")
        return int(r.split()[1])

    def stat(self) -> dict:
        return json.loads(_request(self.admin_path, "STAT"))

    def stop(self) -> None:
        p = self.proc
        if p is None:
            return
        if p.poll() is None:
            p.terminate()
            try:
                p.wait(30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        self.proc = None
