"""Control of the per-GPU HBM broker (``native/hbmbroker``, docs/HBM_TURNOVER.md).

The broker holds a GPU's shareable HBM as VMM granules and lends each pod its own granules,
zeroed between pods, so an admission never waits for amdgpu to wipe the HBM a retired pod freed.
The granter (the device plugin at Allocate, or the bench acting for it) grants a pod's bytes
under a per-pod token on the broker's admin socket. The pod's quota shim takes the grant with
that token (``GPUSHARE_HBM_BROKER`` / ``GPUSHARE_HBM_TOKEN`` in its env) and serves the pod's
``hipMalloc`` from it.

No counterpart in the reference: there a pod's memory is whatever cGPU lets the driver hand out
(``pkg/gpu/nvidia/allocate.go:114-127``).
"""
from __future__ import annotations

import collections
import hashlib
import hmac
import json
import os
import secrets
import socket
import subprocess
import threading
import time

from .. import const
from ..utils import log
from ..utils.native import ensure_built

ENV_SOCKET = const.ENV_HBM_BROKER
ENV_TOKEN = const.ENV_HBM_TOKEN
GRANULE = 1 << 30


def broker_exe() -> str:
    """The broker binary (``GPUSHARE_HBM_BROKER_EXE`` overrides it: tests run a stand-in)."""
    return os.environ.get("GPUSHARE_HBM_BROKER_EXE") or ensure_built("hbmbroker")


def new_token() -> str:
    return secrets.token_hex(16)


def socket_name(gpu_index: int) -> str:
    """The broker socket of GPU ``gpu_index`` inside the broker directory."""
    return f"hbm{gpu_index}.sock"


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
                 granule_mib: int = 1024, wait_s: float = 30.0, env: dict | None = None, pci_bus_id: str | None = None):
        self.socket_path = socket_path
        self.device, self.gib, self.reserve_gib = device, gib, reserve_gib
        self.pci_bus_id = pci_bus_id
        self.granule_mib, self.wait_s = granule_mib, wait_s
        self.env = env
        self.proc: subprocess.Popen | None = None
        self.info: dict = {}
        self.last_stderr = ""

    @classmethod
    def attach(cls, socket_path: str) -> "HBMBroker":
        return cls(socket_path)

    @property
    def admin_path(self) -> str:
        return self.socket_path + ".admin"

    def start(self, timeout: float = 180.0) -> dict:
        cmd = [broker_exe(), "--socket", self.socket_path, "--granule-mib", str(self.granule_mib),
               "--wait-s", str(self.wait_s)]
        cmd += ["--pci-bus-id", self.pci_bus_id] if self.pci_bus_id else ["--device", str(self.device)]
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

    def stop(self) -> int | None:
        """Stop the broker; returns its exit status (SIGTERM ends it cleanly: 0). Its stderr is
        kept in ``last_stderr``."""
        p = self.proc
        if p is None:
            return None
        if p.poll() is None:
            p.terminate()
            try:
                p.wait(30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        try:
            self.last_stderr = p.stderr.read() if p.stderr else ""
        except (OSError, ValueError):
            self.last_stderr = ""
        self.proc = None
        return p.returncode


class HBMGranter:
    """The device plugin's side (``--hbm-broker-dir``): grants each shared container its HBM on
    its GPU's broker when the plugin prepares the container's Allocate answer (before the bind
    when the extender labelled the pod), from a background thread, under a token derived from
    the pod UID and the container slot with a per-process secret. The same pod always gets the
    same token, so a re-prepared or replayed answer is byte-identical.

    The grant is ``fraction`` of the container's quota, rounded down to whole 1 GiB granules
    (the shim charges it to the container's ledger, and what the runtime still takes from the
    driver is charged on top, within the quota). Below 2 granules there is no arena. A broker
    that cannot be reached is skipped for ``backoff_s``: the answer then carries no token and the
    pod allocates from the driver as without a broker (a grant that fails after its answer went
    out: the pod's TAKE times out at the broker and the pod uses the driver)."""

    def __init__(self, host_dir: str, fraction: float = 0.94, secret: bytes | None = None,
                 timeout_s: float = 0.2, backoff_s: float = 5.0):
        self.host_dir = host_dir
        self.fraction = fraction
        self.secret = secret or os.urandom(32)
        self.timeout_s, self.backoff_s = timeout_s, backoff_s
        self._mu = threading.Lock()
        self._granted: collections.OrderedDict = collections.OrderedDict()   # token -> bytes
        self._down_until: dict[int, float] = {}
        self.grants = self.failures = 0
        import queue
        self._q: "queue.Queue" = queue.Queue()
        self._queued: set[str] = set()
        self._idle = threading.Event()
        self._idle.set()
        threading.Thread(target=self._worker, name="hbm-granter", daemon=True).start()

    def submit(self, gpu_index: int, token: str, quota_bytes: int) -> bool:
        """Grant in the background; True = the answer carries the token. The answer is prepared
        on the pod watch thread, which must not wait for a broker (its event loop can be inside
        a scrub); the broker holds the pod's TAKE until the grant has arrived."""
        nbytes = self.arena_bytes(quota_bytes)
        if not nbytes:
            return False
        with self._mu:
            if self._granted.get(token) == nbytes or token in self._queued:
                return True
            if self._down_until.get(gpu_index, 0.0) > time.monotonic():
                return False
            self._queued.add(token)
            self._idle.clear()
        self._q.put((gpu_index, token, quota_bytes))
        return True

    def flush(self, timeout: float = 5.0) -> bool:
        """Wait until every submitted grant was sent (tests)."""
        return self._idle.wait(timeout)

    def _worker(self) -> None:
        while True:
            gpu_index, token, quota_bytes = self._q.get()
            try:
                self.grant(gpu_index, token, quota_bytes)
            except Exception as e:  # noqa: BLE001 - the granter thread must survive
                log.warning("hbm broker grant failed: %s", e)
            with self._mu:
                self._queued.discard(token)
                if not self._queued:
                    self._idle.set()

    def container_socket(self, gpu_index: int) -> str:
        return f"{const.HBM_BROKER_CONTAINER_DIR}/{socket_name(gpu_index)}"

    def token(self, pod_uid: str, slot: int) -> str:
        return hmac.new(self.secret, f"{pod_uid}/{slot}".encode(), hashlib.sha256).hexdigest()[:32]

    def arena_bytes(self, quota_bytes: int) -> int:
        n = int(quota_bytes * self.fraction) // GRANULE
        return n * GRANULE if n >= 2 else 0

    def grant(self, gpu_index: int, token: str, quota_bytes: int) -> bool:
        nbytes = self.arena_bytes(quota_bytes)
        if not nbytes:
            return False
        with self._mu:
            if self._granted.get(token) == nbytes:
                return True
        path = os.path.join(self.host_dir, socket_name(gpu_index)) + ".admin"
        try:
            r = _request(path, f"GRANT {token} {nbytes}", timeout=self.timeout_s)
            ok = r.startswith("OK ")
        except OSError as e:
            r, ok = str(e), False
        with self._mu:
            if ok:
                self.grants += 1
                self._granted[token] = nbytes
                while len(self._granted) > 8192:
                    self._granted.popitem(last=False)
                return True
            self.failures += 1
            self._down_until[gpu_index] = time.monotonic() + self.backoff_s
        log.warning("hbm broker of GPU %d: no grant (%s); its pods allocate from the driver for %.0f s",
                    gpu_index, r, self.backoff_s)
        return False
