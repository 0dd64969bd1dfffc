"""Control of the per-GPU HBM brokers (``native/hbmbroker``, docs/HBM_TURNOVER.md).

The broker holds a GPU's shareable HBM as VMM granules and lends each pod its own granules,
zeroed between pods, so an admission never waits for amdgpu to wipe the HBM a retired pod freed.
The granter (the device plugin) grants a pod's bytes under a per-pod token on the broker's admin
socket; the pod's quota shim takes the grant with that token (``GPUSHARE_HBM_BROKER`` /
``GPUSHARE_HBM_TOKEN`` in its env) and serves the pod's allocations from it.

Host directory layout (``--hbm-broker-dir``, the node's hostPath):

* ``gpu<i>/hbm<i>.sock`` — GPU ``i``'s pod socket (0666). A container is given only its own
  GPU's ``gpu<i>`` directory, read-only: it can reach that one pod socket and nothing else.
* ``admin/hbm<i>.sock`` — GPU ``i``'s admin socket (0600, in a 0700 directory that is never
  mounted into a container; the broker also checks the peer's uid).
* ``admin/token.key`` — the node's token secret (0600): tokens are HMACs of the pod UID and the
  container slot under it, so they survive a plugin restart and a journal replay.

The granter is level-triggered, like the rest of the plugin after a restart
(``pkg/gpu/nvidia/gpumanager.go:63-108`` re-derives devices and assignments from scratch): it
keeps the set of tokens that live pods need — answers prepared here plus the pods on this node
with a GPU assignment — and makes every broker's grants equal to it. A broker's boot id (STAT)
tells it when a broker restarted and lost its grants; a token no live pod needs any more is
REVOKEd, so a deleted pod's token is refused.

No counterpart in the reference: there a pod's memory is whatever cGPU lets the driver hand out
(``pkg/gpu/nvidia/allocate.go:114-127``).
"""
from __future__ import annotations

import dataclasses
import errno
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


# ---- host directory layout ----------------------------------------------------------------------
def socket_name(gpu_index: int) -> str:
    return f"hbm{gpu_index}.sock"


def pod_dir(host_dir: str, gpu_index: int) -> str:
    """What a container of GPU ``gpu_index`` mounts: this GPU's pod socket, nothing else."""
    return os.path.join(host_dir, f"gpu{gpu_index}")


def pod_socket(host_dir: str, gpu_index: int) -> str:
    return os.path.join(pod_dir(host_dir, gpu_index), socket_name(gpu_index))


def admin_dir(host_dir: str) -> str:
    return os.path.join(host_dir, "admin")


def admin_socket(host_dir: str, gpu_index: int) -> str:
    return os.path.join(admin_dir(host_dir), socket_name(gpu_index))


def secret_path(host_dir: str) -> str:
    return os.path.join(admin_dir(host_dir), "token.key")


def prepare_dirs(host_dir: str, gpu_indices=()) -> None:
    os.makedirs(host_dir, exist_ok=True)
    os.makedirs(admin_dir(host_dir), mode=0o700, exist_ok=True)
    os.chmod(admin_dir(host_dir), 0o700)
    for i in gpu_indices:
        os.makedirs(pod_dir(host_dir, i), mode=0o755, exist_ok=True)


def load_secret(host_dir: str) -> bytes:
    """The node's token secret, created on first use (mode 0600, next to the admin sockets)."""
    prepare_dirs(host_dir)
    path = secret_path(host_dir)
    for _ in range(50):
        try:
            with open(path, "rb") as f:
                key = f.read()
            if len(key) >= 32:
                return key[:32]
        except FileNotFoundError:
            pass
        try:
            fd = os.open(path + ".tmp", os.O_WRONLY | os.O_CREAT | os.O_EXCL, 0o600)
        except FileExistsError:     # another process is writing it: read it in a moment
            time.sleep(0.02)
            continue
        try:
            os.write(fd, os.urandom(32))
            os.fsync(fd)
        finally:
            os.close(fd)
        try:
            os.link(path + ".tmp", path)        # never replaces a key another process wrote first
        except FileExistsError:
            pass
        os.unlink(path + ".tmp")
    raise OSError(errno.EIO, f"cannot read or create the token secret {path}")


def _request(path: str, line: str, timeout: float = 10.0) -> str:
    s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    s.settimeout(timeout)
    try:
        s.connect(path)
        s.sendall(line.encode() + b"\n")
        buf = b""
        while not buf.endswith(b"\n"):
            chunk = s.recv(65536)
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
                 granule_mib: int = 1024, wait_s: float = 30.0, env: dict | None = None, pci_bus_id: str | None = None,
                 admin_path: str | None = None, extra_args=(), exe: str | None = None):
        self.socket_path = socket_path
        self.exe = exe
        self.admin_path = admin_path or socket_path + ".admin"
        self.device, self.gib, self.reserve_gib = device, gib, reserve_gib
        self.pci_bus_id = pci_bus_id
        self.granule_mib, self.wait_s = granule_mib, wait_s
        self.env = env
        self.extra_args = list(extra_args)
        self.proc: subprocess.Popen | None = None
        self.info: dict = {}
        self.last_stderr = ""

    @classmethod
    def for_gpu(cls, host_dir: str, gpu_index: int, **kw) -> "HBMBroker":
        """GPU ``gpu_index``'s broker in the node layout (the plugin's ``--hbm-broker-dir``)."""
        prepare_dirs(host_dir, [gpu_index])
        return cls(pod_socket(host_dir, gpu_index), admin_path=admin_socket(host_dir, gpu_index), **kw)

    @classmethod
    def attach(cls, socket_path: str, admin_path: str | None = None) -> "HBMBroker":
        return cls(socket_path, admin_path=admin_path)

    def start(self, timeout: float = 180.0) -> dict:
        cmd = [self.exe or broker_exe(), "--socket", self.socket_path, "--admin-socket", self.admin_path,
               "--granule-mib", str(self.granule_mib), "--wait-s", str(self.wait_s)]
        cmd += ["--pci-bus-id", self.pci_bus_id] if self.pci_bus_id else ["--device", str(self.device)]
        cmd += ["--gib", str(self.gib)] if self.gib else ["--reserve-gib", str(self.reserve_gib)]
        cmd += self.extra_args
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
            raise RuntimeError(f"hbm broker did not start (exit {p.returncode}): {self.last_stderr[-2000:]}")
        self.info = got
        return got

    def grant(self, token: str, nbytes: int, limit: int | None = None) -> int:
        """Grant ``nbytes`` (rounded up to granules) to the pod holding ``token``; returns the
        number of granules. ``limit``: the pod's whole quota, up to which it may borrow granules
        no grant claims beyond its grant (EXTEND); None = the grant only."""
        line = f"GRANT {token} {int(nbytes)}" + (f" {int(limit)}" if limit else "")
        r = _request(self.admin_path, line)
        if not r.startswith("OK "):
            raise RuntimeError(f"hbm broker refused the grant: {r!r}")
        return int(r.split()[1])

    def size(self, granules: int | str) -> tuple[int, int]:
        """How much of the GPU the broker may hold (``"max"``: all it is sized for; 0: nothing, a
        cgpu-disabled node); returns (granules held now, target)."""
        r = _request(self.admin_path, f"SIZE {granules}")
        if not r.startswith("OK "):
            raise RuntimeError(f"hbm broker refused the size: {r!r}")
        return int(r.split()[1]), int(r.split()[2])

    def revoke(self, token: str) -> int:
        """The token can never be taken again; returns how many granules its holder still has."""
        r = _request(self.admin_path, f"REVOKE {token}")
        if not r.startswith("OK "):
            raise RuntimeError(f"hbm broker refused the revocation: {r!r}")
        return int(r.split()[1])

    def list(self) -> dict:
        return json.loads(_request(self.admin_path, "LIST"))

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


@dataclasses.dataclass
class _Want:
    gpu: int
    nbytes: int
    t: float                 # submitted at (monotonic)
    quota: int = 0           # the container's whole quota: the grant's limit


@dataclasses.dataclass
class _GPUState:
    boot: str = ""           # the broker instance whose grants ``sent`` describes
    up: bool = False
    last_ok: float = 0.0     # last successful STAT (monotonic; 0 = never)
    sent: dict = dataclasses.field(default_factory=dict)     # token -> bytes this broker instance holds
    absent: dict = dataclasses.field(default_factory=dict)   # token -> first time no live pod needed it
    reported: bool | None = None                              # readiness last told to on_readiness
    restarts: int = 0
    stat: dict = dataclasses.field(default_factory=dict)      # the broker's last STAT


class HBMGranter:
    """The device plugin's side (``--hbm-broker-dir``): keeps every GPU broker's grants equal to
    what the node's live pods need (see the module docstring).

    * ``submit`` (an answer being prepared, before the bind when the extender labelled the pod)
      records the token and wakes the granter thread; the answer is never held up by a broker
      (its event loop may be busy). The answer carries the token when the GPU's broker is up, or
      is expected to come up: never seen yet within ``startup_grace_s`` of the plugin's start,
      or last seen within ``down_grace_s``. The pod's shim waits for the broker and its grant;
      a broker that stays away longer gets answers without a token (the pod allocates from the
      driver at once), and ``on_readiness`` tells the engine to re-prepare its answers.
    * every ``poll_s`` the thread reads each broker's STAT. A new boot id (first contact, or a
      broker restart) makes it read the broker's LIST, so it re-grants whatever that instance
      lacks. Then it GRANTs every needed token the broker does not hold, and REVOKEs every
      token the broker holds that no live pod has needed for ``revoke_grace_s`` — never in the
      first ``startup_grace_s`` after start, while the pod view is still filling.
    * ``live()`` (the engine) returns ``{token: (gpu, quota bytes)}`` for the pods on this node
      with a GPU assignment, or None when the pod view is unavailable (then nothing is revoked).

    The grant is ``fraction`` of the container's quota, rounded down to whole 1 GiB granules (the
    shim charges it to the container's ledger). Below 2 granules there is no arena. The grant's
    limit is the whole quota: the pod may borrow granules no grant claims beyond its grant, so it
    can use all of its quota on a packed GPU (the driver serves what the broker cannot).

    ``disabled`` (the node's ``cgpu.disable.isolation=true`` label, ``set_disabled``): no answer
    carries a token, every grant is revoked and each broker is told to hold nothing (SIZE 0), so
    the whole GPU is the driver's, as on the reference's cgpu-disabled nodes
    (``podmanager.go:62-75``, ``allocate.go:125-127``); clearing it sizes them back (SIZE max)."""

    def __init__(self, host_dir: str, fraction: float = 0.94, secret: bytes | None = None,
                 timeout_s: float = 0.5, poll_s: float = 1.0, live=None, startup_grace_s: float = 120.0,
                 down_grace_s: float = 60.0, submit_ttl_s: float = 600.0, revoke_grace_s: float = 5.0,
                 on_readiness=None, start: bool = True, disabled: bool = False):
        self.host_dir = host_dir
        self.fraction = fraction
        self.secret = secret or load_secret(host_dir)
        self.timeout_s, self.poll_s = timeout_s, poll_s
        self.live = live
        self.startup_grace_s, self.down_grace_s = startup_grace_s, down_grace_s
        self.submit_ttl_s, self.revoke_grace_s = submit_ttl_s, revoke_grace_s
        self.on_readiness = on_readiness
        self._t0 = time.monotonic()
        self._mu = threading.Lock()
        self._submits: dict[str, _Want] = {}
        self._unsent: set[str] = set()          # submitted, not yet acknowledged by its broker
        self._gpus: dict[int, _GPUState] = {}
        self._wake = threading.Event()
        self._idle = threading.Condition(self._mu)
        self._stop = threading.Event()
        self._full_passes = 0
        self._force_full = False
        self.disabled = disabled
        self.grants = self.failures = self.revokes = self.regrants = self.resizes = 0
        self._thread = None
        if start:
            self._thread = threading.Thread(target=self._worker, name="hbm-granter", daemon=True)
            self._thread.start()

    # -- the answer side ------------------------------------------------------------------
    def container_socket(self, gpu_index: int) -> str:
        return f"{const.HBM_BROKER_CONTAINER_DIR}/{socket_name(gpu_index)}"

    def mount_dir(self, gpu_index: int) -> str:
        return pod_dir(self.host_dir, gpu_index)

    def token(self, pod_uid: str, slot: int) -> str:
        return hmac.new(self.secret, f"{pod_uid}/{slot}".encode(), hashlib.sha256).hexdigest()[:32]

    def arena_bytes(self, quota_bytes: int) -> int:
        n = int(quota_bytes * self.fraction) // GRANULE
        return n * GRANULE if n >= 2 else 0

    def ready(self, gpu_index: int, now: float | None = None) -> bool:
        """Whether answers for this GPU carry a token (see the class docstring)."""
        now = time.monotonic() if now is None else now
        st = self._gpus.get(gpu_index)
        if st is not None and st.up:
            return True
        if st is not None and st.last_ok:
            return now - st.last_ok < self.down_grace_s
        return now - self._t0 < self.startup_grace_s

    def grantable(self, gpu_index: int, quota_bytes: int) -> bool:
        """Whether ``submit`` would take this grant now (the answer carries the token)."""
        return bool(self.arena_bytes(quota_bytes)) and not self.disabled and self.ready(gpu_index)

    def submit(self, gpu_index: int, token: str, quota_bytes: int, wake: bool = True) -> bool:
        """Record the grant and have the granter thread send it (woken now, or at ``kick()``
        when ``wake`` is false); True = the answer carries the token. Runs on the pod watch /
        prepare threads: never waits for a broker."""
        nbytes = self.arena_bytes(quota_bytes)
        if not nbytes or self.disabled or not self.ready(gpu_index):
            return False
        with self._mu:
            w = self._submits.get(token)
            if w is not None and w.gpu == gpu_index and w.nbytes == nbytes:
                w.t = time.monotonic()
                return True
            self._submits[token] = _Want(gpu_index, nbytes, time.monotonic(), int(quota_bytes))
            st = self._gpus.get(gpu_index)
            if st is None or st.sent.get(token) != nbytes:
                self._unsent.add(token)
        if wake:
            self._wake.set()
        return True

    def kick(self) -> None:
        self._wake.set()

    def flush(self, timeout: float = 5.0) -> bool:
        """Wait until every submitted grant was acknowledged, or until a full pass has tried the
        ones that were not (tests)."""
        end = time.monotonic() + timeout
        with self._mu:
            target = self._full_passes + 2            # one may be under way: the next one started after
            while self._unsent and self._full_passes < target:
                left = end - time.monotonic()
                if left <= 0:
                    return False
                self._force_full = True
                self._wake.set()
                self._idle.wait(left)
        return True

    def reconcile_now(self, timeout: float = 10.0) -> bool:
        """Wait for one full pass that started after this call (tests, SIGHUP)."""
        end = time.monotonic() + timeout
        with self._mu:
            target = self._full_passes + 2
            while self._full_passes < target:
                left = end - time.monotonic()
                if left <= 0:
                    return False
                self._force_full = True
                self._wake.set()
                self._idle.wait(left)
        return True

    def stop(self) -> None:
        self._stop.set()
        self._wake.set()

    def set_disabled(self, disabled: bool) -> None:
        """The node's cgpu.disable.isolation label changed: brokers are sized to nothing (and
        every grant revoked) or back to the whole GPU on the next pass, started now."""
        if disabled == self.disabled:
            return
        self.disabled = disabled
        log.warning("hbm granter: %s", "cgpu isolation disabled on this node: brokers hold no HBM" if disabled
                    else "cgpu isolation enabled again: brokers take the GPU's HBM back")
        with self._mu:
            self._force_full = True
        self._wake.set()

    def stats(self) -> dict:
        with self._mu:
            return {"grants": self.grants, "failures": self.failures, "revokes": self.revokes,
                    "regrants": self.regrants, "resizes": self.resizes, "disabled": self.disabled,
                    "submitted": len(self._submits), "unsent": len(self._unsent),
                    "gpus": {str(i): {"up": st.up, "boot": st.boot, "held": len(st.sent), "restarts": st.restarts}
                             for i, st in sorted(self._gpus.items())}}

    def exposition(self) -> str:
        """The brokers' state as Prometheus text, from each broker's last STAT (one per poll):
        granules by state, takes / releases / timeouts, bytes zeroed, quarantine and scrub
        timings, and the granter's own grant counters."""
        with self._mu:
            gpus = {i: (st.up, dict(st.stat), st.restarts) for i, st in self._gpus.items()}
            own = {"grants": self.grants, "failures": self.failures, "revokes": self.revokes, "regrants": self.regrants,
                   "resizes": self.resizes}
        out = ["# HELP gpushare_hbm_broker_up 1 if the GPU's HBM broker answered the last poll\n"
               "# TYPE gpushare_hbm_broker_up gauge\n"]
        out += [f'gpushare_hbm_broker_up{{gpu="{i}"}} {int(up)}\n' for i, (up, _, _) in sorted(gpus.items())]
        out.append("# HELP gpushare_hbm_broker_granules Granules of the GPU's HBM broker by state\n"
                   "# TYPE gpushare_hbm_broker_granules gauge\n")
        for i, (_, stat, _) in sorted(gpus.items()):
            for state in ("granules", "granules_max", "target", "free", "held", "owed", "extra", "scrubbing",
                          "quarantined"):
                if state in stat:
                    out.append(f'gpushare_hbm_broker_granules{{gpu="{i}",state="{state}"}} {stat[state]}\n')
        for name, key, help_ in (("takes", "takes", "TAKEs served"), ("releases", "releases", "connections that returned granules"),
                                 ("timeouts", "timeouts", "TAKEs refused after waiting"),
                                 ("extended", "extended", "granules lent beyond grants (EXTEND)"),
                                 ("given_back", "given_back", "granules given back to the driver (SIZE, pressure)"),
                                 ("pressure_given", "pressure_given", "granules given back because the driver ran short"),
                                 ("ends", "ends", "streams ended with granules still owed (deadline, revocation)"),
                                 ("scrubbed_bytes", "scrubbed_bytes", "bytes zeroed between pods"),
                                 ("lost", "lost", "granules never lent again (untraceable holder)")):
            out.append(f"# HELP gpushare_hbm_broker_{name}_total {help_}\n# TYPE gpushare_hbm_broker_{name}_total counter\n")
            out += [f'gpushare_hbm_broker_{name}_total{{gpu="{i}"}} {stat[key]}\n'
                    for i, (_, stat, _) in sorted(gpus.items()) if key in stat]
        out.append("# HELP gpushare_hbm_broker_restarts_total Broker restarts seen (a new boot id)\n"
                   "# TYPE gpushare_hbm_broker_restarts_total counter\n")
        out += [f'gpushare_hbm_broker_restarts_total{{gpu="{i}"}} {r}\n' for i, (_, _, r) in sorted(gpus.items())]
        for key in ("quarantine_ms_max", "take_wait_ms_max", "scrub_ms_last"):
            out.append(f"# HELP gpushare_hbm_broker_{key} From the broker's STAT\n# TYPE gpushare_hbm_broker_{key} gauge\n")
            out += [f'gpushare_hbm_broker_{key}{{gpu="{i}"}} {stat[key]}\n'
                    for i, (_, stat, _) in sorted(gpus.items()) if key in stat]
        out.append("# HELP gpushare_hbm_granter_total The plugin's grant traffic to the brokers\n"
                   "# TYPE gpushare_hbm_granter_total counter\n")
        out += [f'gpushare_hbm_granter_total{{op="{k}"}} {v}\n' for k, v in own.items()]
        return "".join(out)

    # -- the granter thread ---------------------------------------------------------------
    def _admin(self, gpu: int, line: str) -> str:
        return _request(admin_socket(self.host_dir, gpu), line, timeout=self.timeout_s)

    def _worker(self) -> None:
        next_full = 0.0
        while not self._stop.is_set():
            now = time.monotonic()
            full = now >= next_full or self._force_full
            try:
                if full:
                    self._force_full = False
                    self._full_pass(now)
                    fast = any(not st.up for st in self._gpus.values())
                    next_full = time.monotonic() + (min(0.25, self.poll_s) if fast else self.poll_s)
                else:
                    self._push_unsent()
            except Exception as e:  # noqa: BLE001 - the granter thread must survive
                log.warning("hbm granter: %s", e)
            with self._mu:
                self._full_passes += full
                self._idle.notify_all()
            self._wake.wait(max(0.0, next_full - time.monotonic()))
            self._wake.clear()

    def _want(self, now: float, live: dict | None) -> dict:
        """token -> (gpu, grant bytes, quota bytes) of every grant live pods need (none while
        the node is cgpu-disabled)."""
        want: dict[str, tuple[int, int, int]] = {}
        with self._mu:
            for tok, w in list(self._submits.items()):
                if now - w.t < self.submit_ttl_s or (live is not None and tok in live):
                    want[tok] = (w.gpu, w.nbytes, w.quota)
                else:
                    del self._submits[tok]
                    self._unsent.discard(tok)
        for tok, (gpu, quota) in (live or {}).items():
            nb = self.arena_bytes(quota)
            if nb:
                want.setdefault(tok, (gpu, nb, quota))
        if self.disabled:
            with self._mu:
                self._submits.clear()
                self._unsent.clear()
            return {}
        return want

    def _push_unsent(self) -> None:
        """Submits not yet sent, to brokers that are up (between full passes: no STAT)."""
        with self._mu:
            todo = [(t, self._submits[t]) for t in self._unsent if t in self._submits]
        for tok, w in todo:
            st = self._gpus.get(w.gpu)
            if st is None or not st.up:
                continue                            # the next full pass contacts it
            self._grant(w.gpu, st, tok, w.nbytes, w.quota)

    def _grant(self, gpu: int, st: _GPUState, tok: str, nbytes: int, quota: int = 0) -> bool:
        try:
            r = self._admin(gpu, f"GRANT {tok} {nbytes}" + (f" {quota}" if quota > nbytes else ""))
            ok = r.startswith("OK ")
        except OSError as e:
            r, ok = str(e), False
        with self._mu:
            if ok:
                self.grants += 1
                st.sent[tok] = nbytes
                st.absent.pop(tok, None)
                w = self._submits.get(tok)
                if w is None or w.nbytes == nbytes:
                    self._unsent.discard(tok)
                return True
            self.failures += 1
            st.up = False
        log.warning("hbm broker of GPU %d: grant not acknowledged (%s); retried on its next poll", gpu, r)
        return False

    def _full_pass(self, now: float) -> None:
        live = None
        if self.live is not None:
            try:
                live = self.live()
            except Exception as e:  # noqa: BLE001 - no revocations without a pod view
                log.V(2).info("hbm granter: no pod view (%s)", e)
        want = self._want(now, live)
        gpus = {w[0] for w in want.values()} | set(self._gpus)
        try:
            present = {int(n[3:]) for n in os.listdir(self.host_dir) if n.startswith("gpu") and n[3:].isdigit()}
        except OSError:
            present = set()
        gpus |= present
        # a cgpu-disabled node revokes at once: no pod here may hold the brokers' HBM
        may_revoke = self.disabled or (live is not None and now - self._t0 >= self.startup_grace_s)
        changed = False
        for gpu in sorted(gpus):
            with self._mu:
                st = self._gpus.setdefault(gpu, _GPUState())
            self._sync_gpu(gpu, st, want, may_revoke, now)
            r = self.ready(gpu, now)
            if st.reported is not None and r != st.reported:
                changed = True
                log.warning("hbm broker of GPU %d: %s", gpu, "answers carry its token again" if r else
                            "down for %.0f s: answers carry no token (pods allocate from the driver)" % self.down_grace_s)
            st.reported = r
        if changed and self.on_readiness is not None:
            try:
                self.on_readiness()
            except Exception as e:  # noqa: BLE001
                log.warning("hbm granter: readiness callback: %s", e)

    def _sync_gpu(self, gpu: int, st: _GPUState, want: dict, may_revoke: bool, now: float) -> None:
        try:
            stat = json.loads(self._admin(gpu, "STAT"))
            st.stat = stat
            boot = stat.get("boot", "")
            if boot != st.boot:
                held = json.loads(self._admin(gpu, "LIST")).get("grants", {})
                with self._mu:
                    if st.boot:
                        st.restarts += 1
                        self.regrants += 1
                        log.warning("hbm broker of GPU %d restarted (boot %s -> %s): re-granting its pods", gpu,
                                    st.boot, boot)
                    st.boot = boot
                    st.sent = {t: n * GRANULE for t, n in held.items()}
                    st.absent.clear()
                    for t, (g, nb, _q) in want.items():
                        if g == gpu and st.sent.get(t) != nb:
                            self._unsent.add(t)
        except (OSError, ValueError) as e:
            with self._mu:
                if st.up:
                    log.warning("hbm broker of GPU %d unreachable: %s", gpu, e)
                st.up = False
            return
        with self._mu:
            st.up = True
            st.last_ok = now
        # its size: the whole GPU (less its reserve), or nothing on a cgpu-disabled node
        target = 0 if self.disabled else stat.get("granules_max")
        if target is not None and "target" in stat and stat["target"] != target:
            try:
                r = self._admin(gpu, f"SIZE {target}")
                if r.startswith("OK "):
                    with self._mu:
                        self.resizes += 1
                    log.info("hbm broker of GPU %d sized to %s granules (holds %s)", gpu, target, r.split()[1])
            except OSError as e:
                log.V(2).info("hbm broker of GPU %d: size: %s", gpu, e)
        for tok, (g, nb, q) in want.items():
            if g == gpu and st.sent.get(tok) != nb:
                if not self._grant(gpu, st, tok, nb, q):
                    return
        if not may_revoke:
            return
        for tok in list(st.sent):
            if tok in want and want[tok][0] == gpu:
                st.absent.pop(tok, None)
                continue
            first = st.absent.setdefault(tok, now)
            if now - first < self.revoke_grace_s and not self.disabled:
                continue
            try:
                r = self._admin(gpu, f"REVOKE {tok}")
            except OSError as e:
                log.V(2).info("hbm broker of GPU %d: revoke: %s", gpu, e)
                return
            if r.startswith("OK"):
                with self._mu:
                    st.sent.pop(tok, None)
                    st.absent.pop(tok, None)
                    self.revokes += 1
