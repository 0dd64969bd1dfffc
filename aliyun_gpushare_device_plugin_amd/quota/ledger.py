"""Per-container quota-shim ledgers on the host: isolation, usage export, garbage collection.

With ``--ledger-dir`` the quota shim (native/hipshim/hipquota.cpp) keeps each container's
ledger as a file the node agent can read — what the container holds, its peak and how many
allocations the quota refused (the "shim-reported per-container usage and quota denials" of
SURVEY §5.5) — instead of a POSIX shm object in the pod-private ``/dev/shm``.

Layout (host side)::

    <root>/                      0755, plugin-owned, never mounted
    <root>/<lkey>/               0777, bind-mounted read-write into exactly ONE container at
                                 const.LEDGER_CONTAINER_DIR (Allocate ``Mount``)
    <root>/<lkey>/gpushare-<pod-uid-key>-<slot>.ledger    written by the shim
    <root>/.owners/<lkey>        0600 JSON {"pods": [uid, ...], "t": ...}, plugin-only

A container sees only its own ledger directory, so no tenant can read a neighbour's usage or
rewrite its ``total``/``quota``. ``lkey`` is unique per answered container (pod-uid key,
container slot, random suffix), so a recycled set of fake IDs or a re-answered pod never
lands on an old ledger. The owner record names the pod the answer was matched to and — after
placement truth (``alloc/placement.py``) found that another pod's container holds it — that
pod too; a directory is garbage once none of its owners is alive on the node, whatever the
ledger says is used (a SIGKILLed or OOM-killed container never releases its slot).

Ledger file format (``struct LedgerShm``, little-endian): magic, quota, total, denied, peak
(u64 each), then 256 slots of {i32 pid, i32 pad, u64 used}.
"""
from __future__ import annotations

import dataclasses
import json
import os
import shutil
import struct
import threading
import time

MAGIC = 0x67707573686172          # "gpushar"
N_SLOTS = 256
_HDR = struct.Struct("<5Q")
_SLOT = struct.Struct("<iiQ")
LEDGER_BYTES = _HDR.size + N_SLOTS * _SLOT.size
SUFFIX = ".ledger"
OWNERS = ".owners"


@dataclasses.dataclass(frozen=True)
class LedgerStats:
    name: str           # file name without suffix: gpushare-<uid>-<slot>
    pod_uid_key: str    # the alphanumeric pod-uid key the plugin wrote (see quota.ledger_name)
    container_slot: int
    quota: int
    used: int
    denied: int
    peak: int
    processes: int      # slots with a live (non-zero) pid
    lkey: str = ""      # the per-container directory it lives in ("" = legacy flat layout)


def parse(buf: bytes, name: str = "", lkey: str = "") -> LedgerStats | None:
    if len(buf) < LEDGER_BYTES:
        return None
    magic, quota, total, denied, peak = _HDR.unpack_from(buf, 0)
    if magic != MAGIC:
        return None
    procs = sum(1 for i in range(N_SLOTS) if _SLOT.unpack_from(buf, _HDR.size + i * _SLOT.size)[0] > 0)
    key, slot = name, -1
    if name.startswith("gpushare-"):
        body = name[len("gpushare-"):]
        k, _, s = body.rpartition("-")
        if s.isdigit():
            key, slot = k, int(s)
    return LedgerStats(name, key, slot, quota, total, denied, peak, procs, lkey)


def read(path: str, lkey: str = "") -> LedgerStats | None:
    try:
        with open(path, "rb") as f:
            buf = f.read(LEDGER_BYTES)
    except OSError:
        return None
    base = os.path.basename(path)
    return parse(buf, base[: -len(SUFFIX)] if base.endswith(SUFFIX) else base, lkey)


def uid_key(pod_uid: str) -> str:
    """The key ``quota.ledger_name`` derives from a pod UID."""
    return "".join(ch for ch in pod_uid if ch.isalnum())[:40] or "anon"


class LedgerDir:
    """The plugin's side of ``<root>``: per-container directories and their owner records.

    Directory creation costs a few filesystem syscalls (≈0.1-1 ms on an overlay root), too
    much for the Allocate path, so ``take`` hands out a directory made ahead of time by a
    background thread (a *pool* entry: owner record ``{"pods": [], "pool": true}``, which the
    garbage collector leaves alone) and its owner record is written behind the answer. A pool
    left by a previous plugin instance is adopted on ``prepare``."""

    def __init__(self, root: str, pool_size: int = 32):
        self.root = root
        self._owners = os.path.join(root, OWNERS)
        self.pool_size = pool_size
        self._pool: list[str] = []
        self._pending: list[tuple[str, list]] = []     # owner records to write behind
        self._cv = threading.Condition()
        self._writing = 0                      # owner records taken from _pending, not yet on disk
        self._thread = None

    def prepare(self) -> None:
        os.makedirs(self._owners, exist_ok=True)
        os.chmod(self.root, 0o755)        # tenants never see the root, only their own subdir
        os.chmod(self._owners, 0o700)
        for lkey in self.keys():
            rec = self._record(lkey)
            if rec.get("pool") and not rec.get("pods"):
                self._pool.append(lkey)

    def start(self) -> "LedgerDir":
        """Background pool refill + owner-record writer."""
        if self._thread is None:
            self._thread = threading.Thread(target=self._run, name="ledger-pool", daemon=True)
            self._thread.start()
        return self

    def _run(self):
        while True:
            with self._cv:
                while not self._pending and len(self._pool) >= self.pool_size:
                    self._cv.wait()
                todo, self._pending = self._pending, []
                self._writing = len(todo)
                short = self.pool_size - len(self._pool)
            for lkey, pods in todo:
                try:
                    self._write_owners(lkey, pods)
                except OSError:
                    pass
            with self._cv:
                self._writing = 0
            for _ in range(max(0, short)):
                lkey = self.new_key()
                try:
                    self._mkdir(lkey)
                    self._write_owners(lkey, [], pool=True)
                except OSError:
                    break
                with self._cv:
                    self._pool.append(lkey)

    def new_key(self, pod_uid: str = "", slot: int | None = None) -> str:
        head = f"{uid_key(pod_uid)[:32]}-{slot}-" if pod_uid else "c-"
        return head + os.urandom(6).hex()

    def _mkdir(self, lkey: str) -> str:
        path = os.path.join(self.root, lkey)
        os.makedirs(path, exist_ok=True)
        os.chmod(path, 0o777)             # containers may run as any uid; only one sees it
        return path

    def take(self, owner_uid: str, wake: bool = True) -> str:
        """A fresh per-container directory for ``owner_uid``'s container: its key. Pool hit =
        no syscall on the caller's path; the owner record follows on the background thread
        (woken now, or at ``kick()`` when ``wake`` is false: a caller racing the kubelet's
        Allocate keeps the interpreter to itself until its answer is published)."""
        with self._cv:
            lkey = self._pool.pop() if self._pool else None
            if lkey is not None:
                self._pending.append((lkey, [owner_uid] if owner_uid else []))
                if wake:
                    self._cv.notify()
                return lkey
        lkey = self.new_key(owner_uid, 0)
        self.create(lkey, owner_uid)
        with self._cv:
            self._cv.notify()
        return lkey

    def kick(self) -> None:
        """Wake the background thread for records ``take(wake=False)`` left."""
        with self._cv:
            self._cv.notify()

    def path(self, lkey: str) -> str:
        return os.path.join(self.root, lkey)

    def create(self, lkey: str, owner_uid: str) -> str:
        """Create ``<root>/<lkey>`` (writable by any container uid) and its owner record now;
        returns the host path to mount."""
        path = self._mkdir(lkey)
        self._write_owners(lkey, [owner_uid] if owner_uid else [])
        return path

    def _write_owners(self, lkey: str, pods: list, pool: bool = False) -> None:
        tmp = os.path.join(self._owners, f".{lkey}.tmp")
        rec = {"pods": pods, "t": time.time()}
        if pool:
            rec["pool"] = True
        with open(tmp, "w") as f:
            json.dump(rec, f)
        os.replace(tmp, os.path.join(self._owners, lkey))

    def _record(self, lkey: str) -> dict:
        try:
            with open(os.path.join(self._owners, lkey)) as f:
                return json.load(f)
        except (OSError, ValueError):
            return {}

    def owners(self, lkey: str) -> tuple[list, float]:
        d = self._record(lkey)
        return list(d.get("pods") or []), float(d.get("t") or 0.0)

    def flush(self, timeout: float = 5.0) -> bool:
        """Wait until the queued owner records are written (tests, shutdown)."""
        t = time.monotonic() + timeout
        while time.monotonic() < t:
            with self._cv:
                if not self._pending and not self._writing:
                    return True
            time.sleep(0.005)
        return False

    def add_owner(self, lkey: str, uid: str) -> None:
        """Placement truth: ``uid``'s container holds the grant this ledger was made for."""
        self.flush()
        pods, _ = self.owners(lkey)
        if uid and uid not in pods:
            self._write_owners(lkey, pods + [uid])

    def keys(self) -> list[str]:
        try:
            return sorted(n for n in os.listdir(self.root)
                          if n != OWNERS and not n.startswith(".") and os.path.isdir(os.path.join(self.root, n)))
        except OSError:
            return []

    def remove(self, lkey: str) -> None:
        shutil.rmtree(os.path.join(self.root, lkey), ignore_errors=True)
        try:
            os.unlink(os.path.join(self._owners, lkey))
        except OSError:
            pass


def scan(directory: str) -> list[LedgerStats]:
    """Every ledger under ``directory``: per-container subdirectories, plus ledger files left
    in the root by the legacy flat layout."""
    out = []
    ld = LedgerDir(directory)
    for lkey in ld.keys():
        sub = os.path.join(directory, lkey)
        try:
            names = sorted(os.listdir(sub))
        except OSError:
            continue
        for n in names:
            if n.endswith(SUFFIX):
                st = read(os.path.join(sub, n), lkey)
                if st is not None:
                    out.append(st)
    try:
        flat = sorted(n for n in os.listdir(directory) if n.endswith(SUFFIX))
    except OSError:
        flat = []
    for n in flat:
        st = read(os.path.join(directory, n))
        if st is not None:
            out.append(st)
    return out


def collect(directory: str, metrics, live_uids: set[str] | None = None, gc: bool = True,
            grace_s: float = 60.0) -> list[LedgerStats]:
    """Export every live ledger's numbers as gauges (labelled with the pod that holds it); with
    ``live_uids`` (this node's pods) remove the ledgers of containers whose pods are all gone —
    regardless of the ``used`` they still show (a killed process never releases its slot).
    A directory younger than ``grace_s`` is kept: its pod may not be in the cache yet."""
    ld = LedgerDir(directory)
    now = time.time()
    live_keys = {uid_key(u) for u in live_uids} if live_uids is not None else None
    removed: set[str] = set()
    holder: dict[str, str] = {}
    for lkey in ld.keys():
        rec = ld._record(lkey)
        if rec.get("pool") and not rec.get("pods"):
            continue                            # made ahead, not handed out yet
        pods, t = list(rec.get("pods") or []), float(rec.get("t") or 0.0)
        alive = [u for u in pods if live_uids is None or u in live_uids]
        if alive:
            holder[lkey] = uid_key(alive[-1])   # the latest owner: the pod really running it
        elif gc and live_uids is not None and now - t > grace_s:
            ld.remove(lkey)
            removed.add(lkey)
    metrics.shim_used.clear()
    metrics.shim_quota.clear()
    metrics.shim_peak.clear()
    metrics.shim_denied.clear()
    out = []
    for st in scan(directory):
        if st.lkey in removed:
            continue
        if not st.lkey and gc and live_keys is not None and st.pod_uid_key not in live_keys:
            try:                                # legacy flat ledger of a gone pod
                os.unlink(os.path.join(directory, st.name + SUFFIX))
            except OSError:
                pass
            continue
        out.append(st)
        labels = {"pod_uid": holder.get(st.lkey, st.pod_uid_key), "container": str(st.container_slot)}
        metrics.shim_used.set(st.used, **labels)
        metrics.shim_quota.set(st.quota, **labels)
        metrics.shim_peak.set(st.peak, **labels)
        metrics.shim_denied.set(st.denied, **labels)
    return out
