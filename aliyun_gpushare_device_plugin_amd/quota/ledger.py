"""Reader for the quota shim's per-container ledgers (native/hipshim/hipquota.cpp).

With ``--ledger-dir`` the plugin mounts a host directory into every shared container and
the shim keeps its ledger there as a file (``<dir>/gpushare-<pod-uid>-<slot>.ledger``) instead
of a POSIX shm object in the pod-private ``/dev/shm``. The node agent can then read what each
container actually holds, its peak and how many allocations the quota refused — the "shim-
reported per-container usage and quota denials" of SURVEY §5.5 — and garbage-collect the
ledgers of pods that are gone.

Layout (``struct LedgerShm``, little-endian): magic, quota, total, denied, peak (u64 each),
then 256 slots of {i32 pid, i32 pad, u64 used}.
"""
from __future__ import annotations

import dataclasses
import os
import struct

MAGIC = 0x67707573686172          # "gpushar"
N_SLOTS = 256
_HDR = struct.Struct("<5Q")
_SLOT = struct.Struct("<iiQ")
LEDGER_BYTES = _HDR.size + N_SLOTS * _SLOT.size
SUFFIX = ".ledger"


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


def parse(buf: bytes, name: str = "") -> LedgerStats | None:
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
    return LedgerStats(name, key, slot, quota, total, denied, peak, procs)


def read(path: str) -> LedgerStats | None:
    try:
        with open(path, "rb") as f:
            buf = f.read(LEDGER_BYTES)
    except OSError:
        return None
    return parse(buf, os.path.basename(path)[: -len(SUFFIX)] if path.endswith(SUFFIX) else os.path.basename(path))


def scan(directory: str) -> list[LedgerStats]:
    out = []
    try:
        names = sorted(os.listdir(directory))
    except OSError:
        return out
    for n in names:
        if n.endswith(SUFFIX):
            st = read(os.path.join(directory, n))
            if st is not None:
                out.append(st)
    return out


def uid_key(pod_uid: str) -> str:
    """The key ``quota.ledger_name`` derives from a pod UID."""
    return "".join(ch for ch in pod_uid if ch.isalnum())[:40] or "anon"


def collect(directory: str, metrics, live_uids: set[str] | None = None, gc: bool = True) -> list[LedgerStats]:
    """Export every ledger's numbers as gauges; with ``live_uids`` (this node's pods), remove
    ledgers whose pod no longer exists and whose processes have all exited."""
    stats = scan(directory)
    live_keys = {uid_key(u) for u in live_uids} if live_uids is not None else None
    metrics.shim_used.clear()
    metrics.shim_quota.clear()
    metrics.shim_peak.clear()
    metrics.shim_denied.clear()
    for st in stats:
        if gc and live_keys is not None and st.pod_uid_key not in live_keys and st.used == 0:
            try:
                os.unlink(os.path.join(directory, st.name + SUFFIX))
            except OSError:
                pass
            continue
        labels = {"pod_uid": st.pod_uid_key, "container": str(st.container_slot)}
        metrics.shim_used.set(st.used, **labels)
        metrics.shim_quota.set(st.quota, **labels)
        metrics.shim_peak.set(st.peak, **labels)
        metrics.shim_denied.set(st.denied, **labels)
    return stats
