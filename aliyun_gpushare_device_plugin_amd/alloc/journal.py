"""Allocate decision journal: idempotent answers and durable write-behind.

The reference keeps no state (``allocate.go``) and answers Allocate only after its
``ASSIGNED=true`` PATCH landed (``:132-152``). This build answers first and lands the PATCH
in the background (write-behind, ``alloc/engine.py``), so the journal carries two kinds of
record, in memory and optionally in an append-only JSON-lines file that survives a plugin
restart or crash:

* **answers** (``{"k", "uid", "t", "resp"}``), keyed by the request's fake-device-ID set: if
  the kubelet re-sends an Allocate after the plugin already matched the pod (an RPC deadline
  hit, a restart between the match and the reply), the engine replays the answer — but only
  while the journaled pod still exists on this node *and is still Pending*. The kubelet
  recycles freed fake IDs for new pods, so a key alone is never trusted.
* **pending patches** (``{"op": "patch", "uid", "ns", "name", "ann"}``), written *before* the
  reply leaves the plugin, and **landings** (``{"op": "landed", "uid"}``) once the apiserver
  acknowledged the PATCH. On start-up every pending patch without a landing is re-queued, and
  its pod stays claimed, so a pod can neither be left ``ASSIGNED=false`` forever nor be
  matched a second time by the next plugin instance.

Each record is one ``write(2)`` on an ``O_APPEND`` descriptor (no userspace buffering, no
``fsync``): the journal must survive the *process* (kill, crash, OOM, DaemonSet rollout); a
node crash takes the pods' containers down with it. A write-behind answer and its pending
patch share one record (``{"op": "answer+patch", ...}``), so the journal costs one syscall
on the Allocate path.
"""
from __future__ import annotations

import base64
import collections
import hashlib
import json
import os
import threading
import time

from ..api import v1beta1 as api
from ..utils import log


def request_key(req) -> str:
    body = "\x1e".join("\x1f".join(sorted(c.devices_ids)) for c in req.container_requests)
    return hashlib.sha1(body.encode()).hexdigest()


class AllocJournal:
    def __init__(self, path: str | None = None, ttl_s: float = 120.0, max_entries: int = 4096,
                 pending_ttl_s: float = 24 * 3600.0):
        self.path, self.ttl_s, self.max_entries = path, ttl_s, max_entries
        self.pending_ttl_s = pending_ttl_s
        self._mem: collections.OrderedDict[str, tuple[str, float, bytes]] = collections.OrderedDict()
        self._uids: dict[str, float] = {}                       # pod uid -> time of its answer
        self._pending: collections.OrderedDict[str, dict] = collections.OrderedDict()  # uid -> patch
        self._lock = threading.Lock()
        self._lines = 0
        self._fd = -1
        if path:
            self._load()

    # -- persistence ------------------------------------------------------------------------
    def _load(self):
        try:
            with open(self.path) as f:
                lines = f.readlines()
        except FileNotFoundError:
            return
        now = time.time()
        for line in lines:
            try:
                e = json.loads(line)
                op = e.get("op", "answer")
                if op in ("patch", "answer+patch"):
                    if now - e["t"] <= self.pending_ttl_s:
                        self._pending[e["uid"]] = {k: e[k] for k in ("uid", "ns", "name", "ann", "t")} | {"op": "patch"}
                if op == "patch":
                    continue
                if op == "landed":
                    self._pending.pop(e["uid"], None)
                elif now - e["t"] <= self.ttl_s:
                    self._mem[e["k"]] = (e["uid"], e["t"], base64.b64decode(e["resp"]))
                    self._mem.move_to_end(e["k"])
                    self._uids[e["uid"]] = e["t"]
            except (ValueError, KeyError, TypeError):
                continue                                          # a torn last line after a crash
        while len(self._mem) > self.max_entries:
            self._mem.popitem(last=False)
        self._lines = len(lines)
        log.info("allocation journal %s: %d recent decisions, %d unlanded patches loaded", self.path,
                 len(self._mem), len(self._pending))
        self._compact()

    def _write(self, rec: dict):
        if not self.path:
            return
        try:
            if self._fd < 0:
                os.makedirs(os.path.dirname(self.path) or ".", exist_ok=True)
                self._fd = os.open(self.path, os.O_WRONLY | os.O_APPEND | os.O_CREAT | os.O_CLOEXEC, 0o600)
            os.write(self._fd, (json.dumps(rec, separators=(",", ":")) + "\n").encode())
            self._lines += 1
            if self._lines > 2 * self.max_entries + 2 * len(self._pending) + 64:
                self._compact()
        except OSError as e:
            log.warning("allocation journal write failed: %s", e)

    def _compact(self):
        if not self.path:
            return
        tmp = self.path + ".tmp"
        try:
            os.makedirs(os.path.dirname(self.path) or ".", exist_ok=True)
            with open(tmp, "w") as f:
                for k, (uid, t, blob) in self._mem.items():
                    f.write(json.dumps({"k": k, "uid": uid, "t": t, "resp": base64.b64encode(blob).decode()},
                                       separators=(",", ":")) + "\n")
                for e in self._pending.values():
                    f.write(json.dumps(e, separators=(",", ":")) + "\n")
            if self._fd >= 0:
                os.close(self._fd)
                self._fd = -1
            os.replace(tmp, self.path)
            self._lines = len(self._mem) + len(self._pending)
        except OSError as e:
            log.warning("allocation journal compaction failed: %s", e)

    # -- answers ----------------------------------------------------------------------------
    def record(self, req, pod_uid: str, resp, key: str | None = None) -> None:
        key, t, blob = key or request_key(req), time.time(), resp.SerializeToString()
        with self._lock:
            self._mem[key] = (pod_uid, t, blob)
            self._mem.move_to_end(key)
            self._uids[pod_uid] = t
            while len(self._mem) > self.max_entries:
                _, (u, _, _) = self._mem.popitem(last=False)
                self._uids.pop(u, None)
            self._write({"k": key, "uid": pod_uid, "t": t, "resp": base64.b64encode(blob).decode()})

    def lookup(self, req, key: str | None = None) -> tuple[str, object] | None:
        key = key or request_key(req)
        with self._lock:
            hit = self._mem.get(key)
        if hit is None or time.time() - hit[1] > self.ttl_s:
            return None
        return hit[0], api.AllocateResponse.FromString(hit[2])

    def answered(self, uid: str) -> bool:
        """This plugin (or a previous instance, via the file) answered an Allocate for ``uid``
        recently, or still owes it a PATCH."""
        with self._lock:
            t = self._uids.get(uid)
            return uid in self._pending or (t is not None and time.time() - t <= self.ttl_s)

    def forget(self, uid: str) -> None:
        """``uid``'s answer went to another pod (placement truth): it is no longer answered."""
        with self._lock:
            self._uids.pop(uid, None)

    def answers(self) -> list[tuple[str, str, float, object]]:
        """(key, uid, time, AllocateResponse) of the answers still within the TTL."""
        now = time.time()
        with self._lock:
            items = [(k, u, t, b) for k, (u, t, b) in self._mem.items() if now - t <= self.ttl_s]
        return [(k, u, t, api.AllocateResponse.FromString(b)) for k, u, t, b in items]

    # -- write-behind patches ---------------------------------------------------------------
    def record_pending(self, req, pod_uid: str, resp, ns: str, name: str, ann: dict | None = None,
                       key: str | None = None) -> None:
        """A write-behind answer and its still-pending ASSIGNED patch, in one record/syscall."""
        key, t, blob = key or request_key(req), time.time(), resp.SerializeToString()
        pend = {"op": "patch", "uid": pod_uid, "ns": ns, "name": name, "ann": dict(ann or {}), "t": t}
        with self._lock:
            self._mem[key] = (pod_uid, t, blob)
            self._mem.move_to_end(key)
            self._uids[pod_uid] = t
            while len(self._mem) > self.max_entries:
                _, (u, _, _) = self._mem.popitem(last=False)
                self._uids.pop(u, None)
            self._pending[pod_uid] = pend
            self._write(pend | {"op": "answer+patch", "k": key, "resp": base64.b64encode(blob).decode()})

    def pending(self, uid: str, ns: str, name: str, ann: dict | None = None) -> None:
        rec = {"op": "patch", "uid": uid, "ns": ns, "name": name, "ann": dict(ann or {}), "t": time.time()}
        with self._lock:
            self._pending[uid] = rec
            self._write(rec)

    def landed(self, uid: str) -> None:
        with self._lock:
            if self._pending.pop(uid, None) is not None:
                self._write({"op": "landed", "uid": uid})

    def unlanded(self) -> list[dict]:
        with self._lock:
            return list(self._pending.values())

    def close(self):
        with self._lock:
            if self._fd >= 0:
                os.close(self._fd)
                self._fd = -1

    def __len__(self):
        return len(self._mem)
