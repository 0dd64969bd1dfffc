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

The journal must survive the *process* (kill, crash, OOM, DaemonSet rollout), not the node:
a node crash takes the pods' containers down with it. Records are JSON lines appended into a
``MAP_SHARED`` mapping of a pre-sized file (zero bytes mark the end): a store into the page
cache survives the process exactly like a ``write(2)`` without ``fsync`` does, and costs no
system call on the Allocate path — a syscall there hands the GIL to whichever plugin thread is
busy (the informer decoding the very pod's watch events) and the kubelet waits for it. A
write-behind answer and its pending patch share one record (``{"op": "answer+patch", ...}``).
When the mapping is full the live records are compacted into a fresh file (atomic rename).
"""
from __future__ import annotations

import base64
import collections
import hashlib
import json
import mmap
import os
import threading
import time

from ..api import v1beta1 as api
from ..utils import log


def request_key(req) -> str:
    body = "\x1e".join("\x1f".join(sorted(c.devices_ids)) for c in req.container_requests)
    return hashlib.sha1(body.encode()).hexdigest()


def ids_key(ids) -> str:
    """``request_key`` of a one-container request with these fake IDs."""
    return hashlib.sha1("\x1f".join(sorted(ids)).encode()).hexdigest()


class AllocJournal:
    def __init__(self, path: str | None = None, ttl_s: float = 120.0, max_entries: int = 4096,
                 pending_ttl_s: float = 24 * 3600.0, map_bytes: int = 16 << 20):
        self.path, self.ttl_s, self.max_entries = path, ttl_s, max_entries
        self.pending_ttl_s = pending_ttl_s
        self.map_bytes = map_bytes
        self._mm: mmap.mmap | None = None
        self._off = 0
        self._touched = 0
        self._mem: collections.OrderedDict[str, tuple[str, float, bytes]] = collections.OrderedDict()
        self._uids: dict[str, float] = {}                       # pod uid -> time of its answer
        self._pending: collections.OrderedDict[str, dict] = collections.OrderedDict()  # uid -> patch
        self._lock = threading.Lock()
        self._lines = 0
        # fake ID -> key of the journaled answer that holds it, for answers whose pod may still
        # be retried (Pending): lets the Allocate fast path rule a replay out with one dict probe
        self._by_id: dict[str, str] = {}
        self._ids_of: dict[str, tuple[str, tuple]] = {}       # uid -> (key, ids)
        self._legacy_until = 0.0       # answers loaded without their IDs: probe says "maybe"
        if path:
            self._load()

    # -- persistence ------------------------------------------------------------------------
    def fast_path(self) -> str:
        """The native server's journal file (native/dpserver): its Allocate answers, in the
        same record format, written before each reply."""
        return self.path + ".fast"

    @staticmethod
    def _read_records(path: str) -> list[str] | None:
        try:
            with open(path, "rb") as f:
                raw = f.read()
        except FileNotFoundError:
            return None
        end = raw.find(b"\0")                 # the mapped file's unused tail is zero
        return (raw if end < 0 else raw[:end]).decode(errors="replace").splitlines()

    def _load(self):
        main = self._read_records(self.path)
        fast = self._read_records(self.fast_path())
        if main is None and fast is None:
            return
        # the native answers first: a "landed" record in the main file then closes their patch
        lines = (fast or []) + (main or [])
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
                    ids = tuple(e["ids"].split(",")) if e.get("ids") else None
                    if e.get("req"):
                        r = api.AllocateRequest.FromString(base64.b64decode(e["req"]))
                        ids = tuple(i for c in r.container_requests for i in c.devices_ids)
                    k = e.get("k") or ids_key(ids)
                    self._mem[k] = (e["uid"], e["t"], base64.b64decode(e["resp"]))
                    self._mem.move_to_end(k)
                    self._uids[e["uid"]] = e["t"]
                    if ids:
                        self._index(k, e["uid"], ids)
                    else:
                        self._legacy_until = max(self._legacy_until, e["t"] + self.ttl_s)
            except (ValueError, KeyError, TypeError):
                continue                                          # a torn last line after a crash
        while len(self._mem) > self.max_entries:
            self._mem.popitem(last=False)
        self._lines = len(lines)
        log.info("allocation journal %s: %d recent decisions, %d unlanded patches loaded", self.path,
                 len(self._mem), len(self._pending))
        self._compact()

    def _map(self):
        """Map the journal file (grown to ``map_bytes``) and find the end of its records."""
        os.makedirs(os.path.dirname(self.path) or ".", exist_ok=True)
        fd = os.open(self.path, os.O_RDWR | os.O_CREAT | os.O_CLOEXEC, 0o600)
        try:
            size = max(self.map_bytes, os.fstat(fd).st_size)
            os.ftruncate(fd, size)
            try:
                os.posix_fallocate(fd, 0, size)   # blocks reserved now, not at a page's first store
            except OSError:
                pass
            self._mm = mmap.mmap(fd, size, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
        finally:
            os.close(fd)
        end = self._mm.find(b"\0")
        self._off = len(self._mm) if end < 0 else end
        self._touched = self._off
        self._prefault()

    def prefault(self, ahead: int = 256 << 10) -> None:
        """Fault in the pages the next records will land on (off the Allocate path: the
        patcher calls it), so an answer's store never takes the first-write page fault. Under
        the journal lock: a compaction on a gRPC thread replaces the mapping."""
        with self._lock:
            try:
                self._prefault(ahead)
            except ValueError:           # mapping closed by a failed compaction: next write remaps
                pass

    def _prefault(self, ahead: int = 256 << 10) -> None:
        mm = self._mm
        if mm is None:
            return
        end = min(len(mm), self._off + ahead)
        pos = max(self._touched, self._off)
        pos -= pos % mmap.PAGESIZE
        while pos < end:
            if pos >= self._off:
                mm[pos] = mm[pos]          # a store: write fault now (the byte is still zero)
            pos += mmap.PAGESIZE
        self._touched = max(self._touched, end)

    def _write(self, rec: dict):
        if not self.path:
            return
        data = (json.dumps(rec, separators=(",", ":")) + "\n").encode()
        try:
            if self._mm is None:
                self._map()
            if self._off + len(data) > len(self._mm):
                self._compact(extra=data)
                return
            self._mm[self._off:self._off + len(data)] = data
            self._off += len(data)
            self._lines += 1
        except (OSError, ValueError) as e:
            log.warning("allocation journal write failed: %s", e)

    def _compact(self, extra: bytes = b""):
        """Rewrite the live records (+ ``extra``) into a fresh mapped file, atomically."""
        if not self.path:
            return
        tmp = self.path + ".tmp"
        try:
            os.makedirs(os.path.dirname(self.path) or ".", exist_ok=True)
            parts = [json.dumps({"k": k, "uid": uid, "t": t, "resp": base64.b64encode(blob).decode(),
                                 **({"ids": ",".join(self._ids_of[uid][1])} if uid in self._ids_of else {})},
                                separators=(",", ":")).encode() + b"\n" for k, (uid, t, blob) in self._mem.items()]
            parts += [json.dumps(e, separators=(",", ":")).encode() + b"\n" for e in self._pending.values()]
            body = b"".join(parts) + extra
            if len(body) * 2 > self.map_bytes:      # keep room for the next records
                self.map_bytes = len(body) * 2
            with open(tmp, "wb") as f:
                f.write(body)
                f.truncate(self.map_bytes)
            if self._mm is not None:
                self._mm.close()
                self._mm = None
            os.replace(tmp, self.path)
            self._map()
            self._lines = len(self._mem) + len(self._pending) + (1 if extra else 0)
        except (OSError, ValueError) as e:
            log.warning("allocation journal compaction failed: %s", e)

    # -- replay index -----------------------------------------------------------------------
    def _index(self, key: str, uid: str, ids) -> None:
        old = self._ids_of.pop(uid, None)
        if old is not None:
            for i in old[1]:
                if self._by_id.get(i) == old[0]:
                    del self._by_id[i]
        self._ids_of[uid] = (key, tuple(ids))
        for i in ids:
            self._by_id[i] = key

    def maybe_replay(self, device_id: str) -> bool:
        """False = no journaled answer of a possibly-retried pod holds this fake ID (so the
        request is not a replay); True = check properly (``lookup``)."""
        return device_id in self._by_id or time.time() < self._legacy_until

    def prune_index(self, keep_uids) -> None:
        """Forget the IDs of answers whose pod can no longer be retried (not Pending any more,
        or gone): the kubelet recycles those IDs for new pods at once."""
        with self._lock:
            for u in [u for u in self._ids_of if u not in keep_uids]:
                key, ids = self._ids_of.pop(u)
                for i in ids:
                    if self._by_id.get(i) == key:
                        del self._by_id[i]

    def indexed_uids(self) -> list[str]:
        with self._lock:
            return list(self._ids_of)

    def replay_ids(self) -> list[str]:
        """Every fake ID ``maybe_replay`` answers True for (the native fast table's replay set)."""
        with self._lock:
            return list(self._by_id)

    def note_fast(self, pod_uid: str, ns: str, name: str, t: float, ids) -> None:
        """A native-server answer (its record is already in the fast file): the in-memory state
        ``record_fast`` would have set."""
        pend = {"op": "patch", "uid": pod_uid, "ns": ns, "name": name, "ann": {}, "t": t}
        with self._lock:
            for i in ids:
                self._by_id.setdefault(i, "")
            self._uids[pod_uid] = t
            self._pending[pod_uid] = pend

    def compact(self) -> None:
        """Rewrite the live records now (the native fast file is then redundant)."""
        with self._lock:
            self._compact()

    # -- answers ----------------------------------------------------------------------------
    def record(self, req, pod_uid: str, resp, key: str | None = None) -> None:
        key, t, blob = key or request_key(req), time.time(), resp.SerializeToString()
        ids = [i for c in req.container_requests for i in c.devices_ids]
        with self._lock:
            self._mem[key] = (pod_uid, t, blob)
            self._mem.move_to_end(key)
            self._uids[pod_uid] = t
            self._index(key, pod_uid, ids)
            while len(self._mem) > self.max_entries:
                _, (u, _, _) = self._mem.popitem(last=False)
                self._uids.pop(u, None)
            self._write({"k": key, "uid": pod_uid, "t": t, "resp": base64.b64encode(blob).decode()})

    def record_fast(self, pod_uid: str, ns: str, name: str, head: bytes, req_bytes: bytes, ids=()) -> float:
        """Allocate fast path: the answer + pending-patch record from its prepared ``head``
        (everything but the time and the request) — one store into the mapping. The request
        goes in as its wire bytes; the answer itself is indexed off the hot path
        (``index_answer``), but its fake ``ids`` are marked at once, so a kubelet retry of the
        same set that arrives before that sees "maybe a replay" and takes the full path (which
        indexes first). Returns the record's time."""
        t = time.time()
        pend = {"op": "patch", "uid": pod_uid, "ns": ns, "name": name, "ann": {}, "t": t}
        data = b"".join((head, repr(t).encode(), b',"req":"', base64.b64encode(req_bytes), b'"}\n'))
        with self._lock:
            mark = self._by_id
            for i in ids:
                mark[i] = ""             # placeholder key: index_answer overwrites it
            self._uids[pod_uid] = t
            self._pending[pod_uid] = pend
            if self.path:
                try:
                    if self._mm is None:
                        self._map()
                    if self._off + len(data) <= len(self._mm):
                        self._mm[self._off:self._off + len(data)] = data
                        self._off += len(data)
                        self._lines += 1
                    else:
                        self._compact(extra=data)
                except (OSError, ValueError) as e:
                    log.warning("allocation journal write failed: %s", e)
        return t

    @staticmethod
    def fast_head(pod_uid: str, ns: str, name: str, resp_bytes: bytes) -> bytes:
        """The constant part of a fast-path record (see ``record_fast``)."""
        # the same bytes json.dumps(..., separators=(",", ":")) writes, without its dict walk
        # (this runs on the pod watch thread for every newly bound pod)
        q = json.encoder.encode_basestring_ascii
        return (f'{{"op":"answer+patch","uid":{q(pod_uid)},"ns":{q(ns)},"name":{q(name)},"ann":{{}},'
                f'"resp":"{base64.b64encode(resp_bytes).decode()}","t":').encode()

    def index_answer(self, key: str, pod_uid: str, t: float, blob: bytes, ids) -> None:
        with self._lock:
            self._mem[key] = (pod_uid, t, blob)
            self._mem.move_to_end(key)
            self._index(key, pod_uid, ids)
            while len(self._mem) > self.max_entries:
                _, (u, _, _) = self._mem.popitem(last=False)
                self._uids.pop(u, None)

    def lookup(self, req, key: str | None = None) -> tuple[str, object] | None:
        """(pod uid, the journaled answer) for this request's fake-ID set, or None. The answer
        is returned as a zero-argument callable: parsing it is only worth it on a replay."""
        key = key or request_key(req)
        with self._lock:
            hit = self._mem.get(key)
        if hit is None or time.time() - hit[1] > self.ttl_s:
            return None
        blob = hit[2]
        return hit[0], lambda: api.AllocateResponse.FromString(blob)

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
            self._index(key, pod_uid, [i for c in req.container_requests for i in c.devices_ids])
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
            if self._mm is not None:
                self._mm.close()
                self._mm = None

    def __len__(self):
        return len(self._mem)
