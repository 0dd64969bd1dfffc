"""Allocate decision journal: idempotent answers to a retried admission.

The reference keeps no state (``allocate.go``): if the kubelet re-sends an Allocate after the
plugin already matched the pod and patched it ``ASSIGNED=true`` (an RPC deadline hit, a
plugin restart between the PATCH and the reply), the pod is no longer a candidate and the
retry fails with ``no-gpu-has-N``. This journal remembers recent decisions keyed by the
request's fake-device-ID set, in memory and optionally in an append-only JSON-lines file so
they survive a plugin restart, and the engine replays one only when its pod still exists on
this node *and is still Pending* — i.e. the kubelet is retrying that pod's admission. The
kubelet recycles freed fake IDs for new pods, so a key alone is never trusted: once the
journaled pod is gone or running, the entry is ignored and normal matching runs.
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
    def __init__(self, path: str | None = None, ttl_s: float = 120.0, max_entries: int = 4096):
        self.path, self.ttl_s, self.max_entries = path, ttl_s, max_entries
        self._mem: collections.OrderedDict[str, tuple[str, float, bytes]] = collections.OrderedDict()
        self._lock = threading.Lock()
        self._lines = 0
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
        for line in lines[-self.max_entries:]:
            try:
                e = json.loads(line)
                if now - e["t"] <= self.ttl_s:
                    self._mem[e["k"]] = (e["uid"], e["t"], base64.b64decode(e["resp"]))
                    self._mem.move_to_end(e["k"])
            except (ValueError, KeyError):
                continue
        self._lines = len(lines)
        log.info("allocation journal %s: %d recent decisions loaded", self.path, len(self._mem))

    def _append(self, key: str, uid: str, t: float, blob: bytes):
        os.makedirs(os.path.dirname(self.path) or ".", exist_ok=True)
        line = json.dumps({"k": key, "uid": uid, "t": t, "resp": base64.b64encode(blob).decode()})
        with open(self.path, "a") as f:
            f.write(line + "\n")
        self._lines += 1
        if self._lines > 2 * self.max_entries:
            self._compact()

    def _compact(self):
        tmp = self.path + ".tmp"
        with open(tmp, "w") as f:
            for k, (uid, t, blob) in self._mem.items():
                f.write(json.dumps({"k": k, "uid": uid, "t": t, "resp": base64.b64encode(blob).decode()}) + "\n")
        os.replace(tmp, self.path)
        self._lines = len(self._mem)

    # -- API --------------------------------------------------------------------------------
    def record(self, req, pod_uid: str, resp, key: str | None = None) -> None:
        key, t, blob = key or request_key(req), time.time(), resp.SerializeToString()
        with self._lock:
            self._mem[key] = (pod_uid, t, blob)
            self._mem.move_to_end(key)
            while len(self._mem) > self.max_entries:
                self._mem.popitem(last=False)
            if self.path:
                try:
                    self._append(key, pod_uid, t, blob)
                except OSError as e:
                    log.warning("allocation journal write failed: %s", e)

    def lookup(self, req, key: str | None = None) -> tuple[str, object] | None:
        key = key or request_key(req)
        with self._lock:
            hit = self._mem.get(key)
        if hit is None or time.time() - hit[1] > self.ttl_s:
            return None
        return hit[0], api.AllocateResponse.FromString(hit[2])

    def __len__(self):
        return len(self._mem)
