"""Lease-based leader election for the scheduler extender (``coordination.k8s.io/v1`` Lease).

The extender keeps its per-GPU ledger in memory, so two instances answering ``bind`` at once
could both hand out the same HBM. The reference's extender runs as one replica; here
``--leader-elect`` lets several replicas run with exactly one serving: every replica watches
the pods and keeps a warm ledger, the leader answers ``filter`` / ``bind`` and reports ready
(``/readyz``), the others answer 503 and stay out of the Service's endpoints. A replica that
becomes leader re-syncs the ledger from the pods' annotations first (``on_start``), so the
binds the previous leader made are all counted.

The algorithm is the one Kubernetes components use (client-go ``leaderelection``):

* the Lease names a holder and a duration; a replica may take it when it is free, released, or
  its record has not changed for ``leaseDurationSeconds`` as measured on the replica's **own**
  clock since it last saw the record change — never by comparing the holder's timestamps with
  local time, so clock skew between hosts cannot hand the lease over early;
* every write is a compare-and-swap on the Lease's ``resourceVersion`` (a lost race is a 409);
* the leader renews every ``retry_s``; if it has not renewed for ``renew_s`` (< ``lease_s``),
  it steps down before any other replica can consider the lease expired. A renewal counts from
  the moment it was *started* (a slow PUT must not extend the leader's own view of its term),
  and each of its requests gives up after ``(renew_s - retry_s) / 2`` (client-go's
  RenewDeadline), so a stalled apiserver cannot keep a stale leader serving;
* a follower dates what it observed from the moment the GET *returned*, never earlier;
* a graceful stop releases the lease (empty holder), so a follower takes over at its next try.
"""
from __future__ import annotations

import datetime
import threading
import time

from ..cluster.client import APIError
from ..utils import log


def _micro_time(t: float | None = None) -> str:
    d = datetime.datetime.fromtimestamp(time.time() if t is None else t, datetime.timezone.utc)
    return d.strftime("%Y-%m-%dT%H:%M:%S.%fZ")


class LeaderElector:
    def __init__(self, client, namespace: str, name: str, identity: str, lease_s: float = 15.0,
                 renew_s: float = 10.0, retry_s: float = 2.0, on_start=None, on_stop=None, clock=time.monotonic):
        if not 0 < retry_s < renew_s < lease_s:
            raise ValueError("leader election needs 0 < retry < renew deadline < lease duration")
        self.client, self.namespace, self.name, self.identity = client, namespace, name, identity
        self.lease_s, self.renew_s, self.retry_s = lease_s, renew_s, retry_s
        self.on_start, self.on_stop = on_start, on_stop
        self.clock = clock
        self._leader = False
        self._last_renew = 0.0
        self._observed: tuple | None = None      # (holder, renewTime, resourceVersion) last seen
        self._observed_at = 0.0                  # local clock when it last changed
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None
        self._mu = threading.Lock()              # leadership transitions (start/stop callbacks)
        self.transitions = 0                     # times this replica became leader

    # -- state ---------------------------------------------------------------------------------
    def is_leader(self) -> bool:
        return self._leader and self.clock() - self._last_renew < self.renew_s

    def holder(self) -> str | None:
        return self._observed[0] if self._observed else None

    # -- the Lease -------------------------------------------------------------------------------
    def _path(self) -> str:
        return f"/apis/coordination.k8s.io/v1/namespaces/{self.namespace}/leases/{self.name}"

    def _spec(self, acquire: str, transitions: int) -> dict:
        return {"holderIdentity": self.identity, "leaseDurationSeconds": max(1, int(round(self.lease_s))),
                "acquireTime": acquire, "renewTime": _micro_time(), "leaseTransitions": transitions}

    def _req(self, method: str, path: str, body=None):
        return self.client.request(method, path, body=body, timeout=max(0.1, (self.renew_s - self.retry_s) / 2))

    def try_acquire_or_renew(self) -> bool:
        """One attempt; True when this replica holds the lease afterwards."""
        try:
            lease = self._req("GET", self._path())
        except APIError as e:
            if not e.not_found:
                raise
            body = {"apiVersion": "coordination.k8s.io/v1", "kind": "Lease",
                    "metadata": {"name": self.name, "namespace": self.namespace},
                    "spec": self._spec(_micro_time(), 0)}
            try:
                made = self._req("POST", f"/apis/coordination.k8s.io/v1/namespaces/{self.namespace}/leases", body=body)
            except APIError as e2:
                if e2.status == 409:             # another replica created it first
                    return False
                raise
            self._see(made, self.clock())
            return True
        now = self.clock()                       # observed now that the GET has returned
        spec = lease.get("spec") or {}
        self._see(lease, now)
        holder = spec.get("holderIdentity") or ""
        duration = float(spec.get("leaseDurationSeconds") or self.lease_s)
        if holder and holder != self.identity and now - self._observed_at < duration:
            return False                         # held, and alive as far as this replica has seen
        mine = holder == self.identity
        new = dict(lease)
        new["metadata"] = {k: v for k, v in (lease.get("metadata") or {}).items()
                           if k in ("name", "namespace", "uid", "resourceVersion")}
        new["spec"] = self._spec(spec.get("acquireTime") if mine and spec.get("acquireTime") else _micro_time(),
                                 int(spec.get("leaseTransitions") or 0) + (0 if mine else 1))
        try:
            upd = self._req("PUT", self._path(), body=new)
        except APIError as e:
            if e.status == 409:                  # someone wrote it since the GET
                return False
            raise
        self._see(upd, self.clock())
        return True

    def _see(self, lease: dict, now: float) -> None:
        spec = lease.get("spec") or {}
        rec = (spec.get("holderIdentity") or "", spec.get("renewTime"),
               (lease.get("metadata") or {}).get("resourceVersion"))
        if rec != self._observed:
            self._observed, self._observed_at = rec, now

    def release(self) -> None:
        """Give the lease up (graceful stop): empty holder, so the next try anywhere takes it."""
        try:
            lease = self.client.request("GET", self._path())
            if ((lease.get("spec") or {}).get("holderIdentity") or "") != self.identity:
                return
            lease["spec"] = dict(lease["spec"], holderIdentity="", leaseDurationSeconds=1, renewTime=_micro_time())
            self.client.request("PUT", self._path(), body=lease)
        except Exception as e:  # noqa: BLE001 - the lease then simply expires
            log.warning("leader election: release failed: %s", e)

    # -- the loop --------------------------------------------------------------------------------
    def _set(self, leader: bool) -> None:
        with self._mu:
            if leader == self._leader:
                return
            if leader:
                # ready only after the callback: a new leader re-syncs its ledger before it serves
                if self.on_start:
                    self.on_start()
                self._leader = True
                self.transitions += 1
                log.info("leader election: %s is now the leader of %s/%s", self.identity, self.namespace, self.name)
            else:
                self._leader = False
                log.warning("leader election: %s stopped leading %s/%s", self.identity, self.namespace, self.name)
                if self.on_stop:
                    self.on_stop()

    def step(self) -> None:
        """One round of the loop (tests drive it directly)."""
        started = self.clock()                   # a renewal's term counts from its start
        try:
            ok = self.try_acquire_or_renew()
        except Exception as e:  # noqa: BLE001 - apiserver unreachable: count it as a failed renew
            log.V(2).info("leader election: %s", e)
            ok = False
        now = self.clock()
        if ok:
            self._last_renew = started
            if not self._leader:
                try:
                    self._set(True)
                except Exception as e:  # noqa: BLE001 - could not get ready: give the lease back
                    log.error("leader election: becoming leader failed (%s); releasing", e)
                    self.release()
        elif self._leader and now - self._last_renew >= self.renew_s:
            self._set(False)

    def run(self) -> None:
        while not self._stop.is_set():
            self.step()
            self._stop.wait(self.retry_s)

    def start(self) -> "LeaderElector":
        self._thread = threading.Thread(target=self.run, name="leader-election", daemon=True)
        self._thread.start()
        return self

    def stop(self, release: bool = True) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)
        if self._leader:
            self._set(False)
            if release:
                self.release()
