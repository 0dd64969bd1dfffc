"""Node-local pending-pod sources for Allocate (components C6 + C8 call sites).

Reference: every Allocate does a fresh LIST of ``spec.nodeName=<node>,status.phase=Pending``
pods (≤3 retries × 1 s, ``podmanager.go:227-245``) or, with ``--query-kubelet``, a GET of the
kubelet's ``/pods`` filtered client-side (≤8 retries × 100 ms then LIST fallback,
``podmanager.go:187-225``), dedupes by UID (``:273-291``), keeps "assumed" pods
(``podutils.go:78-119``) and sorts by assume time (``:326-347``).

``WatchCache`` is the MI355X build's main latency lever: a LIST+WATCH informer
of this node's pods, so the per-Allocate LIST becomes an in-memory lookup and only the
PATCH remains on the network path. Correctness under watch lag: a cache miss falls back to
one fresh LIST (``PodSource.candidates(fresh=True)``) and locally-written pods are folded
back into the cache from the PATCH response, so a just-assigned pod is never matched twice.
"""
from __future__ import annotations

import contextlib
import threading
import time

from .. import const
from ..utils import log
from . import objects as O
from .client import APIClient, APIError


def node_field_selector(node: str, pending_only: bool = False) -> str:
    s = f"spec.nodeName={node}"
    return s + ",status.phase=Pending" if pending_only else s


class PodSource:
    """Strategy interface: returns this node's pending pods."""

    def pending_pods(self, fresh: bool = False) -> list[dict]:
        raise NotImplementedError

    def node_pods(self) -> list[dict]:
        """Every non-terminated pod bound to this node, any phase (rare path: swap completion)."""
        return [p for p in self.pending_pods(fresh=True) if not O.is_terminated(p)]

    def observe(self, pod: dict) -> None:
        """Feed back an object we wrote (PATCH response)."""

    def get(self, uid: str) -> dict | None:
        """This node's live pod with ``uid`` (O(1) in the watch cache; a scan elsewhere)."""
        return next((p for p in self.node_pods() if O.uid(p) == uid), None)

    def get_pending(self, uid: str) -> dict | None:
        """This node's pod ``uid`` if it is Pending, else None."""
        p = self.get(uid)
        return p if p is not None and O.phase(p) == "Pending" else None

    @contextlib.contextmanager
    def allocate_view(self):
        """One Allocate's view: sources that fetch per call (LIST, kubelet GET) answer every
        ``pending_pods`` / ``get_pending`` inside the block from a single fetch — the
        reference's cost model is one LIST per Allocate (``allocate.go:63``), not one per
        lookup. A no-op for the watch cache."""
        yield

    def start(self):
        return self

    def stop(self):
        pass


class _PerCallSource(PodSource):
    """A source that fetches on every call, with a per-thread memo inside ``allocate_view``."""

    def __init__(self):
        self._memo = threading.local()

    @contextlib.contextmanager
    def allocate_view(self):
        m = self._memo
        outer = getattr(m, "on", False)
        m.on = True
        try:
            yield
        finally:
            if not outer:
                m.on, m.items = False, None

    def pending_pods(self, fresh: bool = False) -> list[dict]:
        m = self._memo
        if getattr(m, "on", False):
            if getattr(m, "items", None) is None:
                m.items = self._fetch_pending()
            return m.items
        return self._fetch_pending()

    def get_pending(self, uid: str) -> dict | None:
        return next((p for p in self.pending_pods() if O.uid(p) == uid), None)

    def _fetch_pending(self) -> list[dict]:
        raise NotImplementedError


class ListSource(_PerCallSource):
    """The reference's default path: LIST the apiserver on every call."""

    def __init__(self, client: APIClient, node: str, retries: int = 3, retry_sleep: float = 1.0):
        super().__init__()
        self.client, self.node, self.retries, self.retry_sleep = client, node, retries, retry_sleep

    def _fetch_pending(self) -> list[dict]:
        sel = node_field_selector(self.node, pending_only=True)
        err = None
        for i in range(self.retries + 1):
            try:
                items, _ = self.client.list_pods(field_selector=sel)
                return items
            except (APIError, OSError) as e:
                err = e
                if i < self.retries:
                    time.sleep(self.retry_sleep)
        raise RuntimeError(f"failed to get Pods assigned to node {self.node}: {err}")

    def node_pods(self) -> list[dict]:
        items, _ = self.client.list_pods(field_selector=node_field_selector(self.node))
        return [p for p in items if not O.is_terminated(p)]


class KubeletSource(_PerCallSource):
    """``--query-kubelet``: kubelet ``/pods`` then apiserver fallback.

    Unlike the reference, "no Pending pods" is a valid answer, not an error to retry 8 × 100 ms
    (SURVEY §2.4.9): we retry only transport errors, then fall back to the apiserver.
    """

    def __init__(self, kubelet_client, fallback: ListSource, retries: int = 8, retry_sleep: float = 0.1):
        super().__init__()
        self.kubelet, self.fallback, self.retries, self.retry_sleep = kubelet_client, fallback, retries, retry_sleep

    def _fetch_pending(self) -> list[dict]:
        for i in range(self.retries + 1):
            try:
                pods = self.kubelet.get_node_running_pods()
                return [p for p in pods if O.phase(p) == "Pending"]
            except Exception as e:  # noqa: BLE001 - transport errors of any kind
                log.warning("failed to get pending pod list from kubelet (%s), retry", e)
                time.sleep(self.retry_sleep)
        log.warning("not found from kubelet /pods api, start to list apiserver")
        return self.fallback._fetch_pending()

    def node_pods(self) -> list[dict]:
        try:
            return [p for p in self.kubelet.get_node_running_pods() if not O.is_terminated(p)]
        except Exception:  # noqa: BLE001
            return self.fallback.node_pods()


class PrebindWatch:
    """Pods the extender has placed on this node but not bound yet (label
    ``gpushare.amd.com/node=<node>``, ``spec.nodeName`` empty): ``on_pod(pod)`` for each, so the
    Allocate engine can prepare the pod's answer before the bind reaches the node's pod watch
    and, right behind it, the kubelet's Allocate. Pods placed by an extender that does not set
    the label are simply never seen here (the answer is prepared at the bind, as before).
    ``on_gone(pod)`` when a pod leaves that set (bound, deleted, relabelled: a watch's DELETED for
    an object that stops matching carries its previous state, so which one is not known here)."""

    def __init__(self, client: APIClient, node: str, on_pod, watch_timeout: int = 300, on_gone=None, trace=None):
        self.client, self.node, self.on_pod, self.watch_timeout = client, node, on_pod, watch_timeout
        self.on_gone = on_gone
        self.trace = trace          # trace(uid, "pre_read", ns): when the event's bytes arrived
        self._stop = threading.Event()
        self._conn: list = []
        self._thread = None
        self.events = 0

    def start(self) -> "PrebindWatch":
        self._thread = threading.Thread(target=self._run, name="pod-prebind-watch", daemon=True)
        self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        self.client.abort_watch(self._conn)

    def _run(self) -> None:
        backoff = 0.1
        while not self._stop.is_set():
            try:
                for ev in self.client.watch_pods("spec.nodeName=", None, self.watch_timeout, self._stop, self._conn,
                                                 label_selector=f"{const.POD_LABEL_NODE}={self.node}"):
                    typ, obj = ev.get("type"), ev.get("object") or {}
                    try:
                        if typ in ("ADDED", "MODIFIED") and not O.node_name(obj):
                            self.events += 1
                            if self.trace is not None and ev.get("_read_ns"):
                                self.trace(O.uid(obj), "pre_read", ev["_read_ns"])
                            self.on_pod(obj)
                        elif typ == "DELETED" and self.on_gone is not None:
                            self.on_gone(obj)
                    except Exception as e:  # noqa: BLE001 - preparing ahead is an optimisation
                        log.V(2).info("prebind: %s", e)
                backoff = 0.1
            except Exception as e:  # noqa: BLE001 - apiserver restart, expired watch
                if self._stop.is_set():
                    break
                log.V(2).info("prebind watch: %s", e)
                self._stop.wait(backoff)
                backoff = min(backoff * 2, 5.0)


class WatchCache(PodSource):
    """LIST+WATCH informer over ``spec.nodeName=<node>`` pods."""

    def __init__(self, client: APIClient, node: str, fallback: ListSource | None = None,
                 watch_timeout: int = 300, on_event=None):
        self.client, self.node = client, node
        self.fallback = fallback or ListSource(client, node, retries=1, retry_sleep=0.05)
        self.watch_timeout = watch_timeout
        self.on_event = on_event
        self._pods: dict[str, dict] = {}
        self._pending: dict[str, dict] = {}     # the Pending subset, so Allocate never scans Running pods
        self._lock = threading.Lock()
        # bumped on every change of the cached set; ``changed`` wakes consumers that precompute
        # from the cache (the Allocate engine's prepared answers)
        self.version = 0
        # bumped only when the Pending subset changes (what Allocate candidates are made of);
        # ``on_pending_change(version, pod, gone)`` runs under the cache lock at every bump (``pod``:
        # the one pod that joined, changed in or left (``gone``) the set; None after a relist),
        # so a consumer that answers from precomputed state (the native Allocate fast path)
        # never sees the cache ahead of the version it was told
        self.pending_version = 0
        self.on_pending_change = None
        self._pending_cv = threading.Condition(self._lock)
        self.changed = threading.Event()
        self._synced = threading.Event()
        self._stop = threading.Event()
        self._thread = None
        self._rv = ""
        self._conn: list = []
        self.relists = 0
        self.events = 0

    # -- informer loop --------------------------------------------------------------------
    def start(self):
        self._thread = threading.Thread(target=self._run, name="pod-watch", daemon=True)
        self._thread.start()
        return self

    def stop(self):
        self._stop.set()
        self.client.abort_watch(self._conn)

    def wait_synced(self, timeout: float = 10.0) -> bool:
        return self._synced.wait(timeout)

    def _relist(self):
        items, rv = self.client.list_pods(field_selector=node_field_selector(self.node))
        with self._lock:
            self._pods = {O.uid(p): p for p in items}
            self._pending = {u: p for u, p in self._pods.items() if O.phase(p) == "Pending"}
            self._rv = rv
            self.version += 1
            self._pending_bump()
        self.changed.set()
        self.relists += 1
        self._synced.set()

    def _apply(self, ev: dict):
        typ, obj = ev.get("type"), ev.get("object") or {}
        if typ == "BOOKMARK":
            self._rv = O.resource_version(obj) or self._rv
            return
        if typ == "ERROR":
            code = obj.get("code")
            raise APIError(code or 500, obj.get("reason", "watch error"), obj.get("message", ""), obj)
        u = O.uid(obj)
        with self._lock:
            if typ == "DELETED" or O.node_name(obj) != self.node:
                self._pods.pop(u, None)
                if self._pending.pop(u, None) is not None:
                    self._pending_bump(obj, gone=True)
                self.version += 1
            else:
                cur = self._pods.get(u)
                if cur is None or O.rv_int(O.resource_version(obj)) >= O.rv_int(O.resource_version(cur)):
                    self._put(u, obj)
            self._rv = O.resource_version(obj) or self._rv
        self.changed.set()
        self.events += 1
        if self.on_event:
            self.on_event(typ)

    def _run(self):
        backoff = 0.05
        while not self._stop.is_set():
            try:
                if not self._synced.is_set() or not self._rv:
                    self._relist()
                for ev in self.client.watch_pods(node_field_selector(self.node), self._rv,
                                                 self.watch_timeout, self._stop, self._conn):
                    self._apply(ev)
                backoff = 0.05
            except APIError as e:
                if e.gone:  # resourceVersion too old: relist
                    self._synced.clear()
                    self._rv = ""
                else:
                    log.warning("pod watch error: %s", e)
                    time.sleep(backoff)
                    backoff = min(backoff * 2, 5.0)
            except Exception as e:  # noqa: BLE001 - connection loss etc.
                if self._stop.is_set():
                    break
                log.warning("pod watch interrupted: %s", e)
                time.sleep(backoff)
                backoff = min(backoff * 2, 5.0)

    # -- PodSource ------------------------------------------------------------------------
    def pending_pods(self, fresh: bool = False) -> list[dict]:
        if fresh or not self._synced.is_set():
            items = self.fallback.pending_pods(fresh=True)
            for p in items:
                self.observe(p)
            return items
        with self._lock:
            return list(self._pending.values())

    def _pending_bump(self, pod: dict | None = None, gone: bool = False) -> None:
        """Caller holds the cache lock."""
        self.pending_version += 1
        hook = self.on_pending_change
        if hook is not None:
            hook(self.pending_version, pod, gone)
        self._pending_cv.notify_all()

    def wait_pending_change(self, version: int, timeout: float) -> bool:
        """Wait until the Pending set changed since ``version`` (or ``timeout``); True if it did."""
        with self._lock:
            return self._pending_cv.wait_for(lambda: self.pending_version != version, timeout)

    def _put(self, u: str, pod: dict) -> None:
        self.version += 1
        self._pods[u] = pod
        if O.phase(pod) == "Pending":
            self._pending[u] = pod
            self._pending_bump(pod)
        elif self._pending.pop(u, None) is not None:
            self._pending_bump(pod, gone=True)

    def observe(self, pod: dict) -> None:
        if not pod or O.node_name(pod) != self.node:
            return
        u = O.uid(pod)
        with self._lock:
            cur = self._pods.get(u)
            if cur is None or O.rv_int(O.resource_version(pod)) >= O.rv_int(O.resource_version(cur)):
                self._put(u, pod)
        self.changed.set()

    def get(self, uid: str) -> dict | None:
        if not self._synced.is_set():
            return super().get(uid)
        with self._lock:
            p = self._pods.get(uid)
        return None if p is None or O.is_terminated(p) else p

    def node_pods(self) -> list[dict]:
        if not self._synced.is_set():
            return self.fallback.node_pods()
        with self._lock:
            return [p for p in self._pods.values() if not O.is_terminated(p)]

    def snapshot(self) -> list[dict]:
        with self._lock:
            return list(self._pods.values())
