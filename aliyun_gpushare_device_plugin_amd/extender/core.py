"""gpushare-scheduler-extender protocol implementation for MI355X nodes (deployable: ``cli/extender.py``,
``deploy/scheduler-extender.yaml``; the simulator drives the same class in-process).

The reference plugin's partner extender is a separate Go project (linked from the reference
``README.md:14``), not in ``/root/reference`` and not buildable here. What the plugin relies on
is inferred from what it consumes: per-GPU capacity = node ``allocatable[gpu-mem]
/ allocatable[gpu-count]`` (the inspect arithmetic, ``cmd/inspect/nodeinfo.go:116,146``); the
extender picks a node and a GPU index, writes ``ALIYUN_COM_GPU_MEM_IDX/_POD/_ASSUME_TIME`` and
``_ASSIGNED="false"``, then binds.

It places pods with a best-fit bin-packing policy — jointly for the queue of unscheduled pods
it knows about (``extender/packing.py``: online best fit strands HBM when mixed sizes arrive in
an unlucky order, the joint plan does not; a pod the plan leaves out only uses room the plan
does not hold for the others) — keeps its per-GPU ledger like the real extender's cache, and
adds the MI355X capability the north star asks for: pods labelled
``gpushare.amd.com/tp-group=<name>`` with ``…/tp-size=<k>`` are placed as a group on k distinct
GPUs that are pairwise one-hop xGMI per the topology annotation the plugin exports
(``parallel/topology.py``). It serves the extender HTTP routes (``/gpushare-scheduler/filter``
and ``/bind``).

Like the real extender's pod informer, ``update(pod)`` re-accounts a pod whose annotations
changed (the plugin's placement-truth rewrite of ``IDX`` / the allocation JSON, see
``alloc/placement.py``) and ``forget`` drops a deleted or finished one; ``watch()`` drives both
from an apiserver pod watch. The ledger holds no state of its own: a restarted extender
rebuilds it from the pods' annotations (``sync``), placement-truth rewrites included.
"""
from __future__ import annotations

import dataclasses
import http.server
import json
import socketserver
import threading
import time

from .. import const
from ..alloc import annotations as A
from ..cluster import nodestatus, objects as O
from ..cluster.client import APIClient
from ..parallel import topology as T

TP_GROUP_LABEL = "gpushare.amd.com/tp-group"
TP_SIZE_LABEL = "gpushare.amd.com/tp-size"


@dataclasses.dataclass
class NodeState:
    name: str
    gpu_count: int
    per_gpu: int
    used: list
    topology: dict | None
    healthy: list

    def free(self) -> list[int]:
        return [(self.per_gpu - u) if h else -1 for u, h in zip(self.used, self.healthy)]


class Extender:
    def __init__(self, client: APIClient, policy: str = "binpack", group_ttl_s: float = 300.0):
        self.client = client
        self.policy = policy
        self.nodes: dict[str, NodeState] = {}
        self._placed: dict[str, tuple] = {}   # pod uid -> (node, [(gpu, units)])
        # TP groups bound one member at a time through the HTTP bind route: the whole group's
        # xGMI clique is reserved when its first member binds (group -> reservation)
        self._groups: dict[str, dict] = {}
        self.group_ttl_s = group_ttl_s
        # the pending queue (unscheduled gpu-mem pods, not TP groups) and its joint placement
        self._pending: dict[str, dict] = {}
        self._plan: dict[str, tuple[str, int]] = {}
        self._plan_res: dict[tuple[str, int], int] = {}   # (node, gpu) -> HBM the plan holds there
        self._unplanned: dict[str, None] = {}             # queued since the last plan (arrival order)
        self._plan_at = 0.0
        self.plan_budget = 50_000
        self.plan_deadline_s = 0.05
        # queues up to joint_max pods are re-planned jointly on every arrival; a longer queue at
        # most every replan_interval_s, arrivals in between going best fit into the room the
        # plan leaves (a full plan of a long queue is best fit anyway: packing.EXACT_MAX_ITEMS)
        self.joint_max = 128
        self.replan_interval_s = 1.0
        self.plan_enabled = True
        self._lock = threading.Lock()
        self.elector = None                   # extender/leader.py LeaderElector with --leader-elect
        self._touched: dict[str, float] = {}  # pod uid -> when the ledger entry last changed here

    def serving(self) -> bool:
        """Whether this replica answers filter / bind: always without leader election, else
        only while it holds the lease."""
        return self.elector is None or self.elector.is_leader()

    # -- cache ----------------------------------------------------------------------------
    def _touch(self, uid: str) -> None:
        """A ledger change made here (caller holds the lock): a re-sync whose LIST started
        earlier keeps it instead of the LIST's older view of that pod."""
        self._touched[uid] = time.monotonic()

    def sync(self):
        """Rebuild the ledger from the apiserver (extender cache warm-up, periodic resync). The
        LISTs run outside the lock, so filter / bind keep going meanwhile; what changed here
        after they started (binds, informer updates, deletions) wins over what they returned."""
        t_fetch = time.monotonic()
        node_list = self.client.list_nodes()
        pods, _ = self.client.list_pods()
        with self._lock:
            recent = {u for u, t in self._touched.items() if t >= t_fetch}
            old_placed = self._placed
            self.nodes.clear()
            self._placed = {}
            for n in node_list:
                cnt = O.node_allocatable(n, const.RESOURCE_COUNT)
                mem = O.node_allocatable(n, const.RESOURCE_NAME)
                cap = O.node_capacity(n, const.RESOURCE_NAME) or mem
                if cnt <= 0 or cap <= 0:
                    continue
                health = json.loads(O.annotations(n).get(const.NODE_ANNOTATION_HEALTH, "{}") or "{}")
                healthy = [bool((health.get(str(i)) or {}).get("healthy", True)) for i in range(cnt)]
                self.nodes[O.name(n)] = NodeState(O.name(n), cnt, cap // cnt, [0] * cnt,
                                                  nodestatus.read_topology(n), healthy)
            for p in pods:
                if O.is_terminated(p) or not O.node_name(p) or O.uid(p) in recent:
                    continue
                st = self.nodes.get(O.node_name(p))
                if st is None or O.gpu_mem_of_pod(p) <= 0:
                    continue
                alloc = A.allocation_from_annotation(p) or {A.gpu_id_from_annotation(p): O.gpu_mem_of_pod(p)}
                parts = []
                for g, mem in alloc.items():
                    if 0 <= g < st.gpu_count:
                        st.used[g] += mem
                        parts.append((g, mem))
                self._placed[O.uid(p)] = (st.name, parts)
            for u in recent:                     # newer than the LIST: as this replica has it
                node, parts = old_placed.get(u, (None, ()))
                st = self.nodes.get(node)
                if st is None:
                    continue
                for g, mem in parts:
                    if 0 <= g < st.gpu_count:
                        st.used[g] += mem
                self._placed[u] = (node, list(parts))
            self._touched = {u: t for u, t in self._touched.items() if t >= t_fetch}
            for r in self._groups.values():      # reserved slots of TP groups still binding
                st = self.nodes.get(r["node"])
                for g in (r["free"] if st else []):
                    st.used[g] += r["req"]

    # -- the pending queue and its joint plan -----------------------------------------------
    def note_pending(self, pod: dict) -> None:
        """An unscheduled pod asking for gpu-mem (pod informer ADDED / MODIFIED, or the
        simulator's create): it joins the queue the next placement plans for."""
        if (O.node_name(pod) or O.gpu_mem_of_pod(pod) <= 0 or O.is_terminated(pod) or O.deleting(pod)
                or self._group_of(pod) is not None):
            return
        with self._lock:
            if O.uid(pod) not in self._pending:
                self._pending[O.uid(pod)] = pod
                self._unplanned[O.uid(pod)] = None

    def _drop_pending_locked(self, uid: str) -> None:
        pod = self._pending.pop(uid, None)
        if pod is not None:
            self._unplanned.pop(uid, None)
            where = self._plan.pop(uid, None)
            if where is not None:
                left = self._plan_res.get(where, 0) - O.gpu_mem_of_pod(pod)
                if left > 0:
                    self._plan_res[where] = left
                else:
                    self._plan_res.pop(where, None)

    def _replan_locked(self) -> None:
        """Joint best placement of the queued pods onto the GPUs' free HBM (extender/packing.py).
        Runs only when pods joined the queue since the last plan; a pod the plan left out does
        not trigger another one."""
        if not self.plan_enabled or self.policy != "binpack" or not self._unplanned:
            return
        from .packing import _Buckets, pack

        bins, free = [], []
        for name, st in sorted(self.nodes.items()):
            for i, f in enumerate(st.free()):
                if f > 0:
                    bins.append((name, i))
                    free.append(f)
        now = time.monotonic()
        if len(self._pending) <= self.joint_max or now - self._plan_at >= self.replan_interval_s:
            uids = list(self._pending)
            sizes = [O.gpu_mem_of_pod(self._pending[u]) for u in uids]
            assign = pack(free, sizes, self.plan_budget, self.plan_deadline_s)
            self._plan, self._plan_res = {}, {}
            for u, a, sz in zip(uids, assign, sizes):
                if a is not None:
                    self._plan[u] = bins[a]
                    self._plan_res[bins[a]] = self._plan_res.get(bins[a], 0) + sz
            self._plan_at = now
        else:
            # the newcomers, best fit into what the current plan leaves free
            bk = _Buckets([f - self._plan_res.get(b, 0) for b, f in zip(bins, free)])
            for u in self._unplanned:
                sz = O.gpu_mem_of_pod(self._pending[u])
                f = bk.best(sz)
                if f is None or sz <= 0:
                    continue
                a = bk.take(f)
                bk.put(f - sz, a)
                self._plan[u] = bins[a]
                self._plan_res[bins[a]] = self._plan_res.get(bins[a], 0) + sz
        self._unplanned.clear()

    def _planned_locked(self, pod: dict, node_names=None) -> tuple[str, int] | None:
        u = O.uid(pod)
        if u not in self._pending:
            return None
        self._replan_locked()
        for attempt in (0, 1):
            choice = self._plan.get(u)
            if choice is None or (node_names is not None and choice[0] not in node_names):
                return None
            st = self.nodes.get(choice[0])
            if st is not None and st.free()[choice[1]] >= O.gpu_mem_of_pod(pod):
                return choice
            if attempt == 0:
                # the room the plan counted on went elsewhere (a pod placed outside the queue,
                # a node re-synced): plan the whole queue again now
                self._unplanned.update(dict.fromkeys(self._pending))
                self._plan_at = 0.0
                self._replan_locked()
        return None

    def forget(self, pod: dict):
        with self._lock:
            self._drop_pending_locked(O.uid(pod))
            self._forget_locked(O.uid(pod))

    def _forget_locked(self, uid: str):
        self._touch(uid)
        placed = self._placed.pop(uid, None)
        if placed:
            st = self.nodes.get(placed[0])
            if st:
                for g, mem in placed[1]:
                    st.used[g] -= mem

    @staticmethod
    def _parts_from_annotations(pod: dict, st: NodeState) -> list | None:
        if A.is_assumed_pod(pod) or A.is_assigned_pod(pod) or A.allocation_from_annotation(pod):
            alloc = A.allocation_from_annotation(pod) or {A.gpu_id_from_annotation(pod): O.gpu_mem_of_pod(pod)}
            return [(g, mem) for g, mem in alloc.items() if 0 <= g < st.gpu_count]
        return None

    def update(self, pod: dict):
        """Pod informer update: re-account the pod from its (possibly rewritten) annotations."""
        if not O.node_name(pod):
            self.note_pending(pod)
            return
        with self._lock:
            u = O.uid(pod)
            self._drop_pending_locked(u)
            if O.is_terminated(pod) or O.deleting(pod):
                self._forget_locked(u)
                return
            st = self.nodes.get(O.node_name(pod))
            if st is None or O.gpu_mem_of_pod(pod) <= 0:
                return
            parts = self._parts_from_annotations(pod, st)
            if parts is None or (u in self._placed and self._placed[u] == (st.name, parts)):
                return
            self._forget_locked(u)
            for g, mem in parts:
                st.used[g] += mem
            self._placed[u] = (st.name, parts)
            self._touch(u)

    def watch(self) -> "Extender":
        """Follow pod updates and deletions from the apiserver (background thread)."""
        self._watch_stop = threading.Event()
        self._watch_holder: list = []

        def loop():
            rv = None
            while not self._watch_stop.is_set():
                try:
                    if rv is None:
                        _, rv = self.client.list_pods()
                    for ev in self.client.watch_pods(resource_version=rv, stop=self._watch_stop,
                                                     holder=self._watch_holder):
                        obj = ev.get("object") or {}
                        rv = (obj.get("metadata") or {}).get("resourceVersion", rv)
                        if ev.get("type") == "DELETED":
                            self.forget(obj)
                        elif ev.get("type") in ("MODIFIED", "ADDED"):
                            self.update(obj)
                except Exception:  # noqa: BLE001 - expired RV, apiserver restart: re-list
                    rv = None
                    self._watch_stop.wait(0.1)

        threading.Thread(target=loop, name="extender-watch", daemon=True).start()
        return self

    def stop_watch(self):
        if getattr(self, "_watch_stop", None) is not None:
            self._watch_stop.set()
            self.client.abort_watch(self._watch_holder)

    # -- scheduling -----------------------------------------------------------------------
    def _fits(self, st: NodeState, req: int) -> list[int]:
        return [i for i, f in enumerate(st.free()) if f >= req]

    def filter(self, pod: dict, node_names: list[str] | None = None) -> list[str]:
        req = O.gpu_mem_of_pod(pod)
        with self._lock:
            names = node_names if node_names is not None else list(self.nodes)
            if self._group_of(pod) is not None:
                self._expire_groups_locked(time.monotonic())
                return [n for n in names if self.group_fits(pod, n)]
            planned = self._planned_locked(pod, names)
            if planned is not None:
                return [planned[0]]          # the queue's joint plan put it there
            res = self._reserved_locked(O.uid(pod))
            return [n for n in names if n in self.nodes
                    and any(f - res.get((n, i), 0) >= req for i, f in enumerate(self.nodes[n].free()))]

    def _reserved_locked(self, uid: str) -> dict:
        """(node, gpu) -> HBM the queue's joint plan holds for the *other* pending pods. A pod
        the plan left out may only use what the plan leaves free: placing it by best fit into
        a planned pod's room would undo the joint placement (and strand that pod)."""
        if uid not in self._pending:
            return {}
        self._replan_locked()
        if uid in self._plan:
            return {}
        return self._plan_res                 # maintained with the plan (read only here)

    def _choose(self, req: int, node_names=None, reserved: dict | None = None) -> tuple[str, int] | None:
        best = None
        for name in node_names or list(self.nodes):
            st = self.nodes.get(name)
            if st is None:
                continue
            for i, f in enumerate(st.free()):
                f -= (reserved or {}).get((name, i), 0)
                if f < req:
                    continue
                left = f - req
                key = (left, name, i) if self.policy == "binpack" else (-left, name, i)
                if best is None or key < best[0]:
                    best = (key, name, i)
        return (best[1], best[2]) if best else None

    def bind(self, pod: dict, node: str, gpu: int, assume_ns: int | None = None) -> dict:
        req = O.gpu_mem_of_pod(pod)
        ns, nm = O.namespace(pod), O.name(pod)
        patched = self.client.patch_pod(ns, nm, {"metadata": {"annotations": {
            const.ENV_RESOURCE_INDEX: str(gpu),
            const.ENV_RESOURCE_BY_POD: str(req),
            const.ENV_RESOURCE_ASSUME_TIME: str(assume_ns or time.time_ns()),
            const.ENV_ASSIGNED_FLAG: "false",
        }, "labels": {const.POD_LABEL_NODE: node}}})   # the node's plugin prepares ahead of the bind
        self.client.bind_pod(ns, nm, node, O.uid(pod))
        return patched

    def decide(self, pod: dict, node_names=None) -> tuple[str, int] | None:
        """Filter + prioritize + reserve (the scheduling cycle; in memory)."""
        req = O.gpu_mem_of_pod(pod)
        with self._lock:
            choice = (self._planned_locked(pod, node_names)
                      or self._choose(req, node_names, self._reserved_locked(O.uid(pod))))
            self._drop_pending_locked(O.uid(pod))
            if choice is None:
                return None
            st = self.nodes[choice[0]]
            st.used[choice[1]] += req
            self._placed[O.uid(pod)] = (choice[0], [(choice[1], req)])
            self._touch(O.uid(pod))
        return choice

    def commit(self, pod: dict, choice: tuple[str, int], assume_ns: int | None = None) -> dict:
        """The binding cycle: write the annotations and bind (undo the reservation on error).
        Returns the pod as the kubelet will see it (annotations + nodeName)."""
        try:
            patched = self.bind(pod, choice[0], choice[1], assume_ns)
        except Exception:
            self.forget(pod)
            raise
        bound = dict(patched or pod)
        bound["spec"] = dict(bound.get("spec") or {}, nodeName=choice[0])
        return bound

    def schedule(self, pod: dict, node_names=None) -> tuple[str, int] | None:
        """Filter + prioritize + bind one pod. Returns (node, gpu) or None if it does not fit."""
        choice = self.decide(pod, node_names)
        if choice is not None:
            self.commit(pod, choice)
        return choice

    def schedule_group(self, pods: list[dict], node_names=None) -> list[tuple[str, int]] | None:
        """Gang-place a tensor-parallel group: one pod per GPU, all GPUs pairwise xGMI."""
        if not pods:
            return []
        req = max(O.gpu_mem_of_pod(p) for p in pods)
        with self._lock:
            best = None
            for name in node_names or list(self.nodes):
                st = self.nodes[name]
                grp = T.best_group(st.topology, st.free(), len(pods), req)
                if grp is None:
                    continue
                key = (sum(st.free()[g] - req for g in grp), name)
                if best is None or key < best[0]:
                    best = (key, name, grp)
            if best is None:
                return None
            _, name, grp = best
            st = self.nodes[name]
            for p, g in zip(pods, grp):
                st.used[g] += O.gpu_mem_of_pod(p)
                self._placed[O.uid(p)] = (name, [(g, O.gpu_mem_of_pod(p))])
                self._touch(O.uid(p))
        out = []
        t = time.time_ns()
        for k, (p, g) in enumerate(zip(pods, grp)):
            self.bind(p, name, g, assume_ns=t + k)
            out.append((name, g))
        return out

    # -- TP groups over the scheduler's one-pod-at-a-time extender protocol ----------------
    def _expire_groups_locked(self, now: float):
        for name, r in list(self._groups.items()):
            if now - r["t"] > self.group_ttl_s:
                st = self.nodes.get(r["node"])
                for g in r["free"]:           # reserved for members that never came
                    if st:
                        st.used[g] -= r["req"]
                del self._groups[name]

    def _group_of(self, pod: dict) -> tuple[str, int] | None:
        labels = (pod.get("metadata") or {}).get("labels") or {}
        grp = labels.get(TP_GROUP_LABEL)
        if not grp:
            return None
        try:
            return f"{O.namespace(pod)}/{grp}", max(1, int(labels.get(TP_SIZE_LABEL, "1")))
        except ValueError:
            return f"{O.namespace(pod)}/{grp}", 1

    def group_fits(self, pod: dict, node: str) -> bool:
        """Filter for a TP-group member: the node holds its group's reservation with a slot
        left, or has a pairwise one-hop xGMI set of GPUs for the whole group."""
        gk = self._group_of(pod)
        st = self.nodes.get(node)
        if gk is None or st is None:
            return False
        r = self._groups.get(gk[0])
        if r is not None:
            return r["node"] == node and bool(r["free"])
        return T.best_group(st.topology, st.free(), gk[1], O.gpu_mem_of_pod(pod)) is not None

    def bind_member(self, pod: dict, node: str) -> int | None:
        """Bind one member of a TP group: reserve the group's clique on ``node`` at the first
        member (best fit, ``best_group``), hand each member the next GPU of it."""
        gk = self._group_of(pod)
        req = O.gpu_mem_of_pod(pod)
        with self._lock:
            self._expire_groups_locked(time.monotonic())
            st = self.nodes.get(node)
            if st is None:
                return None
            r = self._groups.get(gk[0])
            if r is None or r["node"] != node or not r["free"]:
                grp = T.best_group(st.topology, st.free(), gk[1], req)
                if grp is None:
                    return None
                for g in grp:
                    st.used[g] += req
                r = self._groups[gk[0]] = {"node": node, "free": list(grp), "req": req, "t": time.monotonic()}
            g = r["free"].pop(0)
            self._placed[O.uid(pod)] = (node, [(g, req)])
            self._touch(O.uid(pod))
            if not r["free"]:
                del self._groups[gk[0]]       # every member placed
        self.bind(pod, node, g)
        return g

    def usage(self) -> dict:
        with self._lock:
            return {n: {"per_gpu": s.per_gpu, "used": list(s.used)} for n, s in self.nodes.items()}




def serve_http(ext: Extender, host: str = "127.0.0.1", port: int = 0):
    """Extender HTTP endpoints: ``POST /gpushare-scheduler/filter`` (ExtenderArgs →
    ExtenderFilterResult) and ``POST /gpushare-scheduler/bind`` (ExtenderBindingArgs →
    ExtenderBindingResult); ``GET /healthz`` (alive) and ``GET /readyz`` (serving: 503 on a
    replica that is not the leader, which answers the POSTs 503 too)."""

    class H(http.server.BaseHTTPRequestHandler):
        protocol_version = "HTTP/1.1"

        def log_message(self, *a):
            pass

        def _reply(self, obj):
            b = json.dumps(obj).encode()
            self.send_response(200)
            self.send_header("Content-Type", "application/json")
            self.send_header("Content-Length", str(len(b)))
            self.end_headers()
            self.wfile.write(b)

        def _plain(self, code: int, text: str):
            b = text.encode()
            self.send_response(code)
            self.send_header("Content-Type", "text/plain")
            self.send_header("Content-Length", str(len(b)))
            self.end_headers()
            self.wfile.write(b)

        def do_GET(self):
            if self.path == "/healthz":
                return self._plain(200, "ok")
            if self.path == "/readyz":
                return self._plain(200, "leader" if ext.elector else "ok") if ext.serving() else \
                    self._plain(503, "not the leader")
            return self._plain(404, "not found")

        def do_POST(self):
            n = int(self.headers.get("Content-Length") or 0)
            args = json.loads(self.rfile.read(n) or b"{}")
            if not ext.serving():
                # another replica holds the lease: its ledger, not this one's, decides
                b = json.dumps({"Error": "not the leader"}).encode()
                self.send_response(503)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(b)))
                self.end_headers()
                return self.wfile.write(b)
            if self.path.endswith("/filter"):
                pod = args.get("Pod") or args.get("pod") or {}
                names = args.get("NodeNames") or args.get("nodenames") or \
                    [O.name(x) for x in ((args.get("Nodes") or {}).get("items") or [])]
                ok = ext.filter(pod, names)
                failed = {x: "insufficient GPU memory in one device" for x in names if x not in ok}
                return self._reply({"NodeNames": ok, "FailedNodes": failed, "Error": ""})
            if self.path.endswith("/bind"):
                try:
                    pod = ext.client.get_pod(args.get("PodNamespace", "default"), args["PodName"])
                    req = O.gpu_mem_of_pod(pod)
                    if ext._group_of(pod) is not None:
                        g = ext.bind_member(pod, args["Node"])
                        return self._reply({"Error": "" if g is not None else "no xGMI-connected GPU set fits"})
                    with ext._lock:
                        st = ext.nodes.get(args["Node"])
                        fits = ext._fits(st, req) if st else []
                        if not fits:
                            return self._reply({"Error": "no GPU fits"})
                        planned = ext._planned_locked(pod, [args["Node"]])
                        ext._drop_pending_locked(O.uid(pod))
                        g = planned[1] if planned else min(fits, key=lambda i: (st.free()[i] - req, i))
                        st.used[g] += req
                        ext._placed[O.uid(pod)] = (st.name, [(g, req)])
                        ext._touch(O.uid(pod))
                    ext.bind(pod, args["Node"], g)
                    return self._reply({"Error": ""})
                except Exception as e:  # noqa: BLE001
                    return self._reply({"Error": str(e)})
            self.send_response(404)
            self.send_header("Content-Length", "0")
            self.end_headers()

    class S(socketserver.ThreadingMixIn, http.server.HTTPServer):
        daemon_threads = True

    srv = S((host, port), H)
    threading.Thread(target=srv.serve_forever, name="extender-http", daemon=True).start()
    return srv
