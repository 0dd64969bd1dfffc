"""The native Allocate table: the engine's side of the native DevicePlugin server.

``plugin/native_server.py`` serves the kubelet from ``libgpushare_dpserver.so`` (native/dpserver),
which answers the common Allocate from a table of prepared answers without entering Python.
This mixin of ``alloc/engine.py``'s ``Allocator`` keeps that table equal to what the engine's
own candidate rules give (``docs/ALLOCATE_PATH.md``):

* the pod-cache hook (``_on_pending`` / ``_publish_change``, on the watch thread) applies each
  change of the Pending set to the last table at once; a full rebuild (``Allocator._prepare``)
  covers everything else (engine generation changes, relists);
* pods the extender placed here are candidates from before their bind (``precompute``, fed by
  ``cluster/podcache.py`` PrebindWatch): their answers are prepared and published into the table
  at once, so the kubelet's Allocate — whose own watch may deliver the bind before the plugin's —
  finds its pod already there; a pre-bind pod whose bind does not come (deleted, placed
  elsewhere, label moved) is withdrawn from the table after ``PREBIND_CONFIRM_S``
  (``expire_prebind``);
* the server's claims come back through ``_native_loop`` / ``_native_taken`` for the same
  bookkeeping as the engine's own answers (claimed set, grants, replay index, write-behind
  PATCH), and its journal file is compacted into the engine's.

Wire formats: the table blob (``_native_blob``, parsed by ``dpserver.cpp`` ``parse_table``) and
the few protobuf records prepared answers append (``_pb_*``).
"""
from __future__ import annotations

import bisect
import dataclasses
import threading
import time

from ..api import v1beta1 as api
from ..cluster import objects as O
from ..utils import log
from . import annotations as A


@dataclasses.dataclass(frozen=True)
class _Prepared:
    uid: str
    ns: str
    name: str
    size: int              # single-container pods: its units; multi: the first container's
    multi: bool            # multi-container pod: the full path must handle it
    gpu: int
    body: bytes = b""      # serialized AllocateResponse (one container)
    head: bytes = b""      # journal record prefix (AllocJournal.fast_head)
    lkey: str = ""
    # this entry in the native table's wire format, encoded once (_native_blob)
    frag: bytes = dataclasses.field(default=b"", compare=False, repr=False)


NATIVE_NO_TABLE = 1 << 31


# protobuf wire encoding of the few fields _prepared appends (field tags precomputed:
# ContainerAllocateResponse envs = 1, mounts = 2, annotations = 4; entry key = 1, value = 2;
# Mount container_path = 1, host_path = 2)
def _pb_varint(n: int) -> bytes:
    out = bytearray()
    while n >= 0x80:
        out.append((n & 0x7F) | 0x80)
        n >>= 7
    out.append(n)
    return bytes(out)


def _pb_ld(tag: int, b: bytes) -> bytes:
    n = len(b)
    if n < 0x80:                                      # (most fields: one length byte)
        return bytes((tag, n)) + b
    return bytes((tag,)) + _pb_varint(n) + b


def _pb_map_entry(tag: int, k: str, v: str) -> bytes:
    return _pb_ld(tag, _pb_ld(0x0A, k.encode()) + _pb_ld(0x12, v.encode()))


def _native_blob(version: int, gen: int, flags: int, cands, replay_ids) -> bytes:
    """The fast table in the native server's format (native/dpserver/dpserver.cpp "table
    blob"): the prepared candidates in match order, then the fake IDs of possible replays."""
    import struct

    def s(b):
        b = b if isinstance(b, bytes) else b.encode()
        return struct.pack("<I", len(b)) + b
    parts = [struct.pack("<QQIII", version, gen, flags, len(cands), len(replay_ids))]
    for c in cands:
        f = getattr(c, "frag", None)
        if not f:
            f = struct.pack("<IB", c.size, 1 if c.multi else 0) + s(c.uid) + s(c.body) + s(c.head)
            if isinstance(c, _Prepared):
                object.__setattr__(c, "frag", f)      # the entry is immutable: encode it once
        parts.append(f)
    parts += [s(i) for i in replay_ids]
    return b"".join(parts)


class NativeTable:
    """Mixin of ``Allocator``: the native server's table and claims (see the module docstring)."""

    # ------------------------------------------------------------------------------------
    # native fast path (plugin/native_server.py, native/dpserver)
    # ------------------------------------------------------------------------------------
    def attach_native(self, nat) -> None:
        """Serve the fast path from the native server ``nat``: the prepare loop publishes its
        table there instead of answering here, and the server's claims come back through
        ``_native_taken``. Its journal records go to ``<journal>.fast`` (loaded with the journal)."""
        self.native = nat
        with self._mu:
            self._fast = None
            nat.set_gen(self._gen)
        self._hook_pods(nat)
        if self.journal.path:
            # loaded and compacted into the main journal at start-up: the fast file starts empty
            nat.journal_open(self.journal.fast_path(), 32 << 20)
            nat.journal_rotate()
        threading.Thread(target=self._native_loop, args=(nat,), name="native-claims", daemon=True).start()
        ev = getattr(self.pods, "changed", None)
        if ev is not None:
            ev.set()

    def detach_native(self) -> None:
        nat, self.native = self.native, None
        if nat is not None:
            self._drain_native(nat)
            src = self.pods
            if getattr(src, "on_pending_change", None) is not None:
                src.on_pending_change = None
            if self._native_hold:
                self._native_hold = False

    def _hook_pods(self, nat) -> None:
        src = self.pods
        if hasattr(src, "on_pending_change"):
            with src._lock:
                src.on_pending_change = self._on_pending
                nat.set_version(src.pending_version)

    def _on_pending(self, version: int, pod: dict | None = None, gone: bool = False) -> None:
        """Pod-cache hook (the watch thread, cache lock held), at every change of the Pending
        set: the native server learns the version first, so it never answers from a table
        older than the cache. The change itself (one pod joined, changed or left the set) is
        then applied to the last table right here, so the kubelet's Allocate — usually arriving
        right after the same watch event — finds a current table instead of waiting for the
        prepare loop."""
        nat = self.native
        if nat is None:
            return
        if pod is not None and not gone and getattr(nat, "spin_us", 0) > 0 and O.uid(pod) not in self._native_prep:
            # a pod joined the Pending set: the kubelet's Allocate for it is on its way — keep
            # the server's threads hot from now until it has come (``gs_dp_spin``)
            nat.spin(nat.spin_us)
        nat.set_version(version)
        if pod is not None:
            t = time.perf_counter()
            u = O.uid(pod)
            if not gone:
                self._mark(u, "bind_seen")
            try:
                kind = self._publish_change(nat, version, pod, gone)
                if not gone:
                    self._mark(u, "bind_pub" if kind else "bind_skip")
                if kind:
                    self.metrics.table_publish.observe(time.perf_counter() - t, path=f"hook_{kind}")
            except Exception as e:  # noqa: BLE001 - the prepare loop republishes anyway
                log.V(2).info("incremental native table: %s", e)

    def _publish_change(self, nat, version: int, pod: dict, gone: bool) -> str:
        """The table at ``version`` = the table at ``version - 1`` with ``pod`` removed and, if
        it is a candidate now, placed in candidate order (bound before pre-bind, assume time,
        then arrival; the table's keys are ``(pre-bind, assume time)``) — what
        ``_prepare`` would build: anything else that changes candidates (a taint, a placement
        overlay, a reconfigure) bumps the engine generation, and claims made since are marked
        taken in the server."""
        if not self.opts.fast_path or self.opts.compute_isolation == "cu" or time.time() < self.journal._legacy_until:
            return ""
        kicks: list = []
        try:
            return self._publish_change_in(nat, version, pod, gone, kicks)
        finally:
            for k in kicks:                           # the ledger / granter threads, after the publish
                k()

    def _publish_change_in(self, nat, version: int, pod: dict, gone: bool, kicks: list) -> str:
        with self._table_mu:
            last = self._last_table
            gen = self._gen
            if last is None or last[0] != version - 1 or last[1] != gen:
                self.metrics.table_publish_skipped.inc(why="gen" if last is not None and last[1] != gen else "version")
                return ""
            _, _, out, ats = last
            u = O.uid(pod)
            idx = next((i for i, c in enumerate(out) if c.uid == u), None)
            c = at = None
            if not gone:
                p = self._view([pod])[0]
                assumed, _, at, shape = self._info(p)
                if (assumed and shape and not O.deleting(p) and u not in self._assigned and u not in self._claims
                        and u not in self._tainted):
                    g = A.gpu_id_from_annotation(p)
                    if len(shape) > 1:
                        c = _Prepared(u, O.namespace(p), O.name(p), shape[0], True, g)
                    elif self.model.gpu(g) is not None:
                        k = (u, g, shape[0])
                        c = (self._prep_cache.get(k) or self._take_precomputed(k)
                             or self._prepared(p, u, g, shape[0], kicks))
                        self._prep_cache[k] = c
            at = (0, at)                              # a pod of the pod cache: bound here
            keep_at = idx is not None and c is not None and ats[idx] == at
            if idx is not None:
                old = out[idx]
                if c is None or (old.gpu, old.size) != (c.gpu, c.size):
                    self._prep_cache.pop((old.uid, old.gpu, old.size), None)   # left the table
                out, ats = out[:idx] + out[idx + 1:], ats[:idx] + ats[idx + 1:]
            if c is not None:
                i = idx if keep_at else bisect.bisect_right(ats, at)   # same place, or after its equals
                out, ats = out[:i] + (c,) + out[i:], ats[:i] + (at,) + ats[i:]
                self._native_prep.pop(u, None)
                self._native_prep[u] = c
                # the current entries must be the newest: re-append them after the new one
                for e in out:
                    if e.uid != u:
                        self._native_prep.pop(e.uid, None)
                        self._native_prep[e.uid] = e
                self._trim_native_prep(len(out))
            nat.publish(_native_blob(version, gen, 1 if self.podres is not None else 0, list(out),
                                     self.journal.replay_ids()))
            self._last_table = (version, gen, out, ats)
            self._published = (version, gen)
        return "add" if idx is None and c is not None else "other"

    # ---- the per-pod timeline (``/debug/latency`` "pod_trace") ------------------------------
    PTRACE_KEEP = 256
    PTRACE_CPU = frozenset(("pre_seen", "prep_ledger", "prep_hbm", "pre_prep", "pre_pub"))

    def _mark(self, u: str, key: str, t: int | None = None) -> None:
        """First time ``key`` happened for pod ``u`` (CLOCK_MONOTONIC ns, comparable across the
        node's processes): ``pre_seen`` / ``pre_pub`` (the pre-bind watch delivered the placed pod;
        its entry is in the table), ``bind_seen`` / ``bind_pub`` (the pod watch delivered the bind;
        the table has it as bound), ``tab`` (a full rebuild published it), ``alloc_in`` (its
        Allocate reached the server) and the server's waits."""
        # (the watch threads, the claim reader and the metrics endpoint share it: every step below
        # is one operation of the ordered dict or the dict, so no lock is taken on the pre-bind path)
        trace = self._ptrace
        tr = trace.get(u)
        if tr is None:
            tr = trace.setdefault(u, {})
            if len(trace) > self.PTRACE_KEEP:
                try:
                    trace.popitem(last=False)
                except KeyError:
                    pass
        if key not in tr:
            tr.setdefault(key, t if t is not None else time.monotonic_ns())
            if t is None and self._ptrace_cpu and key in self.PTRACE_CPU:
                tr.setdefault(key + "_cpu_ns", time.thread_time_ns())   # this thread's CPU time: wall - cpu = waits

    def pod_trace(self) -> list[dict]:
        """The last pods' timelines, in ms relative to their Allocate's arrival (pods whose
        Allocate came), oldest first."""
        out = []
        items = [(u, dict(tr)) for u, tr in list(self._ptrace.items())]
        for u, tr in items:
            t0 = tr.get("alloc_in")
            if t0 is None:
                continue
            rec = {k: (v if isinstance(v, str) or k.endswith("_ns") else round((v - t0) / 1e6, 3))
                   for k, v in tr.items() if k != "alloc_in"}
            rec["uid"], rec["alloc_in_abs"] = u, t0
            out.append(rec)
        return out

    def _native_loop(self, nat) -> None:
        """Takes in the native server's claims as they happen; rotates its journal file once
        the engine's own journal holds everything it has."""
        last_prefault = 0.0
        while not self._stop.is_set() and self.native is nat:
            rec = nat.taken_next(200)
            if rec is None:
                break
            try:
                if rec:
                    self._native_taken(rec)
                now = time.monotonic()
                if now - self._last_sweep > 1.0:
                    with self._mu:
                        self._sweep_assigned(now)
                if self.journal.path and (rec or now - last_prefault > 5.0):
                    # keep the pages the next native answers journal into writable (after each
                    # answer, and every few seconds against writeback), so the answer never
                    # takes a page fault
                    nat.journal_prefault()
                    last_prefault = now
                if self.journal.path and nat.journal_used() > self.native_rotate_bytes:
                    nat.block()
                    try:
                        self._drain_native(nat)
                        self._drain_post()
                        self.journal.compact()
                        nat.journal_rotate()
                    finally:
                        nat.unblock()
            except Exception as e:  # noqa: BLE001 - one bad record must not stop every later claim's bookkeeping
                log.error("native claim bookkeeping failed: %s", e)
                self._stop.wait(0.05)

    def _drain_native(self, nat=None) -> None:
        nat = nat or self.native
        if nat is None:
            return
        while True:
            rec = nat.taken_next(0)
            if not rec:
                return
            self._native_taken(rec)

    def _native_taken(self, rec) -> None:
        """One native answer: the same claim and bookkeeping as the engine's fast path."""
        uid, rb, t, hns = rec[:4]
        if len(rec) > 4:                              # the server's own timeline of this answer
            t_in, ww, tw = rec[4:7]
            self._mark(uid, "alloc_in", t_in)
            self._mark(uid, "watch_wait_ns", ww)
            self._mark(uid, "table_wait_ns", tw)
        self._mark(uid, "path", "native")
        pick = self._native_prep.get(uid)
        with self._mu:
            self._assigned[uid] = time.monotonic()
            self._unpatched.add(uid)
            self._revoked.discard(uid)
            self._answer_seq += 1
        if pick is None:
            # not expected (every entry of a published table stays in _native_prep): the
            # answer went out, so the pod still owes its ASSIGNED patch — take it from the cache
            p = self.pods.get(uid)
            log.error("native fast path answered pod uid %s outside the prepared answers%s", uid,
                      "" if p is not None else "; the pod is gone from the cache, no patch")
            if p is None:
                with self._mu:
                    self._unpatched.discard(uid)
                return
            pick = self._prepared(p, uid, A.gpu_id_from_annotation(p), self._info(p)[3][0])
        req = api.AllocateRequest.FromString(rb)
        ids = req.container_requests[0].devices_ids
        self.journal.note_fast(uid, pick.ns, pick.name, t, ids)
        self._post.append((rb, pick, t))
        log.info("----Allocating GPU for gpu mem is started---- RequestPodGPUs: %d; pod %s, new allocated GPUs info: "
                 "gpu index %d uuid %s (patch queued, native)", len(ids), pick.name, pick.gpu,
                 self.model.uuid_by_index(pick.gpu))
        self.metrics.allocate_outcomes.inc(outcome="assigned")
        self.metrics.allocate_latency.observe(hns / 1e9, phase="total")
        self.metrics.allocate_latency.observe(hns / 1e9, phase="native")
        self.metrics.allocate_requests.observe(0)
        if self._patch_q is not None:
            from .engine import _PatchJob             # the engine's patcher job (engine imports this module)

            self._patch_q.put(_PatchJob(uid, pick.ns, pick.name, {}))

    def _trim_native_prep(self, n_current: int) -> None:
        """Bound the prepared answers kept for native claims (the current table's entries are
        the last ``n_current`` inserted and always stay)."""
        prep = self._native_prep
        if len(prep) > self.native_prep_keep + n_current:
            for u in list(prep)[:len(prep) - n_current - self.native_prep_keep // 2]:
                del prep[u]

    def precompute(self, pod: dict) -> None:
        """A pod placed on this node but not bound yet (``cluster/podcache.py`` PrebindWatch):
        prepare its Allocate answer now and publish it into the table as a candidate, in assume
        time order, so the kubelet's Allocate finds it even when the kubelet's watch delivered
        the bind before the plugin's (the pod is this node's assumed candidate from the moment
        the extender placed it, ``allocate.go:63-89``). The bind, when the pod watch brings it,
        replaces the entry in place."""
        if (self.native is None or not self.opts.fast_path or self.opts.compute_isolation == "cu"
                or not hasattr(self.pods, "pending_version")):
            return                                    # (pre-bind candidates need the pod watch cache)
        assumed, _, _, shape = self._info(pod)
        if not assumed or len(shape) != 1:
            return
        u, g = O.uid(pod), A.gpu_id_from_annotation(pod)
        self._mark(u, "pre_seen")                    # (pre_read: its watch event's bytes arrived)
        if self.pods.get(u) is not None:
            self._mark(u, "pre_after_bind")
            return                                    # the bind came first: the pod cache has it
        k = (u, g, shape[0])
        if self.model.gpu(g) is None:
            return
        kicks: list = []
        try:
            if k not in self._precomputed and k not in self._prep_cache and u not in self._native_prep:
                c = self._prepared(pod, u, g, shape[0], kicks)
                _native_blob(0, 0, 0, [c], [])        # fills c.frag: the table entry, encoded once
                self._precomputed[k] = (c, time.monotonic())
                while len(self._precomputed) > 1024:
                    self._precomputed.popitem(last=False)
                self._mark(u, "pre_prep")
            with self._table_mu:
                prev = self._prebind.get(u)
                self._prebind[u] = (pod, prev[1] if prev is not None else time.monotonic(), None)
                while len(self._prebind) > 1024:
                    self._prebind.pop(next(iter(self._prebind)))
            how = self._publish_prebind(u, kicks=kicks)
            self._mark(u, "pre_pub" if how == "pub" else f"pre_{how}")
        finally:
            for kk in kicks:                          # the ledger / granter threads, after the publish
                kk()

    # how long a pre-bind candidate whose pre-bind watch entry went away (bound, deleted, label
    # moved: the watch does not say which) stays in the table waiting for the pod watch to show
    # it bound here; and how long one that never went away is kept at all
    PREBIND_CONFIRM_S = 2.0
    PREBIND_TTL_S = 30.0

    def prebind_gone(self, pod: dict) -> None:
        """PrebindWatch: the pod left the unbound-and-labelled set — bound (here, the pod watch
        will show it), deleted, placed elsewhere or relabelled. Its entry stays for
        ``PREBIND_CONFIRM_S`` (``expire_prebind``)."""
        u = O.uid(pod)
        with self._table_mu:
            e = self._prebind.get(u)
            if e is not None and e[2] is None:
                self._prebind[u] = (e[0], e[1], time.monotonic())

    def _prebind_live(self, u: str, now: float) -> bool:
        e = self._prebind.get(u)
        if e is None:
            return False
        _, t0, gone = e
        return now - t0 < self.PREBIND_TTL_S and (gone is None or now - gone < self.PREBIND_CONFIRM_S)

    def _prebind_pods(self) -> list[dict]:
        """Pre-bind candidates the pod cache does not have yet (the engine's ``_candidates``)."""
        if not self._prebind:
            return []
        now = time.monotonic()
        with self._table_mu:
            items = list(self._prebind.items())
        return [e[0] for u, e in items if self._prebind_live(u, now) and self.pods.get(u) is None]

    def expire_prebind(self) -> None:
        """Withdraw pre-bind candidates that the pod cache never showed bound here within their
        window: their entries leave the table unless a native answer already claimed them (that
        answer went to a pod of this node, and the claim stands, as any claim does). A pod the
        cache has now is no longer pre-bind."""
        if not self._prebind:
            return
        now = time.monotonic()
        drop, bound = [], []
        # (the pod cache's lock is never taken under _table_mu: the cache hook takes them the
        # other way round)
        with self._table_mu:
            uids = list(self._prebind)
        cached = {u for u in uids if self.pods.get(u) is not None}
        with self._table_mu:
            for u, e in list(self._prebind.items()):
                if u in cached:
                    bound.append(u)
                elif not self._prebind_live(u, now):
                    drop.append(u)
            for u in bound + drop:
                self._prebind.pop(u, None)
        for u in drop:
            if u in self._assigned:
                log.warning("pod uid %s: answered before its bind, which never reached this node; its answer "
                            "went to another pod of the same size (placement truth reconciles the annotations)", u)
                continue
            self.metrics.allocate_outcomes.inc(outcome="prebind_withdrawn")
            self._publish_prebind(u, remove=True)

    def _publish_prebind(self, u: str, remove: bool = False, kicks: list | None = None) -> str:
        """Insert (or withdraw) pre-bind candidate ``u`` in the last published table, at the same
        cache version: the table is what a full rebuild gives now (``_prepare`` takes the same
        pre-bind set into its candidates). Returns what happened ("pub", or why not)."""
        nat = self.native
        if nat is None or not self.opts.fast_path or self.opts.compute_isolation == "cu":
            return "off"
        in_cache = self.pods.get(u) is not None        # before _table_mu (lock order: cache, then table)
        with self._table_mu:
            last = self._last_table
            if last is None or last[1] != self._gen or time.time() < self.journal._legacy_until:
                # the prepare loop rebuilds (it takes the pre-bind set too)
                return "no_table" if last is None else "gen" if last[1] != self._gen else "legacy"
            version, gen, out, ats = last
            idx = next((i for i, c in enumerate(out) if c.uid == u), None)
            if remove:
                if idx is None or in_cache:
                    return "kept"
                old = out[idx]
                self._prep_cache.pop((old.uid, old.gpu, old.size), None)
                out, ats = out[:idx] + out[idx + 1:], ats[:idx] + ats[idx + 1:]
            else:
                e = self._prebind.get(u)
                if idx is not None:
                    return "present"
                if e is None or u in self._assigned or u in self._claims or u in self._tainted:
                    return "not_candidate"
                p = self._view([e[0]])[0]
                assumed, _, at, shape = self._info(p)
                if not assumed or len(shape) != 1 or O.deleting(p):
                    return "not_candidate"
                g = A.gpu_id_from_annotation(p)
                k = (u, g, shape[0])
                c = self._prep_cache.get(k) or self._take_precomputed(k) or self._prepared(p, u, g, shape[0], kicks)
                self._prep_cache[k] = c
                key = (1, at)                         # after every bound candidate (_candidates)
                i = bisect.bisect_right(ats, key)
                out, ats = out[:i] + (c,) + out[i:], ats[:i] + (key,) + ats[i:]
                self._native_prep.pop(u, None)
                self._native_prep[u] = c
                for en in out:
                    if en.uid != u:
                        self._native_prep.pop(en.uid, None)
                        self._native_prep[en.uid] = en
                self._trim_native_prep(len(out))
            nat.publish(_native_blob(version, gen, 1 if self.podres is not None else 0, list(out),
                                     self.journal.replay_ids()))
            self._last_table = (version, gen, out, ats)
        return "pub"

    # the ledger directory a prepared answer names is kept for a grace period without a pod on
    # this node (quota/ledger.py collect, 60 s): a bind later than this gets a fresh answer
    PRECOMPUTED_TTL_S = 30.0

    def _take_precomputed(self, k) -> "_Prepared | None":
        e = self._precomputed.pop(k, None)
        if e is None or time.monotonic() - e[1] > self.PRECOMPUTED_TTL_S:
            return None
        return e[0]
