"""The Allocate engine — the core of GPU sharing (component C5).

Reference ``pkg/gpu/nvidia/allocate.go:43-201``:
1. request size = number of fake IDs across the request (``:55-57``);
2. under the plugin-wide mutex (``:60-61``) LIST this node's pending pods, keep "assumed"
   ones, order by assume time (``:63-67``);
3. pick the first whose summed container ``gpu-mem`` equals the request (``:79-89``);
4. read the extender's GPU index from ``ALIYUN_COM_GPU_MEM_IDX`` (``:92-111``), answer with
   env vars (``:114-129``) and PATCH the pod ``ASSIGNED=true`` (one retry, ``:132-152``);
5. fallbacks: single-GPU node → GPU 0 without a pod (``:154-181``); otherwise an
   error-shaped *successful* response (``:182-187``, ``buildErrResponse`` ``:25-40``).

MI355X build, same protocol, different mechanics:
* the mutex covers only the in-memory match + claim (µs); the PATCH runs outside it, with
  a local claim set so concurrent Allocates never pick the same pod (quirk 7);
* candidates come from a ``PodSource`` — by default a watch cache, with one fresh LIST on a
  miss;
* the response injects ``/dev/kfd`` + the GPU's render node as ``DeviceSpec``s and the HIP
  quota shim as a read-only ``Mount`` + ``LD_PRELOAD`` — there is no NVIDIA runtime hook;
* multi-container pods are matched container by container (quirk 3) after the
  reference's pod-total rule has been tried;
* conflicts are detected by HTTP status, not by comparing error strings (quirk 8);
* ``--strict-allocate`` returns a gRPC error instead of the soft failure (quirk 6);
* optional write-behind of the ASSIGNED patch (``async_patch``): a matched pod is claimed in
  memory and the annotation is landed by a retrying background patcher, taking the apiserver
  round trip off the kubelet's admission path; candidates are Pending pods only and the claim
  is held until the patch is acknowledged, so a pod is never matched twice;
* optional compute isolation (``compute_isolation="cu"``, ``alloc/cuslots.py``): each pod also
  gets its own run of CU slots, answered as ``HSA_CU_MASK`` / ``ROC_GLOBAL_CU_MASK`` and recorded
  on the pod in the same ASSIGNED patch;
* swap completion: AllocateRequest carries no pod identity, so when the kubelet admits two
  equal-size pods in an order other than their assume times, the first Allocate takes the
  other pod's reservation and its own pod turns Running with ``ASSIGNED=false``. The reference
  then fails the second pod (``allocate.go:182-187``: no Pending candidate left); here, when no
  Pending pod matches, an equal-size pod that is bound, un-assigned, recently assumed and never
  allocated by this process is matched instead — the two pods simply exchange their
  extender-reserved GPUs;
* prepared answers (fast path): a background thread keeps, for every candidate pod in the
  watch cache, its single-container answer already serialized plus its journal record; when
  the cache has not changed since, Allocate only picks the first eligible candidate of the
  request's size (same order and rules as the full match), appends the record to the mapped
  journal and returns the prepared bytes — grants and the replay index follow off the hot
  path. Anything unusual (multi-container pod first in line, possible replay, cache changed,
  CU isolation, sync patch) takes the full path;
* placement truth (``alloc/placement.py``): every answered container is recorded in a grant
  book (fake-ID set → GPU); with the kubelet's pod-resources API configured, the plugin asks
  for ``PreStartContainer`` and, before each container starts (and every ``placement_s``),
  joins the book with which pod holds which IDs and rewrites ``IDX`` / the allocation JSON /
  CU slots to where the containers really run — a swapped admission never leaves the
  extender's ledger pointing at the wrong GPU, so deleting one of the pods frees the GPU it
  actually used.
"""
from __future__ import annotations

import collections
import contextlib
import dataclasses
import functools
import os
import threading
import time

from .. import const
from ..api import v1beta1 as api
from ..cluster import objects as O
from ..cluster.client import APIClient, APIError
from ..cluster.podcache import PodSource
from ..device.model import DeviceModel
from ..quota import ShimConfig, ledger_name
from ..utils import log, units as U
from ..utils.metrics import PluginMetrics
from . import annotations as A
from . import cuslots
from . import placement as PL
from .journal import AllocJournal, request_key
from .native_table import NATIVE_NO_TABLE, NativeTable, _native_blob, _pb_ld, _pb_map_entry, _Prepared  # noqa: F401


class AllocationError(Exception):
    """Raised only in strict mode; the gRPC layer maps it to FAILED_PRECONDITION."""


@dataclasses.dataclass
class AllocatorOptions:
    unit: str = const.GIB
    disable_cgpu: bool = False
    shim: ShimConfig | None = None
    strict: bool = False
    expose_devices: bool = True
    rocr_visible: bool = False
    match_containers: bool = True
    claim_ttl_s: float = 120.0
    # a multi-container pod's containers are allocated back to back by the kubelet; a claim not
    # continued within this window is abandoned
    partial_claim_ttl_s: float = 10.0
    # write-behind: how often the patcher re-checks bound pods that this plugin answered but
    # that still read ASSIGNED=false (lost PATCH, restart) and patches them again
    reconcile_s: float = 30.0
    complete_swaps: bool = True
    # host directory for file-backed shim ledgers (mounted read-write into every shared
    # container at const.LEDGER_CONTAINER_DIR); None = pod-private POSIX shm ledgers
    ledger_dir: str | None = None
    # allocation journal (alloc/journal.py): in memory always, persisted when a path is given
    journal_path: str | None = None
    journal_ttl_s: float = 120.0
    # Write-behind ASSIGNED=true PATCH: Allocate answers after the in-memory claim and a
    # background patcher lands the annotation (retrying); the claim blocks re-matching until it
    # has. False = the reference's synchronous PATCH inside Allocate (allocate.go:132-152).
    async_patch: bool = False
    # "cu": per-pod CU-slot masks (alloc/cuslots.py); "none": pods time-slice the whole GPU
    compute_isolation: str = "none"
    # CDI: also (or instead of DeviceSpecs, expose_devices=False) name the GPU as a CDI device
    # "<kind>=<index>" — the spec AMD's container toolkit generates (e.g. amd.com/gpu=3) carries
    # /dev/kfd and the GPU's render node; None = no CDI devices
    cdi_kind: str | None = None
    # placement truth (alloc/placement.py): periodic pass interval, and how long an answer whose
    # fake IDs no pod holds yet counts as "in flight" (kubelet checkpoint not visible yet)
    placement_s: float = 2.0
    in_flight_s: float = 30.0
    # prepared answers for the common admission (see module docstring); write-behind only
    fast_path: bool = True
    # admission identity from the kubelet's pod-resources List when the request's size is
    # ambiguous or a multi-container admission is in progress (see _identify). The List runs
    # outside the engine lock with this timeout; after a timeout or error identity is skipped
    # (size matching) for identify_backoff_s
    identify: bool = True
    identify_timeout_s: float = 0.2
    identify_backoff_s: float = 5.0
    # an Allocate for a pod the pod watch has not delivered yet (the kubelet's own watch can be
    # ahead of the plugin's) waits up to this long for the watch before it falls back to a LIST
    # (a round trip to the apiserver on the kubelet's path)
    watch_grace_s: float = 0.005
    # per-GPU HBM brokers (native/hbmbroker): their socket directory on the host, and the share of
    # a container's quota granted as broker granules (quota/hbmbroker.py HBMGranter); None = off
    hbm_broker_dir: str | None = None
    hbm_broker_fraction: float = 0.94
    # the node's read-only comgr cache (quota/comgr_cache.py) on the host; None = off
    comgr_cache_dir: str | None = None
    # HBMGranter keyword arguments (poll_s, startup_grace_s, down_grace_s, revoke_grace_s, ...)
    hbm_granter_args: dict = dataclasses.field(default_factory=dict)


@dataclasses.dataclass
class _Claim:
    uid: str
    pod: dict
    gpu_index: int
    next_container: int    # gpu containers of ``shape`` already answered
    shape: tuple           # the pod's gpu-mem requests, one per gpu container, in container order
    t: float               # last time a container of this pod was answered
    slots: cuslots.SlotRun | None = None
    swap: bool = False     # matched through swap completion (the pod is bound, not Pending)


@dataclasses.dataclass(frozen=True)
class _Fast:
    version: int           # pod-cache version the candidates were read at
    gen: int               # engine state generation (overlays, taints, rebuilds)
    cands: tuple           # _Prepared in the full match's order


class Allocator(NativeTable):
    def __init__(self, model: DeviceModel, pods: PodSource, client: APIClient | None, node: str,
                 opts: AllocatorOptions | None = None, metrics: PluginMetrics | None = None):
        self.model, self.pods, self.client, self.node = model, pods, client, node
        self.opts = opts or AllocatorOptions()
        self.metrics = metrics or PluginMetrics()
        self._mu = threading.Lock()
        self._claims: dict[str, _Claim] = {}      # in-flight (multi-container or PATCH pending)
        self._partial: _Claim | None = None       # the multi-container pod being admitted right now
        self._tainted: dict[str, float] = {}      # uid -> time: reservation partly used by another pod
        self._assigned: dict[str, float] = {}     # uid -> time we assigned it (stale-cache guard)
        self._unpatched: set[str] = set()         # assigned locally, PATCH not yet acknowledged
        self._pinfo: dict[tuple, tuple] = {}      # memoised per-pod-version facts (see _info)
        self._patch_q = None
        self._slot_mu = threading.Lock()
        self._slot_pending: dict[str, tuple] = {}  # uid -> (gpu, SlotRun, t): chosen, not yet on the pod
        self._stop = threading.Event()
        self._last_reconcile = time.monotonic()
        self._last_sweep = 0.0
        self.journal = AllocJournal(self.opts.journal_path, self.opts.journal_ttl_s)
        # placement truth: answered containers, the kubelet's pod-resources view, and the
        # annotation changes this plugin has queued but the pod cache may not show yet
        self.grants = PL.GrantBook()
        self.prestart_hooks: list = []          # run at PreStartContainer (after the placement pass)
        self._ledgers = self._ledger_dir(self.opts)
        self._hbm = self._hbm_granter(self.opts, live=self._hbm_live, on_readiness=self._hbm_readiness)
        if self._hbm is not None and not getattr(self, "_hbm_metrics", False):
            self.metrics.registry.add_collector(lambda: self._hbm.exposition() if self._hbm is not None else "")
            self._hbm_metrics = True
        self.podres = None
        self._overlay: dict[str, dict] = {}       # uid -> annotations written, not yet landed
        self._overlay_gen: dict[str, int] = {}
        self._revoked: set[str] = set()           # reservation re-armed: its assign job must not re-claim
        self._place_mu = threading.Lock()
        self._place_thread = None
        self._last_grant = 0.0
        self._placed_at = 0.0                     # start of the last completed placement pass
        self._answer_seq = 0                      # answers given (invalidates the identity List)
        self._ident_cache = None                  # (monotonic, answer_seq, pod-resources List)
        self._ident_off_until = 0.0
        # fast path: prepared answers, engine-state generation, answers awaiting bookkeeping
        self._fast: _Fast | None = None
        self._gen = 0
        self.gen_bumps: dict[str, int] = {}
        self.placement_log: list[dict] = []
        self._prep_cache: dict[tuple, _Prepared] = {}
        self._post: "collections.deque" = collections.deque()
        self._post_mu = threading.Lock()
        # native fast path (plugin/native_server.py): the server answers from the published
        # table; its claims come back through _native_taken
        self.native = None
        self._native_prep: dict[str, _Prepared] = {}
        self._native_hold = False                 # a block kept while a multi-container claim is open
        self._published = (-1, -1)                # (pending version, gen) of the last native table
        # the last native table: (version, gen, entries, their assume times) — a pod the watch
        # adds is published into it at once from the cache hook (_publish_added)
        self._last_table: tuple | None = None
        self._table_mu = threading.Lock()
        self._resp_tmpl: dict[tuple, api.ContainerAllocateResponse] = {}   # _container_response
        # answers prepared before the bind (PrebindWatch -> precompute), by (uid, gpu, units)
        self._precomputed: collections.OrderedDict = collections.OrderedDict()
        # pods placed here but not bound yet: uid -> (pod, first seen, pre-bind watch gone at | None);
        # candidates already (native_table.py precompute / expire_prebind)
        self._prebind: dict[str, tuple] = {}
        # per-pod timeline of the fast path, CLOCK_MONOTONIC ns (native_table.py ``pod_trace``)
        self._ptrace: collections.OrderedDict = collections.OrderedDict()
        # with each mark this thread's CPU time too (a syscall each): GPUSHARE_TRACE_CPU=1 (bench.py)
        self._ptrace_cpu = os.environ.get("GPUSHARE_TRACE_CPU") == "1"
        self._tmpl_bytes: dict[tuple, bytes] = {}                          # _prepared
        self.native_rotate_bytes = 16 << 20       # rotate the native journal file past this
        self.native_prep_keep = 4096              # prepared answers kept for native claims past the current table
        for k, uid, t, resp in self.journal.answers():   # grants of a previous instance (journal TTL)
            if len(resp.container_responses) == 1:
                self.grants.record(k, self._grant_from(resp.container_responses[0], uid, t))
        if self.opts.async_patch:
            import queue
            self._patch_q = queue.Queue()
            # a previous instance answered these pods but never saw their PATCH land (crash,
            # kill, apiserver outage): they stay claimed and are patched again first
            for e in self.journal.unlanded():
                self._assigned[e["uid"]] = time.monotonic()
                self._unpatched.add(e["uid"])
                self._patch_q.put(_PatchJob(e["uid"], e["ns"], e["name"], e.get("ann") or {}, recovered=True))
                self.metrics.allocate_outcomes.inc(outcome="patch_recovered")
                log.warning("write-behind: re-queueing the unlanded ASSIGNED patch of pod %s/%s (uid %s)",
                            e["ns"], e["name"], e["uid"])
            threading.Thread(target=self._patcher, name="assign-patcher", daemon=True).start()
            threading.Thread(target=self._prepare_loop, name="prepare-answers", daemon=True).start()

    @staticmethod
    def _hbm_granter(opts: AllocatorOptions, live=None, on_readiness=None):
        # also on a cgpu-disabled node: there it holds the brokers at nothing (quota/hbmbroker.py)
        if not (opts.hbm_broker_dir and opts.shim is not None and opts.shim.enabled):
            return None
        from ..quota.hbmbroker import HBMGranter
        return HBMGranter(opts.hbm_broker_dir, opts.hbm_broker_fraction, live=live, on_readiness=on_readiness,
                          disabled=opts.disable_cgpu, **opts.hbm_granter_args)

    def _hbm_live(self) -> dict | None:
        """The HBM tokens the pods on this node need (the granter's pod view): every gpu container
        of every pod here with a GPU assignment (``ALIYUN_COM_GPU_MEM_IDX``), whether it is running
        or still being admitted. None when the pod view is unavailable (nothing is revoked then)."""
        hbm = self._hbm
        if hbm is None:
            return None
        try:
            pods = self.pods.node_pods()
        except Exception:  # noqa: BLE001 - the granter retries on its next pass
            return None
        out = {}
        for p in pods:
            shape = self._info(p)[3]
            idx = O.annotations(p).get(const.ENV_RESOURCE_INDEX) if shape else None
            if idx is None or not idx.isdigit():
                continue
            g = int(idx)
            dev = self.model.gpu(g)
            if dev is None:
                continue
            u = O.uid(p)
            for slot, units in enumerate(shape):
                out[hbm.token(u, slot)] = (g, U.quota_bytes(units, dev.units, dev.vram_bytes))
        return out

    def _hbm_readiness(self) -> None:
        """A GPU's broker went away for good or came back: answers prepared with (or without) its
        token are re-prepared."""
        with self._mu:
            self._bump_gen("hbm_readiness")
            self._fast = None
            self._prep_cache.clear()
        self._precomputed.clear()

    @staticmethod
    def _ledger_dir(opts: AllocatorOptions):
        if not (opts.ledger_dir and opts.shim is not None):
            return None
        from ..quota.ledger import LedgerDir
        ld = LedgerDir(opts.ledger_dir)
        try:
            ld.prepare()
        except OSError as e:
            log.warning("ledger dir %s: %s", opts.ledger_dir, e)
        return ld.start()

    def reconfigure(self, model: DeviceModel, pods: PodSource, client: APIClient | None,
                    opts: AllocatorOptions) -> "Allocator":
        """Plugin rebuild (kubelet restart, SIGHUP; ``gpumanager.go:82-96``): new devices, pod
        source and node-label options, but the same claims, assigned set, pending patches and
        patcher — a rebuild must never forget a pod it already answered (write-behind)."""
        with self._mu:
            self.model, self.pods, self.client = model, pods, client
            async_patch = self.opts.async_patch
            ledger_dir = self.opts.ledger_dir
            self.opts = dataclasses.replace(opts, async_patch=async_patch, journal_path=self.opts.journal_path)
            if opts.ledger_dir != ledger_dir:
                self._ledgers = self._ledger_dir(self.opts)
            # the same granter across rebuilds (its grants and pod view stay); a new one only when
            # the broker directory or the share changed
            old = self._hbm
            if old is None or (opts.hbm_broker_dir, opts.hbm_broker_fraction) != (old.host_dir, old.fraction):
                if old is not None:
                    old.stop()
                self._hbm = self._hbm_granter(self.opts, live=self._hbm_live, on_readiness=self._hbm_readiness)
            if self._hbm is not None and not getattr(self, "_hbm_metrics", False):
                self.metrics.registry.add_collector(lambda: self._hbm.exposition() if self._hbm is not None else "")
                self._hbm_metrics = True
            if self._hbm is not None:
                self._hbm.set_disabled(self.opts.disable_cgpu)
            self._pinfo.clear()
            self._bump_gen("reconfigure")
            self._fast = None
            self._prep_cache.clear()
        if self.native is not None:
            self._hook_pods(self.native)
        return self

    def set_cgpu_disabled(self, disabled: bool) -> None:
        """The node's ``cgpu.disable.isolation`` label changed while the plugin runs (the
        reference reads it once, at start: ``podmanager.go:62-75``). Answers prepared from now on
        carry ``CGPU_DISABLE=true`` and no shim (or the shim again), and the HBM brokers are sized
        to nothing (or to the GPU again)."""
        with self._mu:
            if self.opts.disable_cgpu == disabled:
                return
            self.opts = dataclasses.replace(self.opts, disable_cgpu=disabled)
            self._bump_gen("cgpu_disable")
            self._fast = None
            self._prep_cache.clear()
            self._resp_tmpl.clear()
            self._tmpl_bytes.clear()
        self._precomputed.clear()
        if self._hbm is not None:
            self._hbm.set_disabled(disabled)
        log.warning("cgpu isolation %s on this node", "disabled" if disabled else "enabled")

    def close(self):
        self._stop.set()
        if self._hbm is not None:
            self._hbm.stop()
        if self._patch_q is not None:
            self._patch_q.put(None)

    def gen_bump_counts(self) -> dict[str, int]:
        """``gen_bumps``, copied under the engine lock (the debug endpoint's thread)."""
        with self._mu:
            return dict(self.gen_bumps, **({"last_fixes": list(self.placement_log)} if self.placement_log else {}))

    def _bump_gen(self, why: str = "other") -> None:
        """A change of engine state the prepared answers depend on (caller holds ``_mu``): the
        native table built before it is no longer served, and the prepare loop rebuilds.
        ``gen_bumps`` counts them by cause (/debug/latency, the bench line)."""
        self.gen_bumps[why] = self.gen_bumps.get(why, 0) + 1
        self._gen += 1
        nat = self.native
        if nat is not None:
            nat.set_gen(self._gen)
        ev = getattr(self.pods, "changed", None)
        if ev is not None:
            ev.set()

    # ------------------------------------------------------------------------------------
    # candidate selection
    # ------------------------------------------------------------------------------------
    def _info(self, p: dict) -> tuple[bool, int, int, tuple]:
        """(assumed, pod gpu-mem, assume time, gpu-container shape) of one pod version,
        memoised: every Allocate scans all Pending pods, and re-parsing their specs dominated
        the handler. The key carries the two annotations the plugin itself
        rewrites, so an object updated in place (no new resourceVersion) is never served stale."""
        ann = O.annotations(p)
        # a pod's gpu-mem requests cannot change (extended resources are not resizable in
        # place), so the key is the pod plus the two annotations the result depends on — not
        # its resourceVersion: the bind (a new version) hits what the pre-bind pass parsed
        k = (O.uid(p), ann.get(const.ENV_ASSIGNED_FLAG), ann.get(const.ENV_RESOURCE_ASSUME_TIME))
        v = self._pinfo.get(k)
        if v is None:
            shape = tuple(x for x in O.gpu_mem_per_container(p) if x > 0)
            v = (A.is_assumed_pod(p), sum(shape), A.assume_time(p), shape)
            if len(self._pinfo) > 8192:
                self._pinfo.clear()
            self._pinfo[k] = v
        return v

    def _view(self, pods: list[dict]) -> list[dict]:
        """Pods as they will read once this plugin's queued placement patches have landed."""
        ov = self._overlay
        if not ov:
            return pods
        out = []
        for p in pods:
            a = ov.get(O.uid(p))
            if a is not None:
                md = dict(p.get("metadata") or {})
                ann = dict(md.get("annotations") or {})
                for k, v in a.items():
                    if v is None:
                        ann.pop(k, None)
                    else:
                        ann[k] = v
                md["annotations"] = ann
                p = dict(p, metadata=md)
            out.append(p)
        return out

    def _sweep_assigned(self, now: float) -> None:
        """Forget claims older than claim_ttl_s whose patch has landed (caller holds ``_mu``;
        amortised to once a second). The full path sweeps before matching; with the native
        server answering, the claim reader does (``native_table.py`` ``_native_loop``)."""
        if now - self._last_sweep > 1.0:
            self._last_sweep = now
            for u, t in list(self._assigned.items()):
                if now - t > self.opts.claim_ttl_s and u not in self._unpatched:
                    del self._assigned[u]

    def _candidates(self, fresh: bool) -> list[dict]:
        """Pending assumed pods in match order: assume time, then arrival — and every pod the
        pod cache shows bound here before any pre-bind one (the kubelet admits only
        bound pods, and the pod watch delivers binds in order, so an unbound pod older than a
        bound one of the same size is one whose bind is still in flight, or failed: the
        reference, which sees bound pods only, ``podmanager.go:228``, would pick the bound one)."""
        pre = self._prebind_pods()
        pre_u = {O.uid(p) for p in pre}
        pods = self._view(A.dedupe_by_uid(self.pods.pending_pods(fresh=fresh), self.node) + pre)
        now = time.monotonic()
        self._sweep_assigned(now)
        if fresh and self._tainted:   # forget a withheld reservation once its pod is gone
            live = {O.uid(p) for p in self.pods.node_pods() if not O.deleting(p)}
            for u in [u for u in self._tainted if u not in live]:
                del self._tainted[u]
        out = []
        for p in pods:
            assumed, _, at, _ = self._info(p)
            u = O.uid(p)
            # a pod being deleted is never admitted by the kubelet
            if assumed and u not in self._assigned and u not in self._tainted and not O.deleting(p):
                out.append((1 if u in pre_u else 0, at, len(out), p))
        out.sort(key=lambda e: e[:3])             # bound first, assume time, then arrival order (stable)
        if log.V(4):
            for _, at, _, p in out:
                log.info("candidate pod %s in ns %s with timestamp %d is found.", O.name(p), O.namespace(p), at)
        return [p for _, _, _, p in out]

    def _partial_state(self, c: _Claim, cands: list[dict], now: float) -> str:
        """"live": the claimed pod can still be continued; "stale": it exists but the claim
        outlived ``partial_claim_ttl_s`` — or, not matched through swap completion, it is no
        longer Pending (it started: some of its containers ran on answers from other
        reservations, and the ones answered from its own may be in use); "gone": deleted or
        being deleted."""
        if c.swap:
            alive = any(O.uid(p) == c.uid and not O.deleting(p) for p in self.pods.node_pods())
        elif any(O.uid(p) == c.uid for p in cands):
            alive = True
        else:
            p = self.pods.get(c.uid)
            if p is None or O.deleting(p) or O.is_terminated(p):
                return "gone"
            return "stale"
        if not alive:
            return "gone"
        return "stale" if now - c.t > self.opts.partial_claim_ttl_s else "live"

    def _match(self, sizes: tuple, fresh: bool, held=None) -> tuple[_Claim | None, bool]:
        """Returns (claim, complete). ``complete`` = every gpu container of the pod is now
        allocated, so the pod must be PATCHed ASSIGNED.

        ``sizes`` = the request's per-container unit counts. The kubelet admits one pod at a
        time and calls Allocate once per gpu container, back to back; an AllocateRequest names
        no pod. So a pod only ever matches a request of its own *shape*: a single-container
        request takes a single-container pod of that size, never a multi-container pod whose
        total happens to be equal (the reference's pod-total rule, ``allocate.go:79-89``, is the
        special case shape == (total,)). A multi-container pod is claimed on its first container
        and continued only by the very next Allocate, while the pod still exists; anything else
        abandons the claim and the pod becomes a candidate again."""
        k = len(sizes)
        now = time.monotonic()
        cands = self._candidates(fresh)
        if held is not None and (self._partial is not None or self._ambiguous(cands, sizes)):
            ident = self._identify(cands, sizes, held)
            if ident is not None:
                return self._match_identified(ident, sizes, now)
        c = self._partial
        if c is not None:
            state = self._partial_state(c, cands, now)
            if state == "live" and c.shape[c.next_container:c.next_container + k] == sizes:
                self._partial = None
                c.next_container += k
                c.t = now
                done = c.next_container == len(c.shape)
                if not done:
                    self._partial = c
                return c, done
            if not fresh:
                return None, False           # decide on an authoritative LIST, not on the cache
            self._partial = None
            self._claims.pop(c.uid, None)
            if state == "gone":
                # the claimed pod is deleted: it was the pod being admitted, nothing is in use
                self.metrics.allocate_outcomes.inc(outcome="claim_abandoned")
                log.warning("pod %s: deleted after %d/%d gpu containers were allocated; claim released",
                            O.name(c.pod), c.next_container, len(c.shape))
            else:
                # The pod still exists but the kubelet did not continue it: the containers
                # answered from its reservation went to another pod of the same leading shape
                # (out-of-order admission), which may be running on them. The reservation is
                # never handed out again while the pod lives (no double booking of its HBM);
                # its own admission, if it comes, is matched elsewhere or refused.
                self._tainted[c.uid] = now
                self._bump_gen("claim_tainted")
                self.metrics.allocate_outcomes.inc(outcome="claim_tainted")
                log.warning("pod %s: %d/%d gpu containers answered from its reservation, then the kubelet moved on "
                            "(%s); reservation withheld", O.name(c.pod), c.next_container, len(c.shape),
                            "stale" if state == "stale" else f"next container {list(sizes)}")
                cands = [p for p in cands if O.uid(p) != c.uid]
                if state == "live":
                    # the pod being admitted is another one whose gpu containers start with what
                    # was answered: continue it when it is reserved on the same GPU
                    done_shape = c.shape[:c.next_container] + sizes
                    for p in cands:
                        shape = self._info(p)[3]
                        if (O.uid(p) not in self._claims and shape[:len(done_shape)] == done_shape
                                and A.gpu_id_from_annotation(p) == c.gpu_index):
                            self.metrics.allocate_outcomes.inc(outcome="claim_retargeted")
                            log.warning("pod %s: containers answered so far fit pod %s (same GPU %d); claim moved",
                                        O.name(c.pod), O.name(p), c.gpu_index)
                            if len(shape) == len(done_shape):
                                return _Claim(O.uid(p), p, c.gpu_index, len(done_shape), shape, now), True
                            return self._start_partial(p, shape, len(done_shape), now, swap=False), False
        cands = [p for p in cands if O.uid(p) not in self._claims]
        # 1) the earliest-assumed pod whose gpu containers start with this request: exactly
        #    this shape (single-container pods: the reference rule), or the first containers of
        #    a multi-container pod (claimed, continued by the next Allocates)
        for p in cands:
            shape = self._info(p)[3]
            if shape == sizes:
                return _Claim(O.uid(p), p, A.gpu_id_from_annotation(p), k, sizes, now), True
            if self.opts.match_containers and len(shape) > k and shape[:k] == sizes:
                return self._start_partial(p, shape, k, now, swap=False), False
        # 2) swap completion (authoritative pass only): see the module docstring
        if fresh and self.opts.complete_swaps:
            p = self._swap_partner(sizes)
            if p is not None:
                shape = self._info(p)[3]
                self.metrics.allocate_outcomes.inc(outcome="swap")
                log.warning("no pending pod requests %s%s: completing a swapped admission with pod %s (gpu %d)",
                            list(sizes), self.opts.unit, O.name(p), A.gpu_id_from_annotation(p))
                if len(shape) > k:
                    return self._start_partial(p, shape, k, now, swap=True), False
                return _Claim(O.uid(p), p, A.gpu_id_from_annotation(p), k, shape, now, swap=True), True
        return None, False

    def _ambiguous(self, cands: list[dict], sizes: tuple) -> bool:
        """More than one candidate could be the pod this request belongs to."""
        n = 0
        for p in cands:
            if O.uid(p) in self._claims:
                continue
            shape = self._info(p)[3]
            if shape[:len(sizes)] == sizes:
                n += 1
                if n > 1:
                    return True
        return False

    def _identity_list(self, sizes: tuple):
        """The kubelet's pod-resources List for admission identity (``_identify``), or None.
        Fetched only when the request is ambiguous, and never under the engine lock: a slow or
        rate-limited kubelet must not stall every Allocate of the node (the reference's global
        lock, quirk 7). Short timeout; after a failure identity is off for a while (size
        matching decides, placement truth repairs a swap afterwards). One List serves a
        retried or concurrent request until the next answer is given."""
        src = self.podres
        if src is None or not self.opts.identify or time.monotonic() < self._ident_off_until:
            return None
        with self._mu:
            need = self._partial is not None or self._ambiguous(self._candidates(False), sizes)
            seq = self._answer_seq
        if not need:
            return None
        c = self._ident_cache
        if c is not None and c[1] == seq and time.monotonic() - c[0] < 0.5:
            return c[2]
        t = time.monotonic()
        try:
            try:
                held = src.list(include_empty=True, timeout=self.opts.identify_timeout_s)
            except TypeError:                     # a pod-resources view without a timeout argument
                held = src.list(include_empty=True)
        except Exception as e:  # noqa: BLE001 - kubelet restarting or overloaded
            self._ident_off_until = time.monotonic() + self.opts.identify_backoff_s
            self.metrics.allocate_outcomes.inc(outcome="identity_unavailable")
            log.warning("admission identity unavailable (%s): size matching for %.0f s", e,
                        self.opts.identify_backoff_s)
            return None
        self._ident_cache = (t, seq, held)
        return held

    def _identify(self, cands: list[dict], sizes: tuple, held) -> tuple[dict, int] | None:
        """Admission identity: the kubelet adds a pod to its pod manager right before admitting
        it and checkpoints each container's fake IDs as soon as that container's Allocate
        returns, so in the pod-resources List (``held``) the pod being admitted is the one
        Pending pod of this node whose gpu containers do not all hold IDs yet. Returns (pod,
        number of its gpu containers already allocated), or None when that is not exactly one pod."""
        pending = {(O.namespace(p), O.name(p)): p for p in self._view(A.dedupe_by_uid(
            self.pods.pending_pods(fresh=False), self.node))}
        for p in cands:
            pending.setdefault((O.namespace(p), O.name(p)), p)
        found = []
        for pd in held:
            p = pending.get((pd.namespace, pd.name))
            if p is None or O.deleting(p):
                continue
            have = {cn for cn, ids in pd.containers if ids}
            gpu_ctrs = [name for _, name, _ in PL._gpu_containers(p)]
            done = sum(1 for cn in gpu_ctrs if cn in have)
            if gpu_ctrs and done < len(gpu_ctrs):
                found.append((p, done))
        if len(found) != 1:
            return None
        p, done = found[0]
        if self._info(p)[3][done:done + len(sizes)] != sizes:
            log.warning("admission identity: pod %s is being admitted but its next gpu containers are not %s; "
                        "falling back to matching by size", O.name(p), list(sizes))
            return None
        return p, done

    def _match_identified(self, ident: tuple[dict, int], sizes: tuple, now: float) -> tuple[_Claim | None, bool]:
        """Match the pod the kubelet is admitting (``_identify``): its own reservation, never
        another pod's — no swap, no stray partial claim."""
        p, done = ident
        u = O.uid(p)
        shape = self._info(p)[3]
        c = self._partial
        if c is not None and c.uid == u and c.next_container == done:
            self._partial = None
            c.next_container += len(sizes)
            c.t = now
            if c.next_container < len(c.shape):
                self._partial = c
                return c, False
            return c, True
        if c is not None:
            # a claim started by size matching belongs to another pod: its answered containers
            # went to the pods admitted since, so its reservation is withheld (see _match)
            self._partial = None
            self._claims.pop(c.uid, None)
            if self.pods.get(c.uid) is not None:
                self._tainted[c.uid] = now
                self._bump_gen("claim_tainted")
                self.metrics.allocate_outcomes.inc(outcome="claim_tainted")
        if u in self._tainted or u in self._claims or (u in self._assigned and done == 0):
            log.warning("admission identity: pod %s is being admitted but its reservation is no longer whole", O.name(p))
            return None, False
        self.metrics.allocate_outcomes.inc(outcome="identified")
        claim = _Claim(u, p, A.gpu_id_from_annotation(p), done + len(sizes), shape, now)
        if claim.next_container == len(shape):
            return claim, True
        self._claims[u] = claim
        self._partial = claim
        return claim, False

    def _start_partial(self, p: dict, shape: tuple, k: int, now: float, swap: bool) -> _Claim:
        c = _Claim(O.uid(p), p, A.gpu_id_from_annotation(p), k, shape, now, swap=swap)
        self._claims[c.uid] = c
        self._partial = c
        return c

    def _swap_partner(self, sizes: tuple) -> dict | None:
        """A bound, un-assigned pod of the request's shape whose own admission took another
        pod's reservation (equal shapes only, so per-GPU accounting stays exact)."""
        now_ns = time.time_ns()
        ttl_ns = int(self.opts.claim_ttl_s * 1e9)
        k = len(sizes)
        out = []
        for p in self._view(A.dedupe_by_uid(self.pods.node_pods(), self.node)):
            u = O.uid(p)
            if (O.phase(p) == "Pending" or O.deleting(p) or not A.is_assumed_pod(p) or u in self._assigned
                    or u in self._claims or u in self._tainted or self.journal.answered(u) or now_ns - A.assume_time(p) > ttl_ns):
                continue
            shape = self._info(p)[3]
            if shape[:k] == sizes:
                out.append(p)
        out = A.order_by_assume_time(out)
        return out[0] if out else None

    # ------------------------------------------------------------------------------------
    # response building
    # ------------------------------------------------------------------------------------
    def _container_response(self, gpu_index: int, pod_units: int, ctr_units: int, pod_uid: str,
                            slot: int, cu: cuslots.SlotRun | None = None) -> api.ContainerAllocateResponse:
        """One container's answer: what depends only on (GPU, sizes, configuration) comes from a
        cached template (a copy in C), then the per-pod quota-ledger parts are added — this runs
        on the watch thread for every newly bound pod (``_publish_change``)."""
        if cu is not None:
            r = self._container_base(gpu_index, pod_units, ctr_units, cu)
        else:
            key = (self._gen, gpu_index, pod_units, ctr_units)
            base = self._resp_tmpl.get(key)
            if base is None:
                base = self._container_base(gpu_index, pod_units, ctr_units, None)
                if len(self._resp_tmpl) > 512:
                    self._resp_tmpl.clear()
                self._resp_tmpl[key] = base
            r = api.ContainerAllocateResponse()
            r.CopyFrom(base)
        shim = self.opts.shim
        if shim is not None and shim.enabled and not self.opts.disable_cgpu:
            r.envs[const.ENV_SHIM_LEDGER] = ledger_name(pod_uid or f"{gpu_index}-{time.time_ns()}", slot)
            if self._ledgers is not None:
                # this container's own ledger directory (quota/ledger.py): a tenant never sees
                # another container's ledger
                try:
                    lkey = self._ledgers.take(pod_uid)
                    host = self._ledgers.path(lkey)
                except OSError as e:
                    log.warning("ledger dir for pod %s: %s (pod-private shm ledger instead)", pod_uid, e)
                else:
                    r.mounts.add(container_path=const.LEDGER_CONTAINER_DIR, host_path=host, read_only=False)
                    r.envs[const.ENV_SHIM_LEDGER_DIR] = const.LEDGER_CONTAINER_DIR
                    r.annotations[const.CTR_ANNOTATION_LEDGER] = lkey
            hbm = self._hbm
            if hbm is not None:
                g = self.model.gpu(gpu_index)
                tok = hbm.token(pod_uid or f"{gpu_index}-{time.time_ns()}", slot)
                if hbm.submit(gpu_index, tok, U.quota_bytes(ctr_units, g.units, g.vram_bytes)):
                    r.envs[const.ENV_HBM_TOKEN] = tok
        return r

    def _container_base(self, gpu_index: int, pod_units: int, ctr_units: int,
                        cu: cuslots.SlotRun | None) -> api.ContainerAllocateResponse:
        """The container answer without its per-pod ledger parts."""
        g = self.model.gpu(gpu_index)
        envs = {
            const.ENV_RESOURCE_INDEX: str(gpu_index),
            const.ENV_RESOURCE_BY_POD: str(pod_units),
            const.ENV_RESOURCE_BY_CONTAINER: str(ctr_units),
            const.ENV_RESOURCE_BY_DEV: str(g.units),
            const.ENV_GPU_UUID: g.uuid,
        }
        r = api.ContainerAllocateResponse(envs=envs)
        if self.opts.disable_cgpu:
            r.envs[const.ENV_CGPU_DISABLE] = "true"
        if self.opts.rocr_visible:
            r.envs[const.ENV_ROCR_VISIBLE] = g.uuid
        if cu is not None:
            # the container sees only this GPU when its render node is the one handed out
            single = self.opts.expose_devices or self.opts.rocr_visible
            r.envs[const.ENV_HSA_CU_MASK] = cuslots.hsa_cu_mask(cu, g.num_xcc, 0 if single else gpu_index)
            if single:
                r.envs[const.ENV_ROC_CU_MASK] = cuslots.roc_cu_mask(cu, g.num_xcc)
            r.envs[const.ENV_CU_SLOTS] = cu.annotation()
        if self.opts.expose_devices:
            r.devices.add(container_path=const.KFD_DEVICE, host_path=const.KFD_DEVICE, permissions="rw")
            if g.render_node:
                r.devices.add(container_path=g.render_node, host_path=g.render_node, permissions="rw")
        if self.opts.cdi_kind:
            r.cdi_devices.add(name=f"{self.opts.cdi_kind}={gpu_index}")
        shim = self.opts.shim
        if shim is not None and shim.enabled and not self.opts.disable_cgpu:
            r.mounts.add(container_path=shim.container_dir, host_path=shim.host_dir, read_only=True)
            r.envs[const.ENV_LD_PRELOAD] = shim.container_lib
            # exact bytes from the SMI-reported HBM size, so the shim needs no device query
            r.envs[const.ENV_SHIM_QUOTA_BYTES] = str(U.quota_bytes(ctr_units, g.units, g.vram_bytes))
            if self._hbm is not None:
                # the GPU's HBM broker: only that GPU's pod-socket directory (never the admin
                # sockets); the pod's token is per pod (_container_response / _prepared)
                r.mounts.add(container_path=const.HBM_BROKER_CONTAINER_DIR, host_path=self._hbm.mount_dir(gpu_index),
                             read_only=True)
                r.envs[const.ENV_HBM_BROKER] = self._hbm.container_socket(gpu_index)
                r.envs[const.ENV_HIP_FORCE_DEV_KERNARG] = "0"
        if self.opts.comgr_cache_dir and not self.opts.disable_cgpu and os.path.isdir(self.opts.comgr_cache_dir):
            # code objects the runtime would build with comgr at the container's first stream:
            # from the cache the DaemonSet's init container filled; read-only, so no pod can put
            # code into another pod's runtime (a miss compiles as without the cache). A directory
            # that is not there (no init container ran) is not mounted: the container would not start
            r.mounts.add(container_path=const.COMGR_CACHE_CONTAINER_DIR, host_path=self.opts.comgr_cache_dir,
                         read_only=True)
            r.envs[const.ENV_COMGR_CACHE] = "1"
            r.envs[const.ENV_COMGR_CACHE_DIR] = const.COMGR_CACHE_CONTAINER_DIR
            if (shim is not None and shim.enabled
                    and os.path.exists(os.path.join(shim.host_dir, const.COMGR_ACTION_LIB_NAME))):
                # the rest of the runtime's compile from the same cache (native/comgrcache),
                # preloaded from the shim's directory after the shim
                r.envs[const.ENV_LD_PRELOAD] = shim.container_lib + ":" + os.path.join(
                    shim.container_dir, const.COMGR_ACTION_LIB_NAME)
                r.envs[const.ENV_COMGR_ACTION_CACHE] = const.COMGR_CACHE_CONTAINER_DIR
        return r

    def _plan_slots(self, claim: _Claim, pod_units: int) -> cuslots.SlotRun | None:
        """CU-slot run for a matched pod (compute isolation), chosen against the runs the GPU's
        other live pods hold plus the choices not yet visible on a pod (patch in flight)."""
        g = self.model.gpu(claim.gpu_index)
        if (self.opts.compute_isolation != "cu" or self.opts.disable_cgpu or g is None or g.num_xcc <= 1
                or g.num_cu < g.num_xcc):
            return None
        if claim.slots is not None:
            return claim.slots
        nslots = g.num_cu // g.num_xcc
        req = O.annotations(claim.pod).get(const.POD_ANNOTATION_CU_SLOTS_REQUEST)
        k = cuslots.wanted_slots(pod_units, g.units, nslots, req)
        try:
            pods = A.dedupe_by_uid(self.pods.node_pods(), self.node)
        except Exception as e:  # noqa: BLE001 - a cache failure must not fail the admission
            log.warning("compute isolation: cannot list pods (%s); pod %s shares the whole GPU", e, O.name(claim.pod))
            return None
        with self._slot_mu:
            now = time.monotonic()
            for u, (_, _, t) in list(self._slot_pending.items()):
                if now - t > self.opts.claim_ttl_s and u not in self._unpatched:
                    del self._slot_pending[u]
            held = cuslots.held_runs([p for p in pods if O.uid(p) not in self._slot_pending], claim.gpu_index,
                                     exclude_uid=claim.uid)
            held += [r for u, (gi, r, _) in self._slot_pending.items() if gi == claim.gpu_index and u != claim.uid]
            run, exclusive = cuslots.choose(held, k, nslots)
            self._slot_pending[claim.uid] = (claim.gpu_index, run, now)
            self.metrics.cu_slots_held.set(sum(r.count for r in held) + run.count, gpu=str(claim.gpu_index))
        claim.slots = run
        if not exclusive:
            self.metrics.allocate_outcomes.inc(outcome="cu_shared")
            log.warning("compute isolation: GPU %d has no free run of %d CU slots; pod %s shares slots %s",
                        claim.gpu_index, k, O.name(claim.pod), run.annotation())
        return run

    def _drop_slots(self, uid: str) -> None:
        """The pod now carries its slot annotation (or is gone): stop tracking it locally."""
        with self._slot_mu:
            self._slot_pending.pop(uid, None)

    def _err_response(self, req, pod_units: int) -> api.AllocateResponse:
        """``buildErrResponse`` (``allocate.go:25-40``) minus the NVIDIA env: no device node is
        handed out, so a misallocated container cannot touch a GPU it was not given."""
        if self.opts.strict:
            raise AllocationError(f"no-gpu-has-{pod_units}{self.opts.unit}-to-run")
        resp = api.AllocateResponse()
        for creq in req.container_requests:
            resp.container_responses.add(envs={
                "GPUSHARE_ALLOCATION_ERROR": f"no-gpu-has-{pod_units}{self.opts.unit}-to-run",
                const.ENV_RESOURCE_INDEX: "-1",
                const.ENV_RESOURCE_BY_POD: str(pod_units),
                const.ENV_RESOURCE_BY_CONTAINER: str(len(creq.devices_ids)),
                const.ENV_RESOURCE_BY_DEV: str(self.model.dev_units()),
            })
        self.metrics.allocate_outcomes.inc(outcome="error")
        return resp

    # ------------------------------------------------------------------------------------
    # RPCs
    # ------------------------------------------------------------------------------------
    def allocate(self, req) -> api.AllocateResponse:
        r = self.allocate_raw(req)
        return api.AllocateResponse.FromString(r) if isinstance(r, bytes) else r

    def allocate_raw(self, req, defer=None):
        """The Allocate RPC: the prepared answer's wire bytes (fast path) or a message.
        ``defer(fn)`` runs ``fn`` once the reply is on its way (gRPC ``context.add_callback``):
        the fast path wakes the patcher there, so that thread never competes with the reply
        for the interpreter."""
        t0 = time.perf_counter()
        fast = self._fast
        if fast is not None and self.native is None:
            body = self._allocate_fast(req, fast, t0, defer)
            if body is not None:
                return body
        return self._allocate_full(req, t0)

    def _allocate_fast(self, req, fast: "_Fast", t0: float, defer=None) -> bytes | None:
        crs = req.container_requests
        if len(crs) != 1 or self._partial is not None:
            return None
        ids = crs[0].devices_ids
        n = len(ids)
        if n == 0 or self.journal.maybe_replay(ids[0]) or fast.version != getattr(
                self.pods, "pending_version", getattr(self.pods, "version", -1)):
            return None
        with self._mu:
            if fast.gen != self._gen or self._partial is not None:
                return None
            el = [c for c in fast.cands if c.size == n and c.uid not in self._assigned
                  and c.uid not in self._claims and c.uid not in self._tainted]
            # a multi-container pod first in line (partial claims), or — with pod-resources —
            # more than one candidate of this size (which one the kubelet is admitting is for
            # admission identity to say): the full path decides
            if not el or el[0].multi or (len(el) > 1 and self.podres is not None):
                return None
            pick = self._take(el[0])
        rb = req.SerializeToString()
        t = self.journal.record_fast(pick.uid, pick.ns, pick.name, pick.head, rb, ids)
        self._post.append((rb, pick, t))
        job = _PatchJob(pick.uid, pick.ns, pick.name, {})
        # the reference logs the request and the outcome (allocate.go:47-58,193-194): one record here
        log.info("----Allocating GPU for gpu mem is started---- RequestPodGPUs: %d; pod %s, new allocated GPUs info: "
                 "gpu index %d uuid %s (patch queued)", n, pick.name, pick.gpu, self.model.uuid_by_index(pick.gpu))
        self.metrics.allocate_outcomes.inc(outcome="assigned")
        dt = time.perf_counter() - t0
        self.metrics.allocate_latency.observe(dt, phase="total")
        self.metrics.allocate_latency.observe(dt, phase="fast")
        self.metrics.allocate_requests.observe(0)
        if defer is None or not defer(lambda: self._patch_q.put(job)):
            self._patch_q.put(job)
        return pick.body

    def _take(self, c: "_Prepared") -> "_Prepared":
        """Claim a prepared candidate (caller holds ``_mu``)."""
        self._answer_seq += 1
        self._assigned[c.uid] = time.monotonic()
        self._unpatched.add(c.uid)
        self._revoked.discard(c.uid)
        return c

    def _drain_post(self) -> None:
        """Bookkeeping of fast-path answers, off the hot path: grant book + journal index."""
        if self.native is not None:
            self._drain_native()
        with self._post_mu:
            while self._post:
                rb, c, t = self._post.popleft()
                ids = tuple(api.AllocateRequest.FromString(rb).container_requests[0].devices_ids)
                key = PL.ids_key(ids)
                self.journal.index_answer(key, c.uid, t, c.body, ids)
                self.grants.record(key, PL.Grant(gpu=c.gpu, units=len(ids), claimed=c.uid, t=t, ledger=c.lkey))
                self._last_grant = time.monotonic()
            self.journal.prefault()

    def _prepare_loop(self):
        """Keep ``self._fast`` current: woken by every pod-cache change."""
        while not self._stop.is_set():
            src = self.pods
            ev = getattr(src, "changed", None)
            if ev is None or not self.opts.fast_path or self.opts.compute_isolation == "cu":
                self._fast = None
                if self.native is not None:
                    self.native.publish(_native_blob(0, 0, NATIVE_NO_TABLE, [], []))   # every Allocate to the engine
                self._stop.wait(1.0)
                continue
            ev.wait(0.5)
            ev.clear()
            try:
                self.expire_prebind()
                if self.native is not None and self._published == (getattr(src, "pending_version", None), self._gen):
                    # the cache hook already applied the change to the native table: a full
                    # rebuild now would only compete with the Allocate it made the table for
                    self._prune_replay_index(src)
                    continue
                self._prepare(src)
            except Exception as e:  # noqa: BLE001 - the full path still answers
                self._fast = None
                log.V(2).info("prepare answers: %s", e)

    def _prepare(self, src) -> None:
        tp = time.perf_counter()
        version = getattr(src, "pending_version", src.version)
        with self._mu:
            gen = self._gen
            cands = self._candidates(fresh=False)
            cands = [p for p in cands if O.uid(p) not in self._claims]
        out, ats, keep = [], [], {}
        for p in cands:
            _, _, at, shape = self._info(p)
            if not shape:
                continue
            u, g = O.uid(p), A.gpu_id_from_annotation(p)
            key = (0 if self.pods.get(u) is not None else 1, at)   # the table's order (see _candidates)
            if len(shape) > 1:
                out.append(_Prepared(u, O.namespace(p), O.name(p), shape[0], True, g))
                ats.append(key)
                continue
            k = (u, g, shape[0])
            c = self._prep_cache.get(k) or self._take_precomputed(k)
            if c is None:
                if self.model.gpu(g) is None:
                    continue
                c = self._prepared(p, u, g, shape[0])
            keep[k] = c
            out.append(c)
            ats.append(key)
        nat = self.native
        with self._mu:
            if gen != self._gen:          # reconfigured meanwhile: answers built from the old model
                return
            self._prep_cache = keep
            if nat is None:
                self._fast = _Fast(version, gen, tuple(out))
        if nat is not None:
            # the native server answers from this table while the cache and the engine are still
            # at (version, gen); a possible replay (IDs of journaled answers) goes to the engine
            self._fast = None
            # every answer a published table holds must stay resolvable when its claim comes
            # back: the current table's entries always; of the older ones, the most recent
            prep = self._native_prep
            for c in out:
                prep.pop(c.uid, None)
                prep[c.uid] = c           # (re)inserted last: the oldest entries are the stale ones
            self._trim_native_prep(len(out))
            legacy = time.time() < self.journal._legacy_until
            with self._table_mu:
                last = self._last_table
                # the cache hook may have published a newer table meanwhile: never go back
                if last is None or (gen, version) >= (last[1], last[0]):
                    nat.publish(_native_blob(version, gen, 1 if self.podres is not None else 0,
                                             [] if legacy else out, self.journal.replay_ids()))
                    self._last_table = (version, gen, () if legacy else tuple(out), () if legacy else tuple(ats))
                    self._published = (version, gen)
                    self.metrics.table_publish.observe(time.perf_counter() - tp, path="prepare")
                    if not legacy:
                        for c in out:
                            self._mark(c.uid, "tab")
        self._prune_replay_index(src)

    def _prune_replay_index(self, src) -> None:
        if self.journal.indexed_uids():         # replay index: only pods that can still be retried
            pend = {O.uid(p) for p in src.pending_pods()}
            self.journal.prune_index(pend)

    def _hold(self, claim, complete: bool) -> None:
        """A full-path match (caller holds ``_mu``): keep the pod claimed across its PATCH."""
        if claim is None:
            return
        self._revoked.discard(claim.uid)
        if complete:
            self._claims[claim.uid] = claim
        if self.native is not None:
            self.native.take(claim.uid)          # never answered from the table again

    def _await_watch(self, v0) -> bool:
        """Wait up to ``watch_grace_s`` for the pod watch to change the Pending set since
        ``v0``; True if it did (a retry of the cache match may now find the pod)."""
        wait = getattr(self.pods, "wait_pending_change", None)
        if wait is None or v0 is None or self.opts.watch_grace_s <= 0:
            return False
        t = time.perf_counter()
        changed = wait(v0, self.opts.watch_grace_s)
        self.metrics.allocate_latency.observe(time.perf_counter() - t, phase="watch_wait")
        return changed

    def _prepared(self, p: dict, u: str, g: int, units: int, kicks: list | None = None) -> "_Prepared":
        """The answer to a single-container pod's Allocate, serialized ahead of the request:
        the cached wire bytes of its (GPU, size) template followed by its per-pod ledger
        fields, encoded directly (protobuf: appended records of repeated / map fields merge
        into the message) — the same message ``_container_response`` builds, at a fraction of
        the cost on the watch thread (``tests/test_allocate_engine.py`` pins the equality).
        ``kicks``: the ledger and granter threads are not woken here; their wake-ups are
        appended, for the caller to run once the answer is published (on the way to the
        kubelet's Allocate, nothing else takes the interpreter)."""
        key = (self._gen, g, units)
        wake = kicks is None
        base = self._tmpl_bytes.get(key)
        if base is None:
            base = self._container_base(g, units, units, None).SerializeToString()
            if len(self._tmpl_bytes) > 512:
                self._tmpl_bytes.clear()
            self._tmpl_bytes[key] = base
        extra, lkey = b"", ""
        shim = self.opts.shim
        if shim is not None and shim.enabled and not self.opts.disable_cgpu:
            extra = _pb_map_entry(0x0a, const.ENV_SHIM_LEDGER, ledger_name(u or f"{g}-{time.time_ns()}", 0))
            if self._ledgers is not None:
                try:
                    lkey = self._ledgers.take(u, wake)
                    self._mark(u, "prep_ledger")
                    host = self._ledgers.path(lkey)
                    if not wake:
                        kicks.append(self._ledgers.kick)
                except OSError as e:
                    log.warning("ledger dir for pod %s: %s (pod-private shm ledger instead)", u, e)
                    lkey = ""
                else:
                    extra += (_pb_ld(0x12, _pb_ld(0x0a, const.LEDGER_CONTAINER_DIR.encode()) + _pb_ld(0x12, host.encode()))
                              + _pb_map_entry(0x0a, const.ENV_SHIM_LEDGER_DIR, const.LEDGER_CONTAINER_DIR)
                              + _pb_map_entry(0x22, const.CTR_ANNOTATION_LEDGER, lkey))
            hbm = self._hbm
            if hbm is not None:
                gg = self.model.gpu(g)
                tok = hbm.token(u or f"{g}-{time.time_ns()}", 0)
                qb = U.quota_bytes(units, gg.units, gg.vram_bytes)
                if wake:
                    ok = hbm.submit(g, tok, qb)
                else:
                    # the grant is recorded (and the granter woken) once the answer is published:
                    # the pod's TAKE comes at its container's start, long after
                    ok = hbm.grantable(g, qb)
                    if ok:
                        kicks.append(functools.partial(hbm.submit, g, tok, qb))
                self._mark(u, "prep_hbm")
                if ok:
                    extra += _pb_map_entry(0x0a, const.ENV_HBM_TOKEN, tok)
        body = _pb_ld(0x0a, base + extra)            # AllocateResponse.container_responses[0]
        return _Prepared(u, O.namespace(p), O.name(p), units, False, g, body,
                         AllocJournal.fast_head(u, O.namespace(p), O.name(p), body), lkey)

    def _allocate_full(self, req, t0: float):
        """The full Allocate path, counting the apiserver round trips it makes (the handler
        thread's requests; write-behind patches run on the patcher thread). With the native
        server, its answers are blocked meanwhile and its claims taken in first, so the two
        never hand out the same pod."""
        count = getattr(self.client, "thread_requests", None)
        n0 = count() if count else 0
        nat = self.native
        if nat is not None:
            nat.block()
            self._drain_native()
        try:
            view = getattr(self.pods, "allocate_view", None)
            with view() if view else contextlib.nullcontext():   # per-call sources: one LIST per Allocate
                return self._allocate_full_in(req, t0)
        finally:
            if count:
                self.metrics.allocate_requests.observe(count() - n0)
            if nat is not None:
                self._native_release(nat)

    def _native_release(self, nat) -> None:
        """End of a full-path Allocate: unblock the native answers — unless a multi-container
        claim is now open, whose next containers the engine must answer (one block is kept
        until that claim ends)."""
        with self._mu:
            open_claim = self._partial is not None
        if open_claim and not self._native_hold:
            self._native_hold = True
            return
        nat.unblock()
        if not open_claim and self._native_hold:
            self._native_hold = False
            nat.unblock()

    def _allocate_full_in(self, req, t0: float):
        sizes = tuple(len(c.devices_ids) for c in req.container_requests)
        pod_units = sum(sizes)
        log.info("----Allocating GPU for gpu mem is started---- RequestPodGPUs: %d", pod_units)
        hist = self.metrics.allocate_latency
        self._drain_post()
        jkey = request_key(req)
        replay = self._replay(req, jkey)
        if replay is not None:
            hist.observe(time.perf_counter() - t0, phase="total")
            return replay
        ta = time.perf_counter()
        try:
            held = self._identity_list(sizes)          # outside the lock (kubelet RPC)
            tl = time.perf_counter()
            v0 = getattr(self.pods, "pending_version", None)
            with self._mu:
                tb = time.perf_counter()
                claim, complete = self._match(sizes, fresh=False, held=held)
                t1 = time.perf_counter()
                self._hold(claim, complete)
            if claim is None and self._await_watch(v0):
                # watch lag: the kubelet saw the bind first; the pod watch delivered within the grace
                with self._mu:
                    claim, complete = self._match(sizes, fresh=False, held=held)
                    self._hold(claim, complete)
            if claim is None:
                # still not in the cache: an authoritative LIST (per-call sources: the view
                # already is one)
                with self._mu:
                    claim, complete = self._match(sizes, fresh=True, held=held)
                    self._hold(claim, complete)
            t2 = time.perf_counter()
            hist.observe(ta - t0, phase="prelude")      # request key, journal replay check
            hist.observe(tl - ta, phase="identity")     # pod-resources List (ambiguous requests only)
            hist.observe(tb - tl, phase="lock")
            hist.observe(t1 - tb, phase="lookup")
            hist.observe(t2 - t1, phase="decide")
        except Exception as e:  # noqa: BLE001 - pod listing failures
            log.info("invalid allocation request: Failed to find candidate pods due to %s", e)
            return self._err_response(req, pod_units)

        if claim is None:
            self.metrics.pending_match_failures.inc()
            if self.model.count() == 1:
                g = self.model.gpu(0)
                log.info("this node has only one gpu device, skip to search pod and directly specify the "
                         "device %d(%s) for container", 0, g.uuid)
                resp = api.AllocateResponse()
                for i, creq in enumerate(req.container_requests):
                    resp.container_responses.append(self._container_response(0, pod_units, len(creq.devices_ids),
                                                                             "", i))
                self._record_grants(req, resp, "", jkey)
                self.metrics.allocate_outcomes.inc(outcome="single_gpu")
                hist.observe(time.perf_counter() - t0, phase="total")
                return resp
            log.warning("invalid allocation request: request GPU memory %d can't be satisfied.", pod_units)
            return self._err_response(req, pod_units)

        idx = claim.gpu_index
        self._mark(claim.uid, "alloc_in", int(t0 * 1e9))     # perf_counter is CLOCK_MONOTONIC here
        self._mark(claim.uid, "path", "full")
        if self.model.gpu(idx) is None:
            log.warning("Failed to find the dev for pod %s because it's not able to find dev with index %d",
                        O.name(claim.pod), idx)
            with self._mu:
                self._claims.pop(claim.uid, None)
                if self._partial is claim:
                    self._partial = None
            return self._err_response(req, pod_units)

        pod_total = O.gpu_mem_of_pod(claim.pod)
        cu = self._plan_slots(claim, pod_total)
        resp = api.AllocateResponse()
        slot0 = claim.next_container - len(req.container_requests)
        for i, creq in enumerate(req.container_requests):
            resp.container_responses.append(self._container_response(idx, pod_total, len(creq.devices_ids),
                                                                     claim.uid, max(0, slot0 + i), cu))
        self._record_grants(req, resp, claim.uid, jkey)
        if not complete:
            log.info("pod %s: container %d/%d of a multi-container pod allocated on GPU %d", O.name(claim.pod),
                     claim.next_container, len(claim.shape), idx)
            self.metrics.allocate_outcomes.inc(outcome="partial")
            hist.observe(time.perf_counter() - t0, phase="total")
            return resp

        t3 = time.perf_counter()
        if self._patch_q is not None:
            job = _PatchJob(claim.uid, O.namespace(claim.pod), O.name(claim.pod), self._extra_annotations(claim.uid))
            # claimed as unpatched before the journal says "answered", so the reconcile pass
            # never queues a second, annotation-less patch for it in between
            with self._mu:
                self._claims.pop(claim.uid, None)
                self._assigned[claim.uid] = time.monotonic()
                self._unpatched.add(claim.uid)
            # journal before the reply (answer + pending PATCH, one write): a crash after the
            # reply must not lose the PATCH
            self.journal.record_pending(req, claim.uid, resp, job.ns, job.name, job.ann, jkey)
            self._patch_q.put(job)
            hist.observe(time.perf_counter() - t3, phase="patch")
            hist.observe(time.perf_counter() - t0, phase="total")
            self.metrics.allocate_outcomes.inc(outcome="assigned")
            log.info("pod %s, new allocated GPUs info: gpu index %d uuid %s (patch queued)", O.name(claim.pod), idx,
                     self.model.uuid_by_index(idx))
            return resp
        try:
            updated = self._patch_assigned(claim.pod)
        except Exception as e:  # noqa: BLE001
            log.warning("Failed due to %s", e)
            with self._mu:
                self._claims.pop(claim.uid, None)
            self._drop_slots(claim.uid)
            return self._err_response(req, pod_units)
        t4 = time.perf_counter()
        with self._mu:
            self._claims.pop(claim.uid, None)
            self._assigned[claim.uid] = time.monotonic()
        if updated:
            self.pods.observe(updated)
            self._drop_slots(claim.uid)
        self.journal.record(req, claim.uid, resp, jkey)
        hist.observe(t4 - t3, phase="patch")
        hist.observe(time.perf_counter() - t0, phase="total")
        self.metrics.allocate_outcomes.inc(outcome="assigned")
        log.info("pod %s, new allocated GPUs info: gpu index %d uuid %s", O.name(claim.pod), idx,
                 self.model.uuid_by_index(idx))
        return resp

    @staticmethod
    def _grant_from(cresp, uid: str, t: float) -> PL.Grant:
        e = cresp.envs
        return PL.Grant(gpu=int(e.get(const.ENV_RESOURCE_INDEX, "-1")), units=int(e.get(const.ENV_RESOURCE_BY_CONTAINER, "0")),
                        claimed=uid, t=t, cu=e.get(const.ENV_CU_SLOTS),
                        ledger=cresp.annotations.get(const.CTR_ANNOTATION_LEDGER, ""))

    def _record_grants(self, req, resp, uid: str, jkey: str) -> None:
        self._answer_seq += 1
        self._last_grant = time.monotonic()
        t = time.time()
        crs = req.container_requests
        for i, cresp in enumerate(resp.container_responses):
            key = jkey if len(crs) == 1 else PL.ids_key(crs[i].devices_ids)
            self.grants.record(key, self._grant_from(cresp, uid, t))

    def _replay(self, req, key: str):
        """Idempotent retry: the same fake-ID set for a pod we already assigned that is still
        Pending on this node gets the journaled answer (see alloc/journal.py)."""
        if not len(self.journal):
            return None
        hit = self.journal.lookup(req, key)
        if hit is None:
            return None
        uid, resp = hit
        # the kubelet recycles freed fake IDs, so under churn most key hits belong to pods that
        # are gone: one O(1) cache lookup decides (round 2 scanned every node pod here); a
        # per-call source answers from the Allocate's one LIST of Pending pods (allocate_view)
        try:
            p = self.pods.get_pending(uid)
        except Exception:  # noqa: BLE001
            return None
        if (p is not None and O.phase(p) == "Pending" and not O.deleting(p)
                and (A.is_assigned_pod(p) or uid in self._assigned)):
            self.metrics.allocate_outcomes.inc(outcome="replay")
            log.warning("Allocate retried for pod %s (same device IDs, still Pending): replaying the "
                        "journaled answer", O.name(p))
            return resp()
        return None

    def _patcher(self):
        """Lands queued ASSIGNED=true patches (retrying with backoff until the pod is gone),
        journals each landing, and when idle reconciles pods this plugin answered that still
        read ASSIGNED=false."""
        import queue
        while not self._stop.is_set():
            try:
                job = self._patch_q.get(timeout=1.0)
            except queue.Empty:
                if time.monotonic() - self._last_reconcile >= self.opts.reconcile_s:
                    self.reconcile()
                continue
            if job is None:
                break
            try:
                self._drain_post()
            except Exception as e:  # noqa: BLE001 - bookkeeping must never stop the patcher
                log.warning("fast-path bookkeeping failed: %s", e)
            delay = 0.05
            while not self._stop.is_set():
                try:
                    updated = self._land(job)
                    if updated:
                        self.pods.observe(updated)
                    self._drop_slots(job.uid)
                    break
                except APIError as e:
                    if e.not_found:
                        self._drop_slots(job.uid)
                        break
                    log.warning("assign patch for %s failed (%s); retrying", job.name, e)
                except Exception as e:  # noqa: BLE001 - transport errors
                    log.warning("assign patch for %s failed (%s); retrying", job.name, e)
                self._stop.wait(delay)
                delay = min(delay * 2, 5.0)
            else:
                break
            self._landed(job)

    def _landed(self, job: "_PatchJob") -> None:
        if job.kind == "placement":
            with self._mu:
                if self._overlay_gen.get(job.uid) == job.gen:
                    self._overlay.pop(job.uid, None)
                    self._overlay_gen.pop(job.uid, None)
                    self._bump_gen("placement_landed")
            return
        self.journal.landed(job.uid)
        with self._mu:
            self._unpatched.discard(job.uid)
            if job.uid not in self._revoked:
                self._assigned[job.uid] = time.monotonic()

    def _land(self, job: "_PatchJob") -> dict | None:
        """One ASSIGNED PATCH of a queued job. The patch carries the pod's UID, and a job
        recovered from the journal (or a conflict) first checks that the pod of that name is
        still the one we answered: a re-created pod with the same name is never patched."""
        if self.client is None:
            return None
        if job.recovered:
            cur = self.client.get_pod(job.ns, job.name)
            if O.uid(cur) != job.uid:
                log.warning("pod %s/%s was re-created (uid %s, answered %s): dropping its pending patch",
                            job.ns, job.name, O.uid(cur), job.uid)
                return None
            if job.kind == "assign" and A.is_assigned_pod(cur):
                return cur
        if job.kind == "placement":
            patch = {"metadata": {"annotations": dict(job.ann)}}
        else:
            patch = A.assigned_patch()
            patch["metadata"]["annotations"].update(job.ann)
        patch["metadata"]["uid"] = job.uid
        try:
            return self.client.patch_pod(job.ns, job.name, patch)
        except APIError as e:
            if e.conflict or e.status == 422:
                job.recovered = True      # re-check the pod's identity on the next attempt
            raise

    def reconcile(self) -> int:
        """Re-queue the ASSIGNED patch of every bound pod this plugin answered (journal) that
        still reads ASSIGNED=false and has no patch in flight — the write-behind counterpart of
        the reference's "answer only after the PATCH landed" (``allocate.go:132-152``)."""
        self._last_reconcile = time.monotonic()
        if self._patch_q is None or self.client is None:
            return 0
        try:
            pods = A.dedupe_by_uid(self.pods.node_pods(), self.node)
        except Exception as e:  # noqa: BLE001
            log.warning("reconcile: cannot list pods: %s", e)
            return 0
        n = 0
        for p in pods:
            u = O.uid(p)
            if O.deleting(p) or A.is_assigned_pod(p) or not A.is_assumed_pod(p) or not self.journal.answered(u):
                continue
            with self._mu:
                if u in self._unpatched:
                    continue
                self._unpatched.add(u)
                self._assigned[u] = time.monotonic()
                if self.native is not None:
                    self.native.take(u)
            self._patch_q.put(_PatchJob(u, O.namespace(p), O.name(p), self._extra_annotations(u), recovered=True))
            self.metrics.allocate_outcomes.inc(outcome="patch_reconciled")
            log.warning("reconcile: pod %s answered by this plugin still reads ASSIGNED=false; patching", O.name(p))
            n += 1
        return n

    # ------------------------------------------------------------------------------------
    # placement truth (alloc/placement.py)
    # ------------------------------------------------------------------------------------
    def set_pod_resources(self, src) -> None:
        """Attach the kubelet's pod-resources view (``api.podresources.PodResourcesClient`` or
        any object with ``list() -> [PodDevices]``) and start the periodic placement pass."""
        self.podres = src
        if src is not None and self._place_thread is None and self.opts.placement_s > 0:
            def loop():
                last = 0.0
                while not self._stop.wait(self.opts.placement_s):
                    # every placement_s while answers are in flight (the kubelet has not shown
                    # who holds them yet), otherwise a slow safety pass: a List of every pod's
                    # devices is not free on a busy node
                    now = time.monotonic()
                    busy = now - self._last_grant < self.opts.in_flight_s
                    if not busy and now - last < 15 * self.opts.placement_s:
                        continue
                    last = now
                    try:
                        self.reconcile_placement()
                    except Exception as e:  # noqa: BLE001 - kubelet restarting, apiserver down
                        log.V(2).info("placement pass failed: %s", e)
            self._place_thread = threading.Thread(target=loop, name="placement", daemon=True)
            self._place_thread.start()

    def prestart(self, req) -> None:
        """``PreStartContainer``: the kubelet checkpointed this container's fake IDs and is
        about to start it — make the pod annotations tell the truth first, then run the
        ``prestart_hooks`` (kernel HBM limits on the pod cgroup, quota/dmem.py)."""
        if self.podres is not None:
            try:
                self.reconcile_placement()
            except Exception as e:  # noqa: BLE001 - never block a container start on bookkeeping
                log.warning("placement check before container start failed: %s", e)
        for hook in list(self.prestart_hooks):
            try:
                hook()
            except Exception as e:  # noqa: BLE001
                log.warning("pre-start hook failed: %s", e)

    def reconcile_placement(self) -> list:
        """One placement pass: join the grant book with the kubelet's pod-resources view and
        queue (write-behind) or apply (sync) the annotation fixes ``placement.plan`` returns."""
        src = self.podres
        if src is None:
            return []
        self._drain_post()
        with self._place_mu:
            t_pass = time.monotonic()
            held = src.list()
            pods = self._view(A.dedupe_by_uid(self.pods.node_pods(), self.node))
            now = time.time()
            fixes = [f for f in PL.plan(pods, held, self.grants, now, self.opts.in_flight_s)
                     if not self._patch_queued(f)]
            for f in fixes:
                self._apply_fix(f)
            live = {O.uid(p) for p in pods}
            self.grants.prune({PL.ids_key(ids) for pd in held for _, ids in pd.containers}, live, now,
                              self.opts.in_flight_s)
            self._placed_at = t_pass
            return fixes

    def _patch_queued(self, f: PL.Fix) -> bool:
        """A holder fix that would only set ASSIGNED=true on a pod whose own answer's ASSIGNED
        patch is still queued (write-behind): that patch says the same. Applying it anyway would
        queue a second PATCH and retire the prepared table twice (placement overlay, then its
        landing), and the next Allocates would wait for a rebuild."""
        if f.reason != "holder" or f.ann or f.assigned is not True:
            return False
        with self._mu:
            return f.uid in self._unpatched

    def settled(self, uid: str) -> bool:
        """The pod's annotations are known to tell where it runs: placement truth is on, a
        placement pass has run since the last answer of this node, and nothing of the pod (its
        answer's PATCH, a placement fix, a multi-container claim) is in flight. The quota
        watchdog kills only settled pods (quota/watchdog.py)."""
        if self.podres is None or self._post or self._placed_at < self._last_grant:
            return False
        if self.native is not None and self.native.pending():
            return False
        with self._mu:
            return uid not in self._overlay and uid not in self._unpatched and uid not in self._claims

    def view(self, pods: list[dict]) -> list[dict]:
        """``pods`` as they read once this plugin's queued annotation fixes have landed."""
        with self._mu:
            return self._view(pods)

    def _apply_fix(self, f: PL.Fix) -> None:
        if f.reason == "rehomed" and f.assigned is None:
            # this plugin claimed the pod (its ASSIGNED patch may still be queued, so the pod
            # can read ASSIGNED=false) but another pod consumed the reservation: re-arm it, and
            # make its annotation say so once the queued patch has landed — else the pod's own
            # Allocate finds it claimed (and, after that patch, assigned) and fails
            with self._mu:
                claimed = f.uid in self._assigned or f.uid in self._unpatched or f.uid in self._claims
            if claimed:
                f = dataclasses.replace(f, assigned=False)
        ann = dict(f.ann)
        if f.assigned is True:
            ann.update(A.assigned_patch()["metadata"]["annotations"])
        elif f.assigned is False:
            ann[const.ENV_ASSIGNED_FLAG] = "false"
        self.metrics.allocate_outcomes.inc(outcome=f"placement_{f.reason}")
        with self._mu:        # the last fixes, for /debug/latency (why a prepared table was retired)
            self.placement_log.append({"uid": f.uid, "reason": f.reason, "ann": sorted(f.ann), "assigned": f.assigned,
                                       "unpatched": f.uid in self._unpatched, "answered": f.uid in self._assigned,
                                       "t": round(time.monotonic(), 3)})
            del self.placement_log[:-16]
        log.warning("placement: pod %s/%s %s -> %s", f.ns, f.name,
                    "holds its containers' grants" if f.reason == "holder" else "reservation re-homed",
                    {k: v for k, v in ann.items() if k != const.ENV_RESOURCE_ASSUME_TIME})
        with self._mu:
            gen = self._overlay_gen.get(f.uid, 0) + 1
            self._overlay_gen[f.uid] = gen
            self._overlay[f.uid] = dict(self._overlay.get(f.uid) or {}, **ann)
            self._bump_gen("placement_overlay")
            if f.assigned is True:
                self._assigned[f.uid] = time.monotonic()
                self._revoked.discard(f.uid)
            elif f.assigned is False:
                # its reservation was consumed by another pod: match it again on admission
                self._assigned.pop(f.uid, None)
                self._revoked.add(f.uid)
                self._claims.pop(f.uid, None)
        if f.assigned is False:
            self.journal.forget(f.uid)
            self._drop_slots(f.uid)
        if self._ledgers is not None:
            for k in f.holder_of:          # the holder's containers write these ledgers
                g = self.grants.get(k)
                if g is not None and g.ledger and g.claimed != f.uid:
                    try:
                        self._ledgers.add_owner(g.ledger, f.uid)
                    except OSError as e:
                        log.warning("ledger owner record %s: %s", g.ledger, e)
        job = _PatchJob(f.uid, f.ns, f.name, ann, kind="placement", gen=gen)
        if self._patch_q is not None:
            self._patch_q.put(job)
            return
        try:
            updated = self._land(job)
            if updated:
                self.pods.observe(updated)
        except APIError as e:
            if not e.not_found:
                raise
        self._landed(job)

    def flush_patches(self, timeout: float = 10.0) -> bool:
        """Wait until every queued ASSIGNED patch has landed (tests, shutdown)."""
        t = time.monotonic() + timeout
        while time.monotonic() < t:
            with self._mu:
                if not self._unpatched and not self._overlay:
                    return True
            time.sleep(0.005)
        return False

    def _extra_annotations(self, uid: str) -> dict:
        with self._slot_mu:
            pend = self._slot_pending.get(uid)
        return {const.POD_ANNOTATION_CU_SLOTS: pend[1].annotation()} if pend is not None else {}

    def _patch_assigned(self, pod: dict) -> dict | None:
        if self.client is None:
            return None
        patch = A.assigned_patch()
        patch["metadata"]["annotations"].update(self._extra_annotations(O.uid(pod)))
        ns, nm = O.namespace(pod), O.name(pod)
        try:
            return self.client.patch_pod(ns, nm, patch)
        except APIError as e:
            if e.conflict:  # optimistic-lock conflict: retry once (allocate.go:140-147)
                return self.client.patch_pod(ns, nm, patch)
            raise

    def preferred(self, req) -> api.PreferredAllocationResponse:
        """``GetPreferredAllocation`` — the reference panics (``server.go:37-40``). Here: prefer
        fake IDs that belong to the GPU the extender chose for the oldest matching pending
        pod, so the kubelet's device checkpoint names the physical GPU actually used."""
        resp = api.PreferredAllocationResponse()
        try:
            with self._mu:
                cands = self._candidates(fresh=False)
        except Exception:  # noqa: BLE001
            cands = []
        for creq in req.container_requests:
            size = creq.allocation_size
            avail = list(creq.available_deviceIDs)
            must = list(creq.must_include_deviceIDs)
            target = None
            for p in cands:
                shape = self._info(p)[3]
                if shape and shape[0] == size:
                    target = self.model.uuid_by_index(A.gpu_id_from_annotation(p))
                    break
            picked = list(must)
            taken = set(must)
            if target:   # one linear pass, no sort: IDs of the target GPU first
                prefix = target + const.FAKE_ID_SEP
                for d in avail:
                    if len(picked) >= size:
                        break
                    if d.startswith(prefix) and d not in taken:
                        picked.append(d)
                        taken.add(d)
            for d in avail:
                if len(picked) >= size:
                    break
                if d not in taken:
                    picked.append(d)
                    taken.add(d)
            resp.container_responses.add(deviceIDs=picked[:max(size, len(must))])
        return resp


@dataclasses.dataclass
class _PatchJob:
    uid: str
    ns: str
    name: str
    ann: dict              # extra annotations landed with ASSIGNED=true (CU slots); placement: all
    recovered: bool = False
    kind: str = "assign"   # "assign" (ASSIGNED=true after an answer) | "placement" (truth fix)
    gen: int = 0           # placement: overlay generation this job lands


def env_shim_host_dir() -> str | None:
    return os.environ.get("GPUSHARE_SHIM_HOST_DIR")
