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
  extender-reserved GPUs, so per-GPU accounting stays exact.
"""
from __future__ import annotations

import dataclasses
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
from ..utils import log
from ..utils.metrics import PluginMetrics
from . import annotations as A
from . import cuslots
from .journal import AllocJournal, request_key


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


@dataclasses.dataclass
class _Claim:
    uid: str
    pod: dict
    gpu_index: int
    next_container: int
    gpu_containers: list   # indices of containers that request gpu-mem
    t: float
    slots: cuslots.SlotRun | None = None


class Allocator:
    def __init__(self, model: DeviceModel, pods: PodSource, client: APIClient | None, node: str,
                 opts: AllocatorOptions | None = None, metrics: PluginMetrics | None = None):
        self.model, self.pods, self.client, self.node = model, pods, client, node
        self.opts = opts or AllocatorOptions()
        self.metrics = metrics or PluginMetrics()
        self._mu = threading.Lock()
        self._claims: dict[str, _Claim] = {}      # in-flight (multi-container or PATCH pending)
        self._assigned: dict[str, float] = {}     # uid -> time we assigned it (stale-cache guard)
        self._unpatched: set[str] = set()         # assigned locally, PATCH not yet acknowledged
        self._pinfo: dict[tuple, tuple] = {}      # memoised per-pod-version facts (see _info)
        self._patch_q = None
        self._slot_mu = threading.Lock()
        self._slot_pending: dict[str, tuple] = {}  # uid -> (gpu, SlotRun, t): chosen, not yet on the pod
        self.journal = AllocJournal(self.opts.journal_path, self.opts.journal_ttl_s)
        if self.opts.async_patch:
            import queue
            self._patch_q = queue.Queue()
            threading.Thread(target=self._patcher, name="assign-patcher", daemon=True).start()

    # ------------------------------------------------------------------------------------
    # candidate selection
    # ------------------------------------------------------------------------------------
    def _info(self, p: dict) -> tuple[bool, int, int]:
        """(assumed, pod gpu-mem, assume time) of one pod version, memoised: every Allocate scans
        all Pending pods, and re-parsing their specs dominated the handler. The
        key carries the two annotations the plugin itself rewrites, so an object updated in
        place (no new resourceVersion) is never served stale."""
        ann = O.annotations(p)
        k = (O.uid(p), O.resource_version(p), ann.get(const.ENV_ASSIGNED_FLAG),
             ann.get(const.ENV_RESOURCE_ASSUME_TIME))
        v = self._pinfo.get(k)
        if v is None:
            v = (A.is_assumed_pod(p), O.gpu_mem_of_pod(p), A.assume_time(p))
            if len(self._pinfo) > 8192:
                self._pinfo.clear()
            self._pinfo[k] = v
        return v

    def _candidates(self, fresh: bool) -> list[dict]:
        pods = A.dedupe_by_uid(self.pods.pending_pods(fresh=fresh), self.node)
        now = time.monotonic()
        for u, t in list(self._assigned.items()):
            if now - t > self.opts.claim_ttl_s and u not in self._unpatched:
                del self._assigned[u]
        out = []
        for p in pods:
            assumed, _, at = self._info(p)
            if assumed and O.uid(p) not in self._assigned:
                out.append((at, len(out), p))
        out.sort(key=lambda e: (e[0], e[1]))      # assume time, then arrival order (stable)
        if log.V(4):
            for at, _, p in out:
                log.info("candidate pod %s in ns %s with timestamp %d is found.", O.name(p), O.namespace(p), at)
        return [p for _, _, p in out]

    def _match(self, req_units: int, fresh: bool) -> tuple[_Claim | None, bool]:
        """Returns (claim, complete). ``complete`` = every gpu container of the pod is now
        allocated, so the pod must be PATCHed ASSIGNED."""
        # 1) continue a multi-container pod already in progress (container order = kubelet order)
        for c in sorted(self._claims.values(), key=lambda c: A.assume_time(c.pod)):
            if c.next_container < len(c.gpu_containers):
                want = O.container_limit(O.containers(c.pod)[c.gpu_containers[c.next_container]])
                if want == req_units:
                    c.next_container += 1
                    return c, c.next_container == len(c.gpu_containers)
        cands = [p for p in self._candidates(fresh) if O.uid(p) not in self._claims]
        # 2) the reference rule: pod-total equals the request
        for p in cands:
            if self._info(p)[1] == req_units:
                gc = [i for i, v in enumerate(O.gpu_mem_per_container(p)) if v > 0]
                c = _Claim(O.uid(p), p, A.gpu_id_from_annotation(p), len(gc), gc, time.monotonic())
                return c, True
        # 3) multi-container pods: first gpu container's request equals this request
        if self.opts.match_containers:
            for p in cands:
                per = O.gpu_mem_per_container(p)
                gc = [i for i, v in enumerate(per) if v > 0]
                if len(gc) > 1 and per[gc[0]] == req_units:
                    c = _Claim(O.uid(p), p, A.gpu_id_from_annotation(p), 1, gc, time.monotonic())
                    self._claims[c.uid] = c
                    return c, False
        # 4) swap completion (authoritative pass only): see the module docstring
        if fresh and self.opts.complete_swaps:
            p = self._swap_partner(req_units)
            if p is not None:
                gc = [i for i, v in enumerate(O.gpu_mem_per_container(p)) if v > 0]
                self.metrics.allocate_outcomes.inc(outcome="swap")
                log.warning("no pending pod requests %d%s: completing a swapped admission with pod %s (gpu %d)",
                            req_units, self.opts.unit, O.name(p), A.gpu_id_from_annotation(p))
                return _Claim(O.uid(p), p, A.gpu_id_from_annotation(p), len(gc), gc, time.monotonic()), True
        return None, False

    def _swap_partner(self, req_units: int) -> dict | None:
        now_ns = time.time_ns()
        ttl_ns = int(self.opts.claim_ttl_s * 1e9)
        out = []
        for p in A.dedupe_by_uid(self.pods.node_pods(), self.node):
            u = O.uid(p)
            if (O.phase(p) == "Pending" or not A.is_assumed_pod(p) or u in self._assigned or u in self._claims
                    or O.gpu_mem_of_pod(p) != req_units or now_ns - A.assume_time(p) > ttl_ns):
                continue
            out.append(p)
        out = A.order_by_assume_time(out)
        return out[0] if out else None

    # ------------------------------------------------------------------------------------
    # response building
    # ------------------------------------------------------------------------------------
    def _container_response(self, gpu_index: int, pod_units: int, ctr_units: int, pod_uid: str,
                            slot: int, cu: cuslots.SlotRun | None = None) -> api.ContainerAllocateResponse:
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
        shim = self.opts.shim
        if shim is not None and shim.enabled and not self.opts.disable_cgpu:
            r.mounts.add(container_path=shim.container_dir, host_path=shim.host_dir, read_only=True)
            r.envs[const.ENV_LD_PRELOAD] = shim.container_lib
            r.envs[const.ENV_SHIM_LEDGER] = ledger_name(pod_uid or f"{gpu_index}-{time.time_ns()}", slot)
            if self.opts.ledger_dir:
                r.mounts.add(container_path=const.LEDGER_CONTAINER_DIR, host_path=self.opts.ledger_dir,
                             read_only=False)
                r.envs[const.ENV_SHIM_LEDGER_DIR] = const.LEDGER_CONTAINER_DIR
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
        t0 = time.perf_counter()
        pod_units = sum(len(c.devices_ids) for c in req.container_requests)
        log.info("----Allocating GPU for gpu mem is started---- RequestPodGPUs: %d", pod_units)
        hist = self.metrics.allocate_latency
        jkey = request_key(req)
        replay = self._replay(req, jkey)
        if replay is not None:
            hist.observe(time.perf_counter() - t0, phase="total")
            return replay
        try:
            with self._mu:
                claim, complete = self._match(pod_units, fresh=False)
                t1 = time.perf_counter()
                if claim is None:
                    # watch lag: the kubelet may see a bind before our cache does
                    claim, complete = self._match(pod_units, fresh=True)
                if claim is not None and complete:
                    self._claims[claim.uid] = claim   # held across the PATCH
                t2 = time.perf_counter()
            hist.observe(t1 - t0, phase="lookup")
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
                self.metrics.allocate_outcomes.inc(outcome="single_gpu")
                hist.observe(time.perf_counter() - t0, phase="total")
                return resp
            log.warning("invalid allocation request: request GPU memory %d can't be satisfied.", pod_units)
            return self._err_response(req, pod_units)

        idx = claim.gpu_index
        if self.model.gpu(idx) is None:
            log.warning("Failed to find the dev for pod %s because it's not able to find dev with index %d",
                        O.name(claim.pod), idx)
            with self._mu:
                self._claims.pop(claim.uid, None)
            return self._err_response(req, pod_units)

        pod_total = O.gpu_mem_of_pod(claim.pod)
        cu = self._plan_slots(claim, pod_total)
        resp = api.AllocateResponse()
        slot0 = claim.next_container - len(req.container_requests)
        for i, creq in enumerate(req.container_requests):
            resp.container_responses.append(self._container_response(idx, pod_total, len(creq.devices_ids),
                                                                     claim.uid, max(0, slot0 + i), cu))
        if not complete:
            log.info("pod %s: container %d/%d of a multi-container pod allocated on GPU %d", O.name(claim.pod),
                     claim.next_container, len(claim.gpu_containers), idx)
            self.metrics.allocate_outcomes.inc(outcome="partial")
            hist.observe(time.perf_counter() - t0, phase="total")
            return resp

        t3 = time.perf_counter()
        if self._patch_q is not None:
            with self._mu:
                self._claims.pop(claim.uid, None)
                self._assigned[claim.uid] = time.monotonic()
                self._unpatched.add(claim.uid)
            self._patch_q.put(claim.pod)
            self.journal.record(req, claim.uid, resp, jkey)
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

    def _replay(self, req, key: str):
        """Idempotent retry: the same fake-ID set for a pod we already assigned that is still
        Pending on this node gets the journaled answer (see alloc/journal.py)."""
        if not len(self.journal):
            return None
        hit = self.journal.lookup(req, key)
        if hit is None:
            return None
        uid, resp = hit
        try:
            pods = self.pods.node_pods()
        except Exception:  # noqa: BLE001
            return None
        for p in pods:
            if (O.uid(p) == uid and O.phase(p) == "Pending" and not (p.get("metadata") or {}).get("deletionTimestamp")
                    and (A.is_assigned_pod(p) or uid in self._assigned)):
                self.metrics.allocate_outcomes.inc(outcome="replay")
                log.warning("Allocate retried for pod %s (same device IDs, still Pending): replaying the "
                            "journaled answer", O.name(p))
                return resp
        return None

    def _patcher(self):
        """Lands queued ASSIGNED=true patches; retries with backoff until the pod is gone."""
        while True:
            pod = self._patch_q.get()
            delay = 0.05
            while True:
                try:
                    updated = self._patch_assigned(pod)
                    if updated:
                        self.pods.observe(updated)
                        self._drop_slots(O.uid(pod))
                    break
                except APIError as e:
                    if e.not_found:
                        self._drop_slots(O.uid(pod))
                        break
                    log.warning("assign patch for %s failed (%s); retrying", O.name(pod), e)
                except Exception as e:  # noqa: BLE001 - transport errors
                    log.warning("assign patch for %s failed (%s); retrying", O.name(pod), e)
                time.sleep(delay)
                delay = min(delay * 2, 5.0)
            with self._mu:
                self._unpatched.discard(O.uid(pod))
                self._assigned[O.uid(pod)] = time.monotonic()

    def flush_patches(self, timeout: float = 10.0) -> bool:
        """Wait until every queued ASSIGNED patch has landed (tests, shutdown)."""
        t = time.monotonic() + timeout
        while time.monotonic() < t:
            with self._mu:
                if not self._unpatched:
                    return True
            time.sleep(0.005)
        return False

    def _patch_assigned(self, pod: dict) -> dict | None:
        if self.client is None:
            return None
        patch = A.assigned_patch()
        with self._slot_mu:
            pend = self._slot_pending.get(O.uid(pod))
        if pend is not None:
            patch["metadata"]["annotations"][const.POD_ANNOTATION_CU_SLOTS] = pend[1].annotation()
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
                if O.gpu_mem_of_pod(p) == size or (O.gpu_mem_per_container(p) or [0])[0] == size:
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


def env_shim_host_dir() -> str | None:
    return os.environ.get("GPUSHARE_SHIM_HOST_DIR")
