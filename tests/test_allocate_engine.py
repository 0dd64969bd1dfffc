"""Allocate engine (component C5) and annotation protocol (C7), without gRPC or HTTP."""
import concurrent.futures as cf
import itertools
import json
import os
import threading
import time

import pytest

from aliyun_gpushare_device_plugin_amd import const
from aliyun_gpushare_device_plugin_amd.alloc import annotations as A
from aliyun_gpushare_device_plugin_amd.alloc.engine import AllocationError, Allocator, AllocatorOptions
from aliyun_gpushare_device_plugin_amd.api import v1beta1 as api
from aliyun_gpushare_device_plugin_amd.cluster.podcache import PodSource
from aliyun_gpushare_device_plugin_amd.device.model import DeviceModel
from aliyun_gpushare_device_plugin_amd.quota import ShimConfig
from tests.test_units_and_model import gpu

NODE = "node-a"


def mkpod(name, mems, idx=None, assume=None, assigned="false", node=NODE, phase="Pending", uid=None):
    mems = [mems] if isinstance(mems, int) else mems
    ann = {}
    if idx is not None:
        ann[const.ENV_RESOURCE_INDEX] = str(idx)
    if assume is not None:
        ann[const.ENV_RESOURCE_ASSUME_TIME] = str(assume)
    if assigned is not None:
        ann[const.ENV_ASSIGNED_FLAG] = assigned
    return {"metadata": {"name": name, "namespace": "default", "uid": uid or f"uid-{name}", "annotations": ann,
                         "resourceVersion": "1"},
            "spec": {"nodeName": node, "containers": [
                {"name": f"c{i}", "resources": {"limits": {const.RESOURCE_NAME: str(m)}} if m else {}}
                for i, m in enumerate(mems)]},
            "status": {"phase": phase}}


class StaticSource(PodSource):
    def __init__(self, pods):
        self.pods = list(pods)
        self.fresh_calls = 0
        self.observed = []

    def pending_pods(self, fresh=False):
        if fresh:
            self.fresh_calls += 1
        return [p for p in self.pods if p["status"]["phase"] == "Pending"]

    def node_pods(self):
        return [p for p in self.pods if p["status"]["phase"] in ("Pending", "Running")]

    def observe(self, pod):
        self.observed.append(pod)
        for i, p in enumerate(self.pods):
            if p["metadata"]["uid"] == pod["metadata"]["uid"]:
                self.pods[i] = pod


class FakeClient:
    """Records PATCHes and applies them to the source's pods."""

    def __init__(self, source, fail=None, delay=0.0):
        self.source, self.fail, self.delay = source, fail, delay
        self.patches = []
        self.lock = threading.Lock()

    def patch_pod(self, ns, name, patch, content_type=None):
        time.sleep(self.delay)
        if self.fail:
            raise self.fail
        with self.lock:
            self.patches.append((ns, name, patch))
            for p in self.source.pods:
                if p["metadata"]["name"] == name:
                    new = json.loads(json.dumps(p))
                    new["metadata"]["annotations"].update(patch["metadata"]["annotations"])
                    new["metadata"]["resourceVersion"] = str(int(p["metadata"]["resourceVersion"]) + 1)
                    return new
        return None


_IDS = itertools.count()


def req(*sizes):
    """Like the kubelet: every admission gets fake IDs no other live pod holds."""
    return api.AllocateRequest(container_requests=[
        api.ContainerAllocateRequest(devices_ids=[f"id-{next(_IDS)}" for _ in range(n)]) for n in sizes])


def make(pods, ngpu=2, gib=4, **opts):
    model = DeviceModel([gpu(i, gib << 30) for i in range(ngpu)], const.GIB)
    src = StaticSource(pods)
    cl = FakeClient(src)
    return Allocator(model, src, cl, NODE, AllocatorOptions(**opts)), src, cl


# ---- annotations -------------------------------------------------------------------------

def test_assumed_pod_rules():
    assert A.is_assumed_pod(mkpod("a", 2, 0, 10))
    assert not A.is_assumed_pod(mkpod("a", 2, 0, 10, assigned="true"))
    assert not A.is_assumed_pod(mkpod("a", 2, 0, None))           # no assume time
    assert not A.is_assumed_pod(mkpod("a", 2, 0, 10, assigned=None))
    assert not A.is_assumed_pod(mkpod("a", 0, 0, 10))             # no gpu-mem


def test_annotation_parsing_and_order():
    p = mkpod("a", 2, "x", "junk")
    assert A.gpu_id_from_annotation(p) == -1 and A.assume_time(p) == 0
    pods = [mkpod("b", 1, 0, 30), mkpod("a", 1, 0, 10), mkpod("c", 1, 0, 20)]
    assert [x["metadata"]["name"] for x in A.order_by_assume_time(pods)] == ["a", "c", "b"]
    patch = A.assigned_patch(123)
    assert patch == {"metadata": {"annotations": {const.ENV_ASSIGNED_FLAG: "true",
                                                  const.ENV_RESOURCE_ASSUME_TIME: "123"}}}


def test_dedupe_drops_other_nodes():
    pods = [mkpod("a", 1, 0, 1), mkpod("a", 1, 0, 1), mkpod("b", 1, 0, 1, node="other")]
    assert [p["metadata"]["name"] for p in A.dedupe_by_uid(pods, NODE)] == ["a"]


def test_allocation_annotation():
    p = mkpod("a", 4, 0, 1)
    p["metadata"]["annotations"][const.GPUSHARE_ALLOCATION_FLAG] = json.dumps({"0": {"1": 2}, "1": {"1": 1, "0": 1}})
    assert A.allocation_from_annotation(p) == {1: 3, 0: 1}
    p["metadata"]["annotations"][const.GPUSHARE_ALLOCATION_FLAG] = "{bad"
    assert A.allocation_from_annotation(p) == {}


# ---- engine ------------------------------------------------------------------------------

def test_matches_oldest_equal_request_and_patches():
    al, src, cl = make([mkpod("young", 2, 1, 200), mkpod("old", 2, 0, 100), mkpod("other", 3, 1, 50)])
    r = al.allocate(req(2))
    envs = dict(r.container_responses[0].envs)
    assert envs[const.ENV_RESOURCE_INDEX] == "0"
    assert envs[const.ENV_RESOURCE_BY_POD] == "2" and envs[const.ENV_RESOURCE_BY_CONTAINER] == "2"
    assert envs[const.ENV_RESOURCE_BY_DEV] == "4" and envs[const.ENV_GPU_UUID] == "GPU-0000000000000000"
    assert "NVIDIA_VISIBLE_DEVICES" not in envs
    assert [d.host_path for d in r.container_responses[0].devices] == ["/dev/kfd", "/dev/dri/renderD128"]
    assert cl.patches[0][1] == "old"
    assert cl.patches[0][2]["metadata"]["annotations"][const.ENV_ASSIGNED_FLAG] == "true"
    # the just-assigned pod is never matched again, even before a cache refresh
    r2 = al.allocate(req(2))
    assert dict(r2.container_responses[0].envs)[const.ENV_RESOURCE_INDEX] == "1"
    assert [p[1] for p in cl.patches] == ["old", "young"]


def test_no_match_multi_gpu_gives_error_response():
    al, src, cl = make([mkpod("a", 3, 0, 1)])
    r = al.allocate(req(2))
    envs = dict(r.container_responses[0].envs)
    assert envs[const.ENV_RESOURCE_INDEX] == "-1"
    assert envs["GPUSHARE_ALLOCATION_ERROR"] == "no-gpu-has-2GiB-to-run"
    assert len(r.container_responses[0].devices) == 0
    assert src.fresh_calls == 1        # cache miss -> one fresh LIST before giving up


def test_strict_mode_raises():
    al, _, _ = make([], strict=True)
    with pytest.raises(AllocationError):
        al.allocate(req(2))


def test_single_gpu_fallback_without_pod():
    al, _, cl = make([], ngpu=1)
    r = al.allocate(req(2))
    envs = dict(r.container_responses[0].envs)
    assert envs[const.ENV_RESOURCE_INDEX] == "0" and not cl.patches


def test_bad_index_annotation_is_error():
    al, _, cl = make([mkpod("a", 2, 7, 1)])
    assert dict(al.allocate(req(2)).container_responses[0].envs)[const.ENV_RESOURCE_INDEX] == "-1"
    assert not cl.patches


def test_patch_failure_releases_claim():
    al, src, cl = make([mkpod("a", 2, 0, 1)])
    cl.fail = RuntimeError("apiserver down")
    assert dict(al.allocate(req(2)).container_responses[0].envs)[const.ENV_RESOURCE_INDEX] == "-1"
    cl.fail = None
    assert dict(al.allocate(req(2)).container_responses[0].envs)[const.ENV_RESOURCE_INDEX] == "0"


def test_multi_container_pod_matched_per_container():
    # reference quirk 3: a pod with 2 gpu containers (1 + 3) never matched a per-container request
    al, src, cl = make([mkpod("mc", [1, 0, 3], 1, 5)])
    r1 = al.allocate(req(1))
    assert dict(r1.container_responses[0].envs)[const.ENV_RESOURCE_INDEX] == "1"
    assert dict(r1.container_responses[0].envs)[const.ENV_RESOURCE_BY_POD] == "4"
    assert not cl.patches                       # not all containers allocated yet
    r2 = al.allocate(req(3))
    assert dict(r2.container_responses[0].envs)[const.ENV_RESOURCE_INDEX] == "1"
    assert [p[1] for p in cl.patches] == ["mc"]


def test_whole_pod_request_matches_only_its_own_shape():
    """One AllocateRequest naming every gpu container (not what the kubelet sends, but valid
    on the wire) matches the pod whose per-container shape it is, never one with an equal
    total but a different shape."""
    al, _, cl = make([mkpod("other", [4], 1, 1), mkpod("mc", [1, 3], 0, 5)])
    r = al.allocate(req(1, 3))
    assert [dict(c.envs)[const.ENV_RESOURCE_INDEX] for c in r.container_responses] == ["0", "0"]
    assert [p[1] for p in cl.patches] == ["mc"]


def test_single_container_request_never_takes_multi_container_pod():
    """Regression (round-1 review): pod M [8,8] on GPU 0 assumed first, pod X [16] on GPU 1.
    The kubelet admits X first: X must get GPU 1, M keeps its reservation for its own two
    Allocate(8) calls."""
    m, x = mkpod("m", [8, 8], 0, 100), mkpod("x", [16], 1, 200)
    al, src, cl = make([m, x], gib=32)
    rx = dict(al.allocate(req(16)).container_responses[0].envs)
    assert rx[const.ENV_RESOURCE_INDEX] == "1"
    assert [p[1] for p in cl.patches] == ["x"]
    x["status"]["phase"] = "Running"
    for _ in range(2):
        assert dict(al.allocate(req(8)).container_responses[0].envs)[const.ENV_RESOURCE_INDEX] == "0"
    assert [p[1] for p in cl.patches] == ["x", "m"]


def test_partial_claim_of_deleted_pod_is_dropped():
    """Regression (round-1 advice): M [8,8] on GPU 0 gets its first container, then M is
    deleted. A later single-container pod Y [8] on GPU 1 must get GPU 1, and M is never
    patched."""
    m, y = mkpod("m", [8, 8], 0, 100), mkpod("y", [8], 1, 200)
    al, src, cl = make([m], gib=32)
    assert dict(al.allocate(req(8)).container_responses[0].envs)[const.ENV_RESOURCE_INDEX] == "0"
    src.pods.remove(m)
    src.pods.append(y)
    assert dict(al.allocate(req(8)).container_responses[0].envs)[const.ENV_RESOURCE_INDEX] == "1"
    assert [p[1] for p in cl.patches] == ["y"]
    assert al.metrics.allocate_outcomes.value(outcome="claim_abandoned") == 1


def test_stale_or_deleting_partial_claim():
    """A claim the kubelet does not continue within partial_claim_ttl_s may have fed a pod
    that is now running: its reservation is withheld (never double-booked). A claim whose pod
    is being deleted is simply dropped."""
    m, y = mkpod("m", [8, 8], 0, 100), mkpod("y", [8], 1, 200)
    al, src, cl = make([m, y], gib=32, partial_claim_ttl_s=0.05)
    assert dict(al.allocate(req(8)).container_responses[0].envs)[const.ENV_RESOURCE_INDEX] == "0"
    time.sleep(0.1)
    assert dict(al.allocate(req(8)).container_responses[0].envs)[const.ENV_RESOURCE_INDEX] == "1"
    assert [p[1] for p in cl.patches] == ["y"]
    assert al.metrics.allocate_outcomes.value(outcome="claim_tainted") == 1
    assert dict(al.allocate(req(8)).container_responses[0].envs)[const.ENV_RESOURCE_INDEX] == "-1"
    # graceful deletion (deletionTimestamp) ends a claim without withholding anything
    m2 = mkpod("m2", [4, 4], 0, 300)
    src.pods.append(m2)
    assert dict(al.allocate(req(4)).container_responses[0].envs)[const.ENV_RESOURCE_INDEX] == "0"
    m2["metadata"]["deletionTimestamp"] = "2026-01-01T00:00:00Z"
    assert dict(al.allocate(req(4)).container_responses[0].envs)[const.ENV_RESOURCE_INDEX] == "-1"
    assert "m2" not in [p[1] for p in cl.patches]
    assert al.metrics.allocate_outcomes.value(outcome="claim_abandoned") == 1


def test_mismatched_continuation_is_retargeted_or_withheld():
    """A claim is continued only by the next Allocate. When that container does not fit the
    claimed pod, another pod with the same first container was being admitted: the claimed
    reservation is withheld (it feeds that pod), and the claim moves to a pod that extends
    the answered containers on the same GPU, or the container is matched afresh."""
    m, p2 = mkpod("m", [2, 6], 0, 100), mkpod("p2", [2, 3], 0, 150)
    z = mkpod("z", [3], 1, 200)
    al, src, cl = make([m, p2, z], gib=16)
    assert dict(al.allocate(req(2)).container_responses[0].envs)[const.ENV_RESOURCE_INDEX] == "0"   # claims m
    assert dict(al.allocate(req(3)).container_responses[0].envs)[const.ENV_RESOURCE_INDEX] == "0"   # it was p2
    assert [p[1] for p in cl.patches] == ["p2"]
    assert al.metrics.allocate_outcomes.value(outcome="claim_retargeted") == 1
    # m's reservation fed p2's first container: never handed out again while m lives
    assert dict(al.allocate(req(2)).container_responses[0].envs)[const.ENV_RESOURCE_INDEX] == "-1"
    assert dict(al.allocate(req(3)).container_responses[0].envs)[const.ENV_RESOURCE_INDEX] == "1"
    assert [p[1] for p in cl.patches] == ["p2", "z"]


def test_swapped_multi_container_pods_exchange_reservations():
    """M2 [4,4] (GPU 1) is admitted before M1 [4,4] (GPU 0, assumed first): M2 takes M1's
    reservation container by container; M1 then completes with M2's (swap completion)."""
    now = time.time_ns()
    m1, m2 = mkpod("m1", [4, 4], 0, now - 2000), mkpod("m2", [4, 4], 1, now - 1000)
    al, src, cl = make([m1, m2], gib=16)
    first = [dict(al.allocate(req(4)).container_responses[0].envs)[const.ENV_RESOURCE_INDEX] for _ in range(2)]
    assert first == ["0", "0"] and [p[1] for p in cl.patches] == ["m1"]
    m2["status"]["phase"] = "Running"
    second = [dict(al.allocate(req(4)).container_responses[0].envs)[const.ENV_RESOURCE_INDEX] for _ in range(2)]
    assert second == ["1", "1"] and [p[1] for p in cl.patches] == ["m1", "m2"]


def test_concurrent_allocates_never_double_assign():
    pods = [mkpod(f"p{i}", 2, i % 2, 100 + i) for i in range(16)]
    al, src, cl = make(pods)
    cl.delay = 0.005            # PATCH in flight while other Allocates run
    with cf.ThreadPoolExecutor(8) as ex:
        rs = list(ex.map(lambda _: al.allocate(req(2)), range(16)))
    names = [p[1] for p in cl.patches]
    assert sorted(names) == sorted(f"p{i}" for i in range(16))
    assert all(dict(r.container_responses[0].envs)[const.ENV_RESOURCE_INDEX] != "-1" for r in rs)


def test_shim_injection_and_cgpu_disable():
    shim = ShimConfig(host_dir="/opt/gpushare/lib")
    al, _, _ = make([mkpod("a", 2, 0, 1)], shim=shim)
    r = al.allocate(req(2)).container_responses[0]
    assert r.envs[const.ENV_LD_PRELOAD] == "/usr/local/gpushare/libgpushare_hipquota.so"
    assert r.envs[const.ENV_SHIM_LEDGER].startswith("/gpushare-uida-")
    assert r.envs[const.ENV_SHIM_QUOTA_BYTES] == str((4 << 30) * 2 // 4)      # 2 of 4 GiB units
    assert r.mounts[0].host_path == "/opt/gpushare/lib" and r.mounts[0].read_only
    al, _, _ = make([mkpod("a", 2, 0, 1)], shim=shim, disable_cgpu=True)
    r = al.allocate(req(2)).container_responses[0]
    assert r.envs[const.ENV_CGPU_DISABLE] == "true" and const.ENV_LD_PRELOAD not in r.envs
    assert len(r.mounts) == 0


def test_preferred_allocation_picks_assigned_gpu():
    al, _, _ = make([mkpod("a", 2, 1, 1)])
    avail = [f"GPU-{g:016x}-_-{j}" for g in (0, 1) for j in range(4)]
    r = al.preferred(api.PreferredAllocationRequest(container_requests=[
        api.ContainerPreferredAllocationRequest(available_deviceIDs=avail, allocation_size=2)]))
    ids = list(r.container_responses[0].deviceIDs)
    assert len(ids) == 2 and all(i.startswith("GPU-0000000000000001") for i in ids)


def test_metrics_recorded():
    al, _, _ = make([mkpod("a", 2, 0, 1)])
    al.allocate(req(2))
    assert al.metrics.allocate_outcomes.value(outcome="assigned") == 1
    assert al.metrics.allocate_latency.count(phase="total") == 1
    assert "gpushare_allocate_latency_seconds_bucket" in al.metrics.registry.render()


def test_async_patch_write_behind_and_retry():
    al, src, cl = make([mkpod(f"p{i}", 2, i % 2, 10 + i) for i in range(4)], async_patch=True)
    cl.fail = RuntimeError("apiserver flaky")
    r = [al.allocate(req(2)) for _ in range(2)]
    assert [dict(x.container_responses[0].envs)[const.ENV_RESOURCE_INDEX] for x in r] == ["0", "1"]
    assert not cl.patches                      # answered before the PATCH landed
    assert not al.flush_patches(0.2)           # still failing -> still pending, claims held
    assert dict(al.allocate(req(2)).container_responses[0].envs)[const.ENV_RESOURCE_INDEX] == "0"  # p2, not p0
    cl.fail = None
    assert al.flush_patches(5.0)
    assert sorted(p[1] for p in cl.patches) == ["p0", "p1", "p2"]
    assert all(p["metadata"]["annotations"][const.ENV_ASSIGNED_FLAG] == "true"
               for p in src.pods if p["metadata"]["name"] in ("p0", "p1", "p2"))


@pytest.mark.parametrize("complete", [True, False])
def test_swapped_admission_order_is_completed(complete):
    """The kubelet admits b before a (equal size): the first Allocate takes a's reservation
    (earliest assume time), b turns Running un-assigned; a's own Allocate then gets b's GPU."""
    now = time.time_ns()
    a, b = mkpod("a", 2, 0, now - 2000), mkpod("b", 2, 1, now - 1000)
    al, src, cl = make([a, b], complete_swaps=complete)
    first = dict(al.allocate(req(2)).container_responses[0].envs)
    assert first[const.ENV_RESOURCE_INDEX] == "0"          # reference rule: earliest assumed pod
    b["status"]["phase"] = "Running"                       # the kubelet started b's containers
    second = dict(al.allocate(req(2)).container_responses[0].envs)
    if complete:
        assert second[const.ENV_RESOURCE_INDEX] == "1"
        assert all(A.is_assigned_pod(p) for p in src.pods)
        assert al.metrics.allocate_outcomes.value(outcome="swap") == 1
    else:
        assert second[const.ENV_RESOURCE_INDEX] == "-1"   # the reference's failure
    # a stale un-assigned running pod (assumed long ago) is never taken
    old = mkpod("old", 2, 1, now - int(600e9), phase="Running")
    al2, _, _ = make([old])
    assert dict(al2.allocate(req(2)).container_responses[0].envs)[const.ENV_RESOURCE_INDEX] == "-1"


def test_ledger_dir_mount_and_env(tmp_path):
    """Round-2 review: every shared container used to get the node-wide ledger directory
    read-write. Now each answered container gets its own subdirectory (root 0755, plugin-owned;
    owner records outside any mount), so a tenant can neither read nor rewrite a neighbour's
    ledger."""
    from aliyun_gpushare_device_plugin_amd.quota import ShimConfig
    from aliyun_gpushare_device_plugin_amd.quota import ledger as L
    root = tmp_path / "ledgers"
    al, _, _ = make([mkpod("p", 2, 1, 10), mkpod("q", 2, 0, 20)], shim=ShimConfig("/opt/gpushare"),
                    ledger_dir=str(root))
    rp, rq = (al.allocate(req(2)).container_responses[0] for _ in range(2))
    mp, mq = ({m.container_path: (m.host_path, m.read_only) for m in r.mounts} for r in (rp, rq))
    assert mp[const.SHIM_CONTAINER_DIR] == ("/opt/gpushare", True)
    hp, hq = mp[const.LEDGER_CONTAINER_DIR][0], mq[const.LEDGER_CONTAINER_DIR][0]
    assert mp[const.LEDGER_CONTAINER_DIR][1] is False
    assert hp != hq and os.path.dirname(hp) == os.path.dirname(hq) == str(root)
    assert os.path.basename(hp) == rp.annotations[const.CTR_ANNOTATION_LEDGER]
    assert rp.envs[const.ENV_SHIM_LEDGER_DIR] == const.LEDGER_CONTAINER_DIR
    assert oct(os.stat(root).st_mode & 0o7777) == "0o755"
    assert oct(os.stat(hp).st_mode & 0o777) == "0o777"
    assert al._ledgers.flush()                   # owner records are written behind the answer
    ld = L.LedgerDir(str(root))
    assert ld.owners(os.path.basename(hp))[0] == ["uid-p"] and ld.owners(os.path.basename(hq))[0] == ["uid-q"]
    # nothing of q's is reachable below p's mount (the only host path p's container sees)
    (tmp_path / "ledgers" / os.path.basename(hq) / "gpushare-uidq-0.ledger").write_bytes(b"x")
    assert os.listdir(hp) == []
    al2, _, _ = make([mkpod("p", 2, 1, 10)], shim=ShimConfig("/opt/gpushare"))
    assert const.ENV_SHIM_LEDGER_DIR not in al2.allocate(req(2)).container_responses[0].envs


def test_journal_replays_retried_admission(tmp_path):
    """The kubelet re-sends Allocate for a pod we already assigned (still Pending): same answer,
    even from a new plugin instance reading the persisted journal; once the pod runs, or the
    IDs come back for another pod, normal matching applies."""
    path = str(tmp_path / "journal.jsonl")
    a, b = mkpod("a", 2, 1, 10), mkpod("b", 2, 0, 20)
    al, src, _ = make([a, b], journal_path=path)
    r = req(2)
    first = dict(al.allocate(r).container_responses[0].envs)
    assert first[const.ENV_RESOURCE_INDEX] == "1"                       # a (oldest)
    again = dict(al.allocate(r).container_responses[0].envs)
    assert again == first and al.metrics.allocate_outcomes.value(outcome="replay") == 1
    # a new plugin process: journal loaded from disk
    al2 = Allocator(al.model, src, al.client, "node-a", AllocatorOptions(journal_path=path))
    assert dict(al2.allocate(r).container_responses[0].envs) == first
    # pod a started running: the same IDs now belong to a new admission -> b is matched
    for p in src.pods:
        if p["metadata"]["name"] == "a":
            p["status"]["phase"] = "Running"
    assert dict(al2.allocate(r).container_responses[0].envs)[const.ENV_RESOURCE_INDEX] == "0"


def test_cdi_device_names():
    """--cdi-kind: the GPU is also named as a CDI device (the spec AMD's container toolkit
    generates carries /dev/kfd and its render node); with DeviceSpecs off it is the only one."""
    al, _, _ = make([mkpod("p", 2, 1, 10)], cdi_kind="amd.com/gpu")
    r = al.allocate(req(2)).container_responses[0]
    assert [c.name for c in r.cdi_devices] == ["amd.com/gpu=1"] and len(r.devices) >= 1
    al2, _, _ = make([mkpod("p", 2, 0, 10)], cdi_kind="amd.com/gpu", expose_devices=False)
    r2 = al2.allocate(req(2)).container_responses[0]
    assert [c.name for c in r2.cdi_devices] == ["amd.com/gpu=0"] and len(r2.devices) == 0


class VersionedSource(StaticSource):
    """A StaticSource with the watch cache's change signal (enables the fast path)."""

    def __init__(self, pods):
        super().__init__(pods)
        self.version = 1
        self.changed = threading.Event()


def test_fast_path_retry_before_bookkeeping_replays():
    """a fast-path answer is indexed for replay off the hot path. A kubelet retry of
    the same fake-ID set that arrives before that bookkeeping must still replay the answer, not
    take the next candidate's reservation (one pod matched twice)."""
    model = DeviceModel([gpu(i, 4 << 30) for i in range(2)], const.GIB)
    src = VersionedSource([mkpod("a", 2, 1, 10), mkpod("b", 2, 0, 20)])
    al = Allocator(model, src, FakeClient(src), NODE, AllocatorOptions(async_patch=True))
    try:
        held = []
        al._patch_q = type("Q", (), {"put": lambda self, j: held.append(j)})()   # patcher never drains
        al._prepare(src)
        assert al._fast is not None
        r = req(2)
        first = al.allocate(r)
        assert al.metrics.allocate_latency.count(phase="fast") == 1 and al._post     # not indexed yet
        again = al.allocate(r)
        assert dict(again.container_responses[0].envs) == dict(first.container_responses[0].envs)
        assert dict(first.container_responses[0].envs)[const.ENV_RESOURCE_INDEX] == "1"
        assert al.metrics.allocate_outcomes.value(outcome="replay") == 1
        # b is still free for its own admission
        assert dict(al.allocate(req(2)).container_responses[0].envs)[const.ENV_RESOURCE_INDEX] == "0"
    finally:
        al.close()


def test_prepare_discards_answers_built_before_a_reconfigure():
    """a _prepare that raced a reconfigure must not install answers built from the
    old device model."""
    model = DeviceModel([gpu(i, 4 << 30) for i in range(2)], const.GIB)
    src = VersionedSource([mkpod("a", 2, 1, 10)])
    al = Allocator(model, src, FakeClient(src), NODE, AllocatorOptions(async_patch=True))
    try:
        orig = al._candidates

        def racing(fresh):
            out = orig(fresh)
            al._gen += 1                  # a reconfigure lands while answers are being built
            return out
        al._candidates = racing
        al._fast = None
        al._prep_cache.clear()
        al._prepare(src)
        assert al._fast is None and not al._prep_cache
    finally:
        al.close()


class LaggingWatch(StaticSource):
    """A watch-backed source whose pod watch delivers a bound pod after the kubelet asked."""

    def __init__(self, pods):
        super().__init__(pods)
        self.pending_version = 1
        self.cv = threading.Condition()
        self.watched = {p["metadata"]["uid"] for p in pods}

    def pending_pods(self, fresh=False):
        got = super().pending_pods(fresh)
        return got if fresh else [p for p in got if p["metadata"]["uid"] in self.watched]

    def deliver(self, pod):
        with self.cv:
            self.pods.append(pod)
            self.watched.add(pod["metadata"]["uid"])
            self.pending_version += 1
            self.cv.notify_all()

    def wait_pending_change(self, version, timeout):
        with self.cv:
            return self.cv.wait_for(lambda: self.pending_version != version, timeout)


def _lag_engine(src, grace):
    model = DeviceModel([gpu(i, 8 << 30) for i in range(2)], const.GIB)
    return Allocator(model, src, FakeClient(src), NODE,
                     AllocatorOptions(async_patch=True, fast_path=False, watch_grace_s=grace))


def test_allocate_waits_for_a_lagging_watch_instead_of_listing():
    """The kubelet's watch delivered the bind before the plugin's: the Allocate waits (up to
    watch_grace_s) for the pod watch and answers from the cache, with no LIST on its path."""
    src = LaggingWatch([])
    al = _lag_engine(src, 0.2)
    try:
        threading.Timer(0.005, src.deliver, args=(mkpod("late", 3, 1, 10),)).start()
        t = time.perf_counter()
        r = al.allocate(req(3))
        assert r.container_responses[0].envs[const.ENV_RESOURCE_INDEX] == "1"
        assert src.fresh_calls == 0 and time.perf_counter() - t < 0.15
    finally:
        al.close()


def test_allocate_lists_once_the_watch_grace_runs_out():
    src = LaggingWatch([])
    al = _lag_engine(src, 0.02)
    try:
        src.pods.append(mkpod("unseen", 3, 0, 10))          # in the apiserver, never in the watch
        r = al.allocate(req(3))
        assert r.container_responses[0].envs[const.ENV_RESOURCE_INDEX] == "0"
        assert src.fresh_calls == 1
    finally:
        al.close()


@pytest.mark.parametrize("shim,ledgers,disable_cgpu,cdi,rocr", [
    (False, False, False, None, False), (True, False, False, None, False), (True, True, False, None, False),
    (True, True, True, None, False), (True, True, False, "amd.com/gpu", True)])
def test_prepared_body_is_the_container_response(tmp_path, shim, ledgers, disable_cgpu, cdi, rocr):
    """The hand-encoded prepared answer (template bytes + per-pod ledger fields) parses to the
    same AllocateResponse the engine builds field by field."""
    model = DeviceModel([gpu(i, 8 << 30) for i in range(2)], const.GIB)
    src = StaticSource([])
    opts = AllocatorOptions(shim=ShimConfig(host_dir=str(tmp_path / "shim")) if shim else None,
                            ledger_dir=str(tmp_path / "ledgers") if ledgers else None,
                            disable_cgpu=disable_cgpu, cdi_kind=cdi, rocr_visible=rocr)
    al = Allocator(model, src, FakeClient(src), NODE, opts)
    try:
        for i in range(3):
            pod = mkpod(f"b{i}", 3, 1, 10)
            c = al._prepared(pod, f"uid-b{i}", 1, 3)
            got = api.AllocateResponse.FromString(c.body)
            want_cr = al._container_response(1, 3, 3, f"uid-b{i}", 0, None)
            # the ledger directory differs per call (a fresh key each time): compare the rest
            for cr in (got.container_responses[0], want_cr):
                if const.CTR_ANNOTATION_LEDGER in cr.annotations:
                    assert cr.annotations[const.CTR_ANNOTATION_LEDGER]
                    del cr.annotations[const.CTR_ANNOTATION_LEDGER]
                for m in [m for m in cr.mounts if m.container_path == const.LEDGER_CONTAINER_DIR]:
                    m.host_path = "<ledger>"
            want = api.AllocateResponse()
            want.container_responses.append(want_cr)
            assert got == want
            assert (c.lkey != "") == (ledgers and shim and not disable_cgpu)
    finally:
        al.close()


class _FakeBrokerAdmin:
    """The admin socket of one GPU's HBM broker: records GRANTs / REVOKEs, answers OK, and STAT /
    LIST with a fixed boot id."""

    def __init__(self, path, ok=True, boot="b00t"):
        import socket as _s

        os.makedirs(os.path.dirname(path), exist_ok=True)
        self.grants, self.revokes = [], []
        self.held: dict = {}
        self.limits: dict = {}
        self.ok, self.boot = ok, boot
        self.ls = _s.socket(_s.AF_UNIX, _s.SOCK_STREAM)
        self.ls.bind(path)
        self.ls.listen(16)
        threading.Thread(target=self._serve, daemon=True).start()

    def _serve(self):
        import json as _j

        while True:
            try:
                c, _ = self.ls.accept()
            except OSError:
                return
            buf = b""
            while not buf.endswith(b"\n"):
                chunk = c.recv(256)
                if not chunk:
                    break
                buf += chunk
            w = buf.decode().split()
            if w[:1] == ["STAT"]:
                c.sendall((_j.dumps({"boot": self.boot}) + "\n").encode())
            elif w[:1] == ["LIST"]:
                c.sendall((_j.dumps({"boot": self.boot, "grants": self.held}) + "\n").encode())
            elif w[:1] == ["REVOKE"]:
                self.revokes.append(w[1])
                self.held.pop(w[1], None)
                c.sendall(b"OK 0\n")
            else:
                _, tok, nbytes = w[:3]
                self.limits[tok] = int(w[3]) if len(w) > 3 else None     # the pod's whole quota
                self.grants.append((tok, int(nbytes)))
                if self.ok:
                    self.held[tok] = int(nbytes) >> 30
                c.sendall(f"OK {int(nbytes) >> 30}\n".encode() if self.ok else b"ERR size\n")
            c.close()


def test_hbm_broker_grant_rides_in_the_prepared_answer(tmp_path):
    """With --hbm-broker-dir the answer mounts only the GPU's pod-socket directory (read-only; the
    admin sockets stay outside it), names the GPU's socket and carries the pod's token, granted on
    that GPU's broker off the thread that prepares the answer; the hand-encoded prepared answer and
    the field-by-field one stay equal, and a re-prepared answer grants nothing new. Tokens come
    from the node secret (0600), so a new plugin instance derives the same ones. A GPU whose
    broker never appears gets tokens during the start-up grace (the pod waits for it), then none
    (the pod allocates from the driver at once)."""
    import time as _t

    from aliyun_gpushare_device_plugin_amd.quota import hbmbroker

    model = DeviceModel([gpu(i, 64 << 30) for i in range(2)], const.GIB)
    src = StaticSource([])
    hdir = tmp_path / "hbm"
    hdir.mkdir()
    admin = _FakeBrokerAdmin(hbmbroker.admin_socket(str(hdir), 1))
    opts = AllocatorOptions(shim=ShimConfig(host_dir=str(tmp_path / "shim")), hbm_broker_dir=str(hdir),
                            hbm_granter_args={"poll_s": 0.1, "startup_grace_s": 1.0, "down_grace_s": 0.5})
    al = Allocator(model, src, FakeClient(src), NODE, opts)
    try:
        assert oct(os.stat(hbmbroker.secret_path(str(hdir))).st_mode & 0o777) == "0o600"
        pod = mkpod("h0", 16, 1, 10)
        c = al._prepared(pod, "uid-h0", 1, 16)
        got = api.AllocateResponse.FromString(c.body).container_responses[0]
        want = al._container_response(1, 16, 16, "uid-h0", 0, None)
        assert got == want
        tok = got.envs[const.ENV_HBM_TOKEN]
        assert got.envs[const.ENV_HBM_BROKER] == f"{const.HBM_BROKER_CONTAINER_DIR}/hbm1.sock"
        assert got.envs[const.ENV_HIP_FORCE_DEV_KERNARG] == "0"     # (hipGraph next to a broker neighbour)
        mounts = [m for m in got.mounts if m.container_path == const.HBM_BROKER_CONTAINER_DIR]
        assert len(mounts) == 1 and mounts[0].host_path == str(hdir / "gpu1") and mounts[0].read_only
        # 16 of 64 GiB -> a 16 GiB quota; 94 % of it in whole granules = 15 GiB, granted once
        assert al._hbm.flush()
        assert admin.grants == [(tok, 15 << 30)] and admin.limits[tok] == 16 << 30   # may borrow up to the quota
        assert al._prepared(pod, "uid-h0", 1, 16).body == c.body
        assert al._hbm.flush() and len(admin.grants) == 1
        # the same node secret in another instance: the same token for the same pod and slot
        g2 = hbmbroker.HBMGranter(str(hdir), start=False)
        assert g2.token("uid-h0", 0) == tok and g2.token("uid-h0", 1) != tok
        # GPU 0 has no broker: within the start-up grace its answers carry the token (the shim
        # waits for the broker); once the grace is over they do not
        r0 = al._container_response(0, 16, 16, "uid-h1", 0, None)
        assert const.ENV_HBM_TOKEN in r0.envs and r0.envs[const.ENV_HBM_BROKER].endswith("hbm0.sock")
        _t.sleep(1.3)
        assert al._hbm.reconcile_now()
        r2 = al._container_response(0, 16, 16, "uid-h2", 0, None)
        assert const.ENV_HBM_TOKEN not in r2.envs
        r3 = al._container_response(1, 16, 16, "uid-h3", 0, None)      # GPU 1's broker is up
        assert const.ENV_HBM_TOKEN in r3.envs
        # too small for two granules: no arena, no grant
        small = al._container_response(1, 1, 1, "uid-h4", 0, None)
        assert const.ENV_HBM_TOKEN not in small.envs
        assert al._hbm.flush() and {t for t, _ in admin.grants} == {tok, r3.envs[const.ENV_HBM_TOKEN]}
    finally:
        al.close()
