"""Compute isolation (``--compute-isolation=cu``, ``alloc/cuslots.py``): CU-slot runs laid out
symmetrically over the MI355X's 8 XCDs, chosen by the Allocate engine and carried on the pod."""
import json

from hypothesis import given, settings, strategies as st

from aliyun_gpushare_device_plugin_amd import const
from aliyun_gpushare_device_plugin_amd.alloc import cuslots as C
from aliyun_gpushare_device_plugin_amd.alloc.engine import Allocator, AllocatorOptions
from aliyun_gpushare_device_plugin_amd.device.model import DeviceModel
from tests.test_allocate_engine import NODE, FakeClient, StaticSource, mkpod, req
from tests.test_units_and_model import MI355X_BYTES, gpu


def test_mask_strings_follow_the_measured_bit_layout():
    # slot s = CU s of every XCD = bits [8s, 8s + 8) (profiles/cu_mask/README.md)
    r = C.SlotRun(0, 16)
    assert C.hsa_cu_mask(r, 8) == "0:0-127"
    assert C.roc_cu_mask(r, 8) == "0x" + "f" * 32
    r = C.SlotRun(14, 7)
    assert list(C.mask_bits(r, 8)) == list(range(112, 168))
    assert C.hsa_cu_mask(r, 8, device=3) == "3:112-167"
    assert int(C.roc_cu_mask(r, 8), 16) == sum(1 << b for b in range(112, 168))
    # every XCD gets the same CUs: bit b lands on XCD b % 8
    assert {b % 8 for b in C.mask_bits(C.SlotRun(5, 1), 8)} == set(range(8))


def test_annotation_roundtrip_and_malformed():
    assert C.SlotRun.parse("14-20") == C.SlotRun(14, 7)
    assert C.SlotRun.parse("3") == C.SlotRun(3, 1)
    assert C.SlotRun(14, 7).annotation() == "14-20"
    for bad in ("", None, "x", "5-2", "-1-3", "a-b"):
        assert C.SlotRun.parse(bad) is None


def test_wanted_slots_floor_by_hbm_share():
    # BASELINE config 3 patterns on 288 GiB / 32 slots: each pattern fits exclusively
    for pattern in ([128, 64, 64, 32], [96, 96, 64, 32], [128, 96, 56, 8], [64, 64, 96, 64]):
        ks = [C.wanted_slots(u, 288, 32) for u in pattern]
        assert sum(ks) <= 32 and min(ks) >= 1
    assert C.wanted_slots(8, 288, 32) == 1            # below one slot -> one slot
    assert C.wanted_slots(288, 288, 32) == 32
    assert C.wanted_slots(8, 288, 32, request="12") == 12
    assert C.wanted_slots(8, 288, 32, request="99") == 32
    assert C.wanted_slots(8, 288, 32, request="junk") == 1


def test_choose_best_fit_then_least_loaded():
    run, excl = C.choose([], 7, 32)
    assert run == C.SlotRun(0, 7) and excl
    held = [C.SlotRun(0, 14), C.SlotRun(20, 4)]          # gaps: [14,20) len 6, [24,32) len 8
    assert C.choose(held, 5, 32) == (C.SlotRun(14, 5), True)    # smallest gap that fits
    assert C.choose(held, 7, 32) == (C.SlotRun(24, 7), True)
    full = [C.SlotRun(0, 16), C.SlotRun(16, 16)]
    run, excl = C.choose(full, 4, 32)
    assert not excl and run == C.SlotRun(0, 4)
    run, excl = C.choose(full + [C.SlotRun(0, 8)], 4, 32)      # least-loaded run
    assert not excl and run == C.SlotRun(8, 4)


@settings(max_examples=200, deadline=None)
@given(st.lists(st.integers(min_value=1, max_value=32), min_size=1, max_size=12))
def test_choose_never_overlaps_while_slots_remain(ks):
    held = []
    for k in ks:
        run, excl = C.choose(held, k, 32)
        assert 0 <= run.start and run.end <= 32 and run.count == k
        busy = {s for r in held for s in range(r.start, r.end)}
        overlap = busy & set(range(run.start, run.end))
        assert excl == (not overlap)
        if 32 - len(busy) >= k and excl is False:
            # exclusive failed only because free slots are fragmented, never because of miscounting
            gaps = [g for g in _gaps(busy) if g >= k]
            assert not gaps
        held.append(run)


def _gaps(busy):
    out, n = [], 0
    for s in range(32):
        if s in busy:
            if n:
                out.append(n)
            n = 0
        else:
            n += 1
    return out + ([n] if n else [])


def _mi355x_allocator(pods, **opts):
    model = DeviceModel([gpu(i, MI355X_BYTES) for i in range(2)], const.GIB, round_policy="nearest")
    src = StaticSource(pods)
    cl = FakeClient(src)
    return Allocator(model, src, cl, NODE, AllocatorOptions(compute_isolation="cu", **opts)), src, cl


def _envs(resp):
    return dict(resp.container_responses[0].envs)


def test_engine_gives_disjoint_runs_and_records_them_on_the_pod():
    sizes = [128, 64, 64, 32]
    pods = [mkpod(f"p{i}", s, 0, 100 + i) for i, s in enumerate(sizes)]
    al, src, cl = _mi355x_allocator(pods)
    runs = []
    for s in sizes:
        e = _envs(al.allocate(req(s)))
        run = C.SlotRun.parse(e[const.ENV_CU_SLOTS])
        assert e[const.ENV_HSA_CU_MASK] == C.hsa_cu_mask(run, 8, 0)
        assert e[const.ENV_ROC_CU_MASK] == C.roc_cu_mask(run, 8)
        runs.append(run)
    assert [r.count for r in runs] == [14, 7, 7, 3]
    assert 'gpushare_cu_slots_held{gpu="0"} 31' in al.metrics.registry.render()
    slots = [s for r in runs for s in range(r.start, r.end)]
    assert len(slots) == len(set(slots))                        # exclusive
    patched = {name: p["metadata"]["annotations"] for _, name, p in cl.patches}
    assert [patched[f"p{i}"][const.POD_ANNOTATION_CU_SLOTS] for i in range(4)] == [r.annotation() for r in runs]


def test_replacement_pod_reuses_the_retired_pods_slots():
    pods = [mkpod(f"p{i}", s, 0, 100 + i) for i, s in enumerate([128, 64, 64, 32])]
    al, src, cl = _mi355x_allocator(pods)
    runs = {}
    for i, s in enumerate([128, 64, 64, 32]):
        runs[f"p{i}"] = C.SlotRun.parse(_envs(al.allocate(req(s)))[const.ENV_CU_SLOTS])
    for p in src.pods:
        p["status"]["phase"] = "Running"
    src.pods = [p for p in src.pods if p["metadata"]["name"] != "p1"]      # retire a 64 GiB pod
    src.pods.append(mkpod("p4", 64, 0, 200))
    e = _envs(al.allocate(req(64)))
    assert C.SlotRun.parse(e[const.ENV_CU_SLOTS]) == runs["p1"]


def test_other_gpu_and_terminal_pods_do_not_hold_slots():
    done = mkpod("done", 128, 0, 1, assigned="true", phase="Succeeded")
    done["metadata"]["annotations"][const.POD_ANNOTATION_CU_SLOTS] = "0-13"
    other = mkpod("other", 128, 1, 2, assigned="true", phase="Running")
    other["metadata"]["annotations"][const.POD_ANNOTATION_CU_SLOTS] = "0-13"
    al, src, cl = _mi355x_allocator([done, other, mkpod("new", 128, 0, 300)])
    assert _envs(al.allocate(req(128)))[const.ENV_CU_SLOTS] == "0-13"


def test_slot_request_annotation_and_oversubscription_metric():
    big = mkpod("big", 8, 0, 1)
    big["metadata"]["annotations"][const.POD_ANNOTATION_CU_SLOTS_REQUEST] = "32"
    al, src, cl = _mi355x_allocator([big, mkpod("small", 16, 0, 2)])
    assert _envs(al.allocate(req(8)))[const.ENV_CU_SLOTS] == "0-31"
    assert _envs(al.allocate(req(16)))[const.ENV_CU_SLOTS] == "0-0"            # shared: least loaded
    text = al.metrics.registry.render()
    assert 'outcome="cu_shared"' in text


def test_write_behind_patch_carries_slots_and_concurrent_admissions_stay_disjoint():
    import concurrent.futures as cf

    pods = [mkpod(f"p{i}", 32, 0, 100 + i) for i in range(8)]   # 8 x 3 slots
    al, src, cl = _mi355x_allocator(pods, async_patch=True)
    with cf.ThreadPoolExecutor(8) as ex:
        outs = list(ex.map(lambda _: _envs(al.allocate(req(32))), range(8)))
    assert al.flush_patches()
    runs = [C.SlotRun.parse(e[const.ENV_CU_SLOTS]) for e in outs]
    slots = [s for r in runs for s in range(r.start, r.end)]
    assert len(slots) == 24 and len(set(slots)) == 24
    ann = {name: p["metadata"]["annotations"][const.POD_ANNOTATION_CU_SLOTS] for _, name, p in cl.patches}
    assert sorted(ann.values()) == sorted(r.annotation() for r in runs)


def test_isolation_off_by_default_and_with_cgpu_disabled():
    model = DeviceModel([gpu(0, MI355X_BYTES)], const.GIB, round_policy="nearest")
    for opts in ({}, {"compute_isolation": "cu", "disable_cgpu": True}):
        src = StaticSource([mkpod("a", 64, 0, 1)])
        al = Allocator(model, src, FakeClient(src), NODE, AllocatorOptions(**opts))
        e = _envs(al.allocate(req(64)))
        assert const.ENV_HSA_CU_MASK not in e and const.ENV_CU_SLOTS not in e


def test_cli_flag_reaches_the_allocator():
    from aliyun_gpushare_device_plugin_amd.cli.main import build_parser, config_from_args

    a = build_parser().parse_args(["--compute-isolation", "cu"])
    assert config_from_args(a).compute_isolation == "cu"
    assert config_from_args(build_parser().parse_args([])).compute_isolation == "none"
    json.dumps({"ok": True})


def test_e2e_compute_isolation_through_the_fake_cluster():
    """Real plugin process, fake kubelet/apiserver/extender: a full MI355X gets 4 pods with
    disjoint CU-slot runs; each run is on the pod object; a replacement reuses the freed run."""
    from aliyun_gpushare_device_plugin_amd.cluster import objects as O
    from aliyun_gpushare_device_plugin_amd.sim.cluster import SimCluster

    with SimCluster([("n", "fake:1x309220868096B")], plugin_mode="process", compute_isolation="cu") as c:
        pods, runs = [], []
        for s in (128, 64, 64, 32):
            pod, where, adm = c.run_pod(s)
            assert where == ("n", 0) and adm.error is None
            e = dict(adm.responses[0].envs)
            run = C.SlotRun.parse(e[const.ENV_CU_SLOTS])
            assert e[const.ENV_HSA_CU_MASK] == C.hsa_cu_mask(run, 8, 0)
            assert O.annotations(c.wait_assigned(pod))[const.POD_ANNOTATION_CU_SLOTS] == run.annotation()
            pods.append(pod)
            runs.append(run)
        slots = [s for r in runs for s in range(r.start, r.end)]
        assert len(slots) == len(set(slots)) == 31
        c.delete_pod(pods[1])
        _, where, adm = c.run_pod(64)
        assert C.SlotRun.parse(dict(adm.responses[0].envs)[const.ENV_CU_SLOTS]) == runs[1]


def test_e2e_slot_request_annotation_survives_scheduling():
    from aliyun_gpushare_device_plugin_amd.sim.cluster import SimCluster

    with SimCluster([("n", "fake:1x309220868096B")], compute_isolation="cu") as c:
        req_ann = {const.POD_ANNOTATION_CU_SLOTS_REQUEST: "16"}
        got = []
        for name in ("a", "b"):
            _, where, adm = c.run_pod(64, name=name, annotations=req_ann)
            assert adm.error is None
            got.append(dict(adm.responses[0].envs)[const.ENV_HSA_CU_MASK])
        assert got == ["0:0-127", "0:128-255"]


def test_slots_survive_a_plugin_restart():
    """The plugin keeps no slot state of its own: after a restart (SIGHUP) it rebuilds the GPU's
    occupied slots from the pods' annotations and hands the next pod a disjoint run."""
    import signal
    import time

    from aliyun_gpushare_device_plugin_amd.sim.cluster import SimCluster

    with SimCluster([("n", "fake:1x309220868096B")], compute_isolation="cu") as c:
        runs = []
        for s in (128, 64):
            pod, _, adm = c.run_pod(s)
            runs.append(C.SlotRun.parse(dict(adm.responses[0].envs)[const.ENV_CU_SLOTS]))
            c.wait_assigned(pod)
        mgr = c.manager("n")
        mgr.events.put(("signal", signal.SIGHUP))
        t = time.time() + 10
        while mgr.restarts < 1 and time.time() < t:
            time.sleep(0.05)
        assert mgr.restarts == 1 and c.nodes["n"].kubelet.registered.wait(10)
        _, _, adm = c.run_pod(64)
        new = C.SlotRun.parse(dict(adm.responses[0].envs)[const.ENV_CU_SLOTS])
        held = {s for r in runs for s in range(r.start, r.end)}
        assert not held & set(range(new.start, new.end)), (runs, new)
