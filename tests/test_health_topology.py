"""BASELINE config 5 on CPU: health path (hot-unplug, reset, ECC) with recovery, and xGMI
topology export + TP-pair placement reconcile, through the real plugin and fake kubelet."""
import json
import time

from aliyun_gpushare_device_plugin_amd import const
from aliyun_gpushare_device_plugin_amd.cluster import nodestatus, objects as O
from aliyun_gpushare_device_plugin_amd.parallel import topology as T
from aliyun_gpushare_device_plugin_amd.sim.cluster import SimCluster


def health_by_gpu(kl, model):
    out = {}
    for g in model.gpus:
        hs = {kl.devices.get(f"{g.uuid}-_-{j}") for j in range(g.units)}
        out[g.index] = hs.pop() if len(hs) == 1 else "mixed"
    return out


def wait(pred, timeout=10.0):
    t = time.time() + timeout
    while time.time() < t:
        if pred():
            return True
        time.sleep(0.02)
    return False


def test_hot_unplug_and_recovery_via_listandwatch():
    with SimCluster([("n", "fake:4x288G")], health_poll_s=0.2) as c:
        mgr, kl = c.manager("n"), c.nodes["n"].kubelet
        model = mgr.model
        assert set(health_by_gpu(kl, model).values()) == {const.HEALTHY}
        t0 = time.time()
        mgr.smi.inject("unplug 2")
        assert wait(lambda: health_by_gpu(kl, model)[2] == const.UNHEALTHY)
        time_to_unhealthy = time.time() - t0
        assert time_to_unhealthy < 2.0
        assert health_by_gpu(kl, model)[0] == const.HEALTHY
        # the node's allocatable drops by one GPU's units; health exported for the extender
        assert wait(lambda: O.node_allocatable(c.client.get_node("n"), const.RESOURCE_NAME) == 3 * 288)
        h = json.loads(O.annotations(c.client.get_node("n"))[const.NODE_ANNOTATION_HEALTH])
        assert h["2"]["healthy"] is False and "missing" in h["2"]["reason"]
        # the extender no longer places pods on GPU 2
        c.extender.sync()
        placed = [c.run_pod(288)[1] for _ in range(4)]
        assert sorted(g for _, g in filter(None, placed)) == [0, 1, 3] and placed.count(None) == 1
        mgr.smi.inject("replug 2")
        assert wait(lambda: health_by_gpu(kl, model)[2] == const.HEALTHY)
        assert model.count() == 4 and model.gpus[2].index == 2   # index stable across unplug


def test_reset_marks_unhealthy_then_recovers():
    with SimCluster([("n", "fake:2x4G")], health_poll_s=0.2) as c:
        mgr, kl = c.manager("n"), c.nodes["n"].kubelet
        seen = []
        orig = mgr.health.handle_event

        def spy(ev):
            seen.append(ev.name)
            orig(ev)
        mgr.health.handle_event = spy
        mgr.smi.inject("reset 1")
        assert wait(lambda: "post_reset" in seen)
        assert wait(lambda: health_by_gpu(kl, mgr.model)[1] == const.HEALTHY)
        assert kl.list_updates >= 3     # initial + unhealthy + healthy again


def test_ecc_uncorrectable_marks_unhealthy_until_reset():
    with SimCluster([("n", "fake:2x4G")], health_poll_s=0.2) as c:
        mgr, kl = c.manager("n"), c.nodes["n"].kubelet
        mgr.smi.inject("ecc 0 2")
        assert wait(lambda: health_by_gpu(kl, mgr.model)[0] == const.UNHEALTHY)
        mgr.smi.inject("reset 0")
        assert wait(lambda: health_by_gpu(kl, mgr.model)[0] == const.HEALTHY)


def test_vmfault_is_ignored():
    with SimCluster([("n", "fake:1x4G")], health_poll_s=0.2) as c:
        mgr, kl = c.manager("n"), c.nodes["n"].kubelet
        mgr.smi.inject("vmfault 0")
        assert wait(lambda: mgr.health.ignored >= 1)
        assert health_by_gpu(kl, mgr.model)[0] == const.HEALTHY


def test_topology_exported_and_tp_pair_placement_reconciles():
    with SimCluster([("n", "fake:8x288G")], health_poll_s=0.2) as c:
        mgr = c.manager("n")
        topo = nodestatus.read_topology(c.client.get_node("n"))
        assert topo and len(topo["link_type"]) == 8
        assert topo["link_type"][0][1] == "xgmi" and topo["hops"][0][1] == 1
        # fill GPUs 0..5 so a TP pair must use 6 and 7, then break the 6<->7 link
        for _ in range(6):
            c.run_pod(288)
        mgr.smi.inject("linkdown 6 7")
        assert wait(lambda: nodestatus.read_topology(c.client.get_node("n"))["link_type"][6][7] == "pcie")
        c.extender.sync()
        pods, placed, adms = c.run_tp_group("g1", 2, 64)
        assert placed is None                      # only 6,7 have room and they are not xGMI peers
        for p in pods:
            c.client.delete_pod("default", O.name(p))
        mgr.smi.inject("linkup 6 7")
        assert wait(lambda: nodestatus.read_topology(c.client.get_node("n"))["link_type"][6][7] == "xgmi")
        c.extender.sync()
        pods, placed, adms = c.run_tp_group("g2", 2, 64)
        assert sorted(g for _, g in placed) == [6, 7]
        assert all(a.error is None for a in adms)


def test_best_group_prefers_connected_and_tight():
    topo = {"link_type": [["self", "xgmi", "pcie"], ["xgmi", "self", "xgmi"], ["pcie", "xgmi", "self"]],
            "hops": [[0, 1, 3], [1, 0, 1], [3, 1, 0]]}
    assert T.best_group(topo, [100, 100, 100], 2, 50) in ([0, 1], [1, 2])
    assert T.best_group(topo, [60, 200, 100], 2, 50) == [0, 1]      # best fit among connected
    assert T.best_group(topo, [100, 0, 100], 2, 50) is None          # 0-2 only over PCIe
    assert T.best_group(None, [100, 0, 100], 2, 50) == [0, 2]        # no topology: capacity only


def test_hbm_used_gauge_follows_smi():
    """SURVEY §5.5 "SMI HBM used per GPU": gpushare_hbm_used_bytes{gpu} is set from the health
    poll (round-2 review: the gauge was declared but never set)."""
    with SimCluster([("n", "fake:2x8G")], health_poll_s=0.1) as c:
        mgr = c.manager("n")
        m = mgr.metrics.hbm_used
        assert m.value(gpu="0") == 0 and m.value(gpu="1") == 0
        mgr.smi.inject("vram 1 3072")
        assert wait(lambda: m.value(gpu="1") == 3 << 30)
        assert m.value(gpu="0") == 0
        assert 'gpushare_hbm_used_bytes{gpu="1"} 3221225472' in mgr.metrics.registry.render()


def test_unarmed_events_make_the_plugin_not_ready():
    """Round-2 review item 3: when SMI event notification is not armed on every GPU (the
    container cannot open /dev/kfd) the plugin logs at error level, sets
    gpushare_health_degraded and /readyz answers 503 with the reason."""
    import urllib.error
    import urllib.request

    from aliyun_gpushare_device_plugin_amd.utils import metrics as M

    with SimCluster([("n", "fake:2x8G")], health_poll_s=0.5) as c:
        mgr = c.manager("n")
        assert mgr.readiness() == (True, "ok") and mgr.metrics.health_degraded.value() == 0
        orig = mgr.smi.health_status
        mgr.smi.health_status = lambda: dict(orig(), events_armed=0, events_last_status=13)
        mgr._start_health()
        ok, why = mgr.readiness()
        assert not ok and "armed on 0/2" in why and mgr.metrics.health_degraded.value() == 1
        srv = M.serve(mgr.metrics.registry, "127.0.0.1:0", ready_fn=mgr.readiness)
        try:
            port = srv.server_address[1]
            try:
                urllib.request.urlopen(f"http://127.0.0.1:{port}/readyz", timeout=5)
                raise AssertionError("expected 503")
            except urllib.error.HTTPError as e:
                assert e.code == 503 and b"armed on 0/2" in e.read()
        finally:
            srv.shutdown()


def test_lost_post_reset_recovers_by_polling():
    """Round-3 review item 5: a pre-reset whose post-reset event never arrives used to strand
    the GPU Unhealthy. The poll returns it to Healthy once it answers SMI on settle_polls (2)
    consecutive polls, and ListAndWatch re-sends both transitions."""
    with SimCluster([("n", "fake:2x4G")], health_poll_s=0.2) as c:
        mgr, kl = c.manager("n"), c.nodes["n"].kubelet
        sends = kl.list_updates
        mgr.smi.inject("prereset 1")
        assert wait(lambda: health_by_gpu(kl, mgr.model)[1] == const.UNHEALTHY)
        t0 = time.time()
        assert wait(lambda: health_by_gpu(kl, mgr.model)[1] == const.HEALTHY, timeout=5.0)
        assert time.time() - t0 <= 3 * 0.2 + 0.5        # within settle_polls (+1) poll intervals
        assert "post-reset event not seen" in mgr.model.gpu(1).reason
        assert kl.list_updates >= sends + 2
        assert health_by_gpu(kl, mgr.model)[0] == const.HEALTHY


def test_ecc_mark_clears_on_a_silent_reset():
    """An ECC uncorrectable-error mark followed by a reset that emits no event at all: the UE
    counters going backwards is the observed reset; the GPU returns and a later UE marks it again."""
    with SimCluster([("n", "fake:2x4G")], health_poll_s=0.2) as c:
        mgr, kl = c.manager("n"), c.nodes["n"].kubelet
        mgr.smi.inject("ecc 0 2")
        assert wait(lambda: health_by_gpu(kl, mgr.model)[0] == const.UNHEALTHY)
        time.sleep(0.5)                                 # stays marked across polls
        assert health_by_gpu(kl, mgr.model)[0] == const.UNHEALTHY
        mgr.smi.inject("silentreset 0")
        assert wait(lambda: health_by_gpu(kl, mgr.model)[0] == const.HEALTHY, timeout=3.0)
        assert "reset observed" in mgr.model.gpu(0).reason
        mgr.smi.inject("ecc 0 1")                       # a new UE after the reset marks it again
        assert wait(lambda: health_by_gpu(kl, mgr.model)[0] == const.UNHEALTHY)


def test_ecc_mark_clears_on_a_pre_reset_without_post_reset():
    with SimCluster([("n", "fake:2x4G")], health_poll_s=0.2) as c:
        mgr, kl = c.manager("n"), c.nodes["n"].kubelet
        mgr.smi.inject("ecc 1 3")
        assert wait(lambda: health_by_gpu(kl, mgr.model)[1] == const.UNHEALTHY)
        mgr.smi.inject("prereset 1")                   # the UE counter is NOT cleared here
        assert wait(lambda: "reset in progress" in mgr.model.gpu(1).reason)
        assert wait(lambda: health_by_gpu(kl, mgr.model)[1] == const.HEALTHY, timeout=3.0)
        time.sleep(0.6)                                 # re-baselined: the old UEs do not re-mark it
        assert health_by_gpu(kl, mgr.model)[1] == const.HEALTHY


def test_a_gpu_enumerated_but_still_resetting_stays_unhealthy():
    """an MI355X stays enumerated during a mode-1 reset, so presence alone must
    not end a reset mark. Fake SMI "resetting 1 5": a pre-reset, then the GPU is listed but fails
    the functional probe (amdgpu gpu_metrics) on its next 5 probes — it stays Unhealthy through
    them, and recovers only after settle_polls (2) working polls."""
    with SimCluster([("n", "fake:2x4G")], health_poll_s=0.2) as c:
        mgr, kl = c.manager("n"), c.nodes["n"].kubelet
        mgr.smi.inject("resetting 1 5")
        assert wait(lambda: health_by_gpu(kl, mgr.model)[1] == const.UNHEALTHY)
        time.sleep(0.2 * 4)                              # 4 polls: listed every time, probe failing
        assert health_by_gpu(kl, mgr.model)[1] == const.UNHEALTHY
        assert "not answering the functional probe" in mgr.model.gpu(1).reason
        assert wait(lambda: health_by_gpu(kl, mgr.model)[1] == const.HEALTHY, timeout=6.0)
        assert "working on 2 polls" in mgr.model.gpu(1).reason
        assert health_by_gpu(kl, mgr.model)[0] == const.HEALTHY


def test_a_post_reset_event_before_the_gpu_works_waits_for_the_probe():
    from aliyun_gpushare_device_plugin_amd.device import smi as S

    with SimCluster([("n", "fake:2x4G")], health_poll_s=0.2) as c:
        mgr, kl = c.manager("n"), c.nodes["n"].kubelet
        mgr.smi.inject("resetting 0 3")
        assert wait(lambda: health_by_gpu(kl, mgr.model)[0] == const.UNHEALTHY)
        mgr.health.handle_event(S.Event(0, S.EV_POST_RESET, "GPU post-reset"))   # early: probe still failing
        assert mgr.model.gpu(0).healthy is False or "reset" in mgr.model.gpu(0).reason
        assert wait(lambda: health_by_gpu(kl, mgr.model)[0] == const.HEALTHY, timeout=6.0)


def test_probe_on_real_backends_reads_gpu_metrics(tmp_path):
    """The functional probe on a sysfs tree: gpu_metrics readable with a header = working; the file
    there but unreadable = not working; no file = unknown (presence decides, as before)."""
    import ctypes

    from aliyun_gpushare_device_plugin_amd.device import smi as S

    lib = S._load()
    root = tmp_path / "root"
    node = root / "sys/class/kfd/kfd/topology/nodes/1"
    node.mkdir(parents=True)
    (node / "gpu_id").write_text("4242\n")
    (node / "properties").write_text("simd_count 1024\narray_count 32\nlocal_mem_size 0\ndrm_render_minor 128\n"
                                     "gfx_target_version 90500\nunique_id 77\nnum_xcc 8\ndomain 0\nlocation_id 1280\n")
    dev = root / "sys/class/drm/renderD128/device"
    dev.mkdir(parents=True)
    (dev / "mem_info_vram_total").write_text(str(288 << 30))
    with S.SMI(f"sysfs:{root}") as s:
        assert s.count() == 1
        assert s.probe(0) is None                                       # no gpu_metrics: unknown
        (dev / "gpu_metrics").write_bytes(bytes([0x80, 0x00, 1, 8]) + bytes(124))
        assert s.probe(0) is True
        (dev / "gpu_metrics").write_bytes(b"")                         # the driver refused the read
        assert s.probe(0) is False
    assert ctypes is not None
