"""End-to-end on CPU: fake apiserver + fake kubelet (gRPC/UDS) + real plugin + extender."""
import os
import signal
import time

import pytest

from aliyun_gpushare_device_plugin_amd import const
from aliyun_gpushare_device_plugin_amd.api import v1beta1 as api
from aliyun_gpushare_device_plugin_amd.cluster import objects as O
from aliyun_gpushare_device_plugin_amd.sim.cluster import SimCluster


def envs(adm, i=0):
    return dict(adm.responses[i].envs)


def test_config1_stub_plugin_roundtrip():
    """BASELINE config 1: 2 fake GPUs x 4 GiB, ListAndWatch/Allocate round trip."""
    with SimCluster([("node-a", "fake:2x4G")], preferred_allocation=True) as c:
        node = c.client.get_node("node-a")
        assert node["status"]["allocatable"][const.RESOURCE_COUNT] == "2"
        assert node["status"]["allocatable"][const.RESOURCE_NAME] == "8"
        kl = c.nodes["node-a"].kubelet
        assert kl.registrations[0] == ("v1beta1", "aliyungpushare.sock", const.RESOURCE_NAME)
        assert len(kl.devices) == 8 and set(kl.devices.values()) == {const.HEALTHY}
        assert kl.options.get_preferred_allocation_available
        gpus = []
        for _ in range(4):
            pod, where, adm = c.run_pod(2)
            assert adm.error is None and envs(adm)[const.ENV_RESOURCE_BY_DEV] == "4"
            gpus.append(int(envs(adm)[const.ENV_RESOURCE_INDEX]))
            got = c.wait_assigned(pod)
            assert O.annotations(got)[const.ENV_ASSIGNED_FLAG] == "true"
            assert O.phase(got) == "Running"
        assert sorted(gpus) == [0, 0, 1, 1]
        # preferred allocation: kubelet's chosen fake IDs belong to the GPU actually used
        assert {d.split("-_-")[0] for d in adm.device_ids[0]} == {c.manager("node-a").model.uuid_by_index(gpus[-1])}
        _, where, _ = c.run_pod(1)
        assert where is None      # node full (8 of 8 GiB)


def test_config3_eight_mi355x_mixed_pods():
    """BASELINE config 3: 8 x MI355X node, 32 mixed 8-128 GiB pods via the extender."""
    sizes = [128, 64, 64, 32, 96, 96, 64, 32, 128, 96, 56, 8, 64, 64, 96, 64] * 2
    with SimCluster([("big", "fake:8x309220868096B")]) as c:
        assert O.node_allocatable(c.client.get_node("big"), const.RESOURCE_NAME) == 8 * 288
        placed, lat = 0, []
        for s in sorted(sizes, reverse=True):
            pod, where, adm = c.run_pod(s)
            if where is not None:
                assert adm.error is None
                placed += 1
                lat += adm.latencies
        usage = c.extender.usage()["big"]
        assert all(u <= 288 for u in usage["used"])      # never over-committed
        assert placed >= 31 and sum(usage["used"]) >= 0.97 * 8 * 288
        assert sorted(lat)[len(lat) // 2] < 0.05


def test_delete_frees_capacity_and_reuse():
    with SimCluster([("n", "fake:1x8G")]) as c:
        p1, _, a1 = c.run_pod(6)
        _, w, _ = c.run_pod(4)
        assert w is None
        c.delete_pod(p1)
        _, w, a = c.run_pod(4)
        assert w == ("n", 0) and a.error is None


def test_kubelet_restart_triggers_reregistration():
    with SimCluster([("n", "fake:1x4G")]) as c:
        kl = c.nodes["n"].kubelet
        mgr = c.manager("n")
        kl.restart()                      # re-creates kubelet.sock like a kubelet restart
        assert kl.registered.wait(15)
        t = time.time() + 10
        while mgr.restarts < 1 and time.time() < t:
            time.sleep(0.05)
        assert mgr.restarts >= 1 and len(kl.registrations) == 2
        _, w, adm = c.run_pod(2)
        assert adm.error is None


def test_sighup_restarts_plugin():
    with SimCluster([("n", "fake:1x4G")]) as c:
        mgr = c.manager("n")
        mgr.events.put(("signal", signal.SIGHUP))
        t = time.time() + 10
        while mgr.restarts < 1 and time.time() < t:
            time.sleep(0.05)
        assert mgr.restarts == 1
        assert c.nodes["n"].kubelet.registered.wait(10)


@pytest.mark.parametrize("source,mode", [("watch", "thread"), ("list", "thread"), ("kubelet", "thread"),
                                         ("kubelet", "process")])
def test_pod_sources(source, mode):
    """Candidates from the informer, a per-Allocate LIST, or the kubelet's /pods (bearer token,
    --kubelet-scheme http against the fake kubelet; through the CLI in process mode)."""
    with SimCluster([("n", "fake:2x4G")], pod_source=source, plugin_mode=mode) as c:
        gpus = []
        for _ in range(3):
            _, w, adm = c.run_pod(2)
            assert adm.error is None and envs(adm)[const.ENV_RESOURCE_INDEX] != "-1"
            gpus.append(envs(adm)[const.ENV_RESOURCE_INDEX])
        assert sorted(gpus) in (["0", "0", "1"], ["0", "1", "1"])


def test_stack_dump_on_sigquit(tmp_path, monkeypatch):
    """SIGQUIT writes every thread's stack to GPUSHARE_DUMP_DIR (coredump.go:10-30)."""
    monkeypatch.setenv("GPUSHARE_DUMP_DIR", str(tmp_path))
    with SimCluster([("n", "fake:1x4G")]) as c:
        c.manager("n").events.put(("signal", signal.SIGQUIT))
        t = time.time() + 10
        while not list(tmp_path.glob("gpushare_*.txt")) and time.time() < t:
            time.sleep(0.05)
        dumps = list(tmp_path.glob("gpushare_*.txt"))
        assert dumps and "plugin-n" in dumps[0].read_text()       # the manager thread's stack
        _, _, adm = c.run_pod(2)                                    # and the plugin keeps serving
        assert adm.error is None


def test_watch_cache_used_instead_of_list():
    with SimCluster([("n", "fake:2x4G")], pod_source="watch") as c:
        store = c.api.store
        before = store.requests["GET pods"]
        for _ in range(4):
            c.run_pod(1)
        # no per-Allocate LIST: the informer serves candidates. An Allocate that races the bind
        # event (the kubelet can see the bind before the plugin's watch does) falls back to one
        # fresh LIST by design, so a loaded CI host may show an occasional one — never one each.
        assert store.requests["GET pods"] - before < 4


def test_plugin_as_separate_process():
    with SimCluster([("n", "fake:2x4G")], plugin_mode="process", preferred_allocation=True) as c:
        _, w, adm = c.run_pod(3)
        assert adm.error is None and envs(adm)[const.ENV_RESOURCE_BY_CONTAINER] == "3"
        assert c.nodes["n"].kubelet.options.get_preferred_allocation_available


def test_kubelet_as_separate_process():
    """Every component in its own interpreter (the bench's layout): apiserver, kubelet, plugin."""
    with SimCluster([("n", "fake:2x4G")], plugin_mode="process", apiserver="process", kubelet="process",
                    preferred_allocation=True) as c:
        kl = c.nodes["n"].kubelet
        assert kl.options.get_preferred_allocation_available and kl.registered.is_set()
        pod, w, adm = c.run_pod(3)
        assert adm.error is None and envs(adm)[const.ENV_RESOURCE_BY_CONTAINER] == "3"
        assert len(adm.latencies) == 1 and adm.latencies[0] > 0
        assert len(kl.allocated_ids()) == 3
        c.delete_pod(pod)
        assert kl.allocated_ids() == set()
        c.kill_plugin("n")
        c.restart_plugin("n")                    # registered.clear() + wait through the pipe
        _, _, adm = c.run_pod(4)
        assert adm.error is None


def test_preferred_allocation_is_opt_in():
    with SimCluster([("n", "fake:1x4G")]) as c:
        assert not c.nodes["n"].kubelet.options.get_preferred_allocation_available
        _, _, adm = c.run_pod(2)
        assert adm.error is None


def test_multi_node_cluster():
    with SimCluster([("a", "fake:1x4G"), ("b", "fake:1x4G")]) as c:
        nodes = set()
        for _ in range(4):
            pod, where, adm = c.run_pod(2)
            assert adm.error is None
            nodes.add(where[0])
        assert nodes == {"a", "b"}


def test_cgpu_label_sets_env():
    with SimCluster([("n", "fake:1x4G")]) as c:
        c.client.patch_node("n", {"metadata": {"labels": {const.NODE_LABEL_DISABLE_CGPU: "true"}}})
        c.manager("n").events.put(("signal", signal.SIGHUP))
        time.sleep(0.5)
        assert c.nodes["n"].kubelet.registered.wait(10)
        t = time.time() + 10
        while c.manager("n").restarts < 1 and time.time() < t:
            time.sleep(0.05)
        time.sleep(0.3)
        _, _, adm = c.run_pod(2)
        assert envs(adm)[const.ENV_CGPU_DISABLE] == "true"


def test_shim_injected_end_to_end(native_shim):
    shim_dir = os.path.dirname(native_shim)
    with SimCluster([("n", "fake:1x4G")], shim_host_dir=shim_dir) as c:
        _, _, adm = c.run_pod(2)
        r = adm.responses[0]
        assert r.envs[const.ENV_LD_PRELOAD].endswith(const.SHIM_LIB_NAME)
        assert r.mounts[0].host_path == shim_dir


def test_children_arm_their_lifeline_after_exec():
    """The simulator's children set PR_SET_PDEATHSIG from the package import (no preexec_fn between
    fork and exec of the threaded parent): the variable is consumed so grandchildren do not inherit
    it, and a child whose parent is not the one named exits at once."""
    import subprocess
    import sys

    code = ("import os, aliyun_gpushare_device_plugin_amd; "
            "print(os.environ.get('GPUSHARE_DIE_WITH_PARENT', 'consumed'))")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, GPUSHARE_DIE_WITH_PARENT=str(os.getpid()), PYTHONPATH=root)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and r.stdout.strip() == "consumed"
    env["GPUSHARE_DIE_WITH_PARENT"] = "1"                     # not our parent: the child leaves quietly
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and r.stdout == ""


def test_an_in_process_plugin_gets_the_extra_plugin_flags(tmp_path):
    """The simulator's thread-mode plugin runs with the same flags a process-mode one is started
    with: a tool passing ``--hbm-broker-dir`` (tools/bench_colocate.py) gets a plugin that grants
    HBM, not one that silently ignores the flag."""
    hdir = tmp_path / "hbm"
    with SimCluster([("n", "fake:1x288G")], extra_plugin_args=["--hbm-broker-dir", str(hdir)],
                    shim_host_dir=str(tmp_path / "shim")) as c:
        m = c.manager("n")
        assert m.cfg.hbm_broker_dir == str(hdir) and m.allocator._hbm is not None
        _, where, adm = c.run_pod(16)
        assert adm.error is None
        assert adm.responses[0].envs[const.ENV_HBM_BROKER].endswith("hbm0.sock")
