"""The shipped manifests, run as a node would run them (sim/deploy.py): the DaemonSet's container
and the scheduler extender's Deployment start from their own commands, env and hostPath volumes;
kube-scheduler's side follows the extender ConfigMap; the reference's bin-pack demo
(deploy/demo/binpack-1) is scheduled and admitted; the probes the manifests declare answer; and
``kubectl-inspect-gpushare`` reports the result. Overrides (no GPU, no cluster) are listed in the
module docstring of sim/deploy.py and asserted below to be nothing else."""
import os
import shutil
import stat
import subprocess
import sys
import tempfile

import pytest

from aliyun_gpushare_device_plugin_amd import const
from aliyun_gpushare_device_plugin_amd.cluster import objects as O
from aliyun_gpushare_device_plugin_amd.cluster.client import APIClient, KubeConfig
from aliyun_gpushare_device_plugin_amd.sim import deploy as D
from aliyun_gpushare_device_plugin_amd.sim.apiserver import FakeAPIServer, make_node
from aliyun_gpushare_device_plugin_amd.sim.kubelet import FakeKubelet

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NODE = "mi355x-0"


@pytest.fixture
def hostroot():
    d = tempfile.mkdtemp(prefix="gsd-", dir="/tmp")       # short: unix socket paths are limited
    yield d
    shutil.rmtree(d, ignore_errors=True)


def _stop(p):
    if p is not None and p.poll() is None:
        p.terminate()
        try:
            p.wait(timeout=10)
        except subprocess.TimeoutExpired:
            p.kill()


def test_shipped_manifests_run_a_node(hostroot, stub_runtime, native_shim):
    api = FakeAPIServer()
    api.start()
    client = APIClient(KubeConfig(api.url))
    client.create_node(make_node(NODE))
    plugin = ext = brokers = None
    kubelet = FakeKubelet(os.path.join(hostroot, "device-plugin"), APIClient(KubeConfig(api.url)), NODE).start()
    try:
        # ---- the DaemonSet, as the kubelet would start it on NODE
        ds = next(d for d in D.load(os.path.join(ROOT, "deploy", "device-plugin-ds.yaml")) if d["kind"] == "DaemonSet")
        assert ds["spec"]["template"]["spec"]["nodeSelector"] == {"gpushare": "true"}
        assert make_node(NODE)["metadata"]["labels"]["gpushare"] == "true"
        mport = D.free_port()
        overrides = {"--smi-backend": "fake:2x288G", "--metrics-addr": f"127.0.0.1:{mport}", "--apiserver": api.url}
        # the init container first, to completion: it fills the comgr cache (no GPU here: nothing
        # to warm) and seals it read-only where the plugin's flag names it
        ict = D.resolve(ds, hostroot, {"spec.nodeName": NODE}, {}, container="comgr-cache")
        init = D.start(ict, os.path.join(hostroot, "comgr-cache.log"))
        assert init.wait(300) == 0, open(os.path.join(hostroot, "comgr-cache.log")).read()[-3000:]
        cache = ict.host_path("/var/lib/gpushare/comgr-cache")
        assert os.path.isdir(cache) and stat.S_IMODE(os.stat(cache).st_mode) == 0o555
        ct = D.resolve(ds, hostroot, {"spec.nodeName": NODE}, overrides, skip_volumes=("sys",))
        assert f"--comgr-cache-dir={cache}" in ct.argv          # the same hostPath as the init container's
        # the kubelet socket directory is the binary's default (not written in the manifest): the
        # container sees it at that path through the device-plugin mount
        ct.argv.append("--device-plugin-dir=" + ct.host_path(const.DEVICE_PLUGIN_PATH))
        # the pod-resources socket the manifest names is the kubelet's (hostPath mount)
        podres = ct.host_path("/var/lib/kubelet/pod-resources/kubelet.sock")
        os.symlink(kubelet.podres_sock, podres)
        assert ct.host_path("/var/lib/kubelet/device-plugins") == kubelet.dir
        assert ct.env["NODE_NAME"] == NODE
        plugin = D.start(ct, os.path.join(hostroot, "plugin.log"))
        # the DaemonSet's second container: one HBM broker per GPU (no GPU here: the brokers are the
        # stub runtime's, over the same fake node the plugin sees)
        bct = D.resolve(ds, hostroot, {"spec.nodeName": NODE}, {"--smi-backend": "fake:2x288G"}, skip_volumes=("sys",),
                        container="hbm-brokers")
        assert bct.host_path("/var/run/gpushare/hbm") == ct.host_path("/var/run/gpushare/hbm")   # one hostPath
        bct.env.update(GPUSHARE_HBM_BROKER_EXE=os.path.join(stub_runtime, "gpushare-hbm-broker"),
                       LD_LIBRARY_PATH=stub_runtime, FAKE_HIP_TOTAL_GIB="288")
        brokers = D.start(bct, os.path.join(hostroot, "brokers.log"))
        assert kubelet.registered.wait(60), open(os.path.join(hostroot, "plugin.log")).read()[-3000:]
        assert D.wait_for(lambda: O.node_allocatable(client.get_node(NODE), const.RESOURCE_NAME) == 576, 30)
        # the probes the manifest declares (port remapped from 9400)
        probes = ds["spec"]["template"]["spec"]["containers"][0]
        for probe in ("livenessProbe", "readinessProbe"):
            path = probes[probe]["httpGet"]["path"]
            assert D.wait_for(lambda: D.http_get(f"http://127.0.0.1:{mport}{path}")[0] == 200, 20), path
        # --install-shim put the quota shim into the gpushare-lib hostPath
        shim = ct.host_path(os.path.join("/var/lib/gpushare/lib", const.SHIM_LIB_NAME))
        assert os.path.isfile(shim)

        # ---- the scheduler extender Deployment and kube-scheduler's config for it
        docs = D.load(os.path.join(ROOT, "deploy", "scheduler-extender.yaml"))
        dep = next(d for d in docs if d["kind"] == "Deployment")
        ect = D.resolve(dep, hostroot, {"metadata.name": "gpushare-scheduler-extender-0"},
                        {"--apiserver": api.url, "--port": "0", "--host": "127.0.0.1", "--resync": "0.5"})
        assert "--leader-elect" in ect.argv and ect.env["POD_NAME"] == "gpushare-scheduler-extender-0"
        ext = D.start(ect, os.path.join(hostroot, "extender.log"))
        eport = int(ext.stdout.readline().split()[1])
        # the Service routes kube-scheduler to a ready replica: the Lease holder
        assert D.wait_for(lambda: D.http_get(f"http://127.0.0.1:{eport}/readyz")[0] == 200, 10.0)
        lease = api.store.leases[("kube-system", "gpushare-scheduler-extender")]
        assert lease["spec"]["holderIdentity"].startswith("gpushare-scheduler-extender-0_")
        cm = next(d for d in docs if d["kind"] == "ConfigMap")
        sched = D.Scheduler(cm["data"]["scheduler-config.yaml"], f"127.0.0.1:{eport}")
        assert sched.managed == [const.RESOURCE_NAME]

        # ---- the reference's bin-pack demo: StatefulSet (3 replicas) + Job, 2 GiB each
        demo = D.load(os.path.join(ROOT, "deploy", "demo", "binpack-1", "binpack-1.yaml")) + \
            D.load(os.path.join(ROOT, "deploy", "demo", "binpack-1", "job.yaml"))
        pods = []
        for d in demo:
            if d["kind"] not in ("StatefulSet", "Job"):
                continue
            tpl = D.pod_template(d)
            for i in range(d["spec"].get("replicas", 1)):
                pod = {"apiVersion": "v1", "kind": "Pod",
                       "metadata": {"name": f"{d['metadata']['name']}-{i}", "namespace": "default",
                                    "labels": dict(tpl.get("metadata", {}).get("labels", {}))},
                       "spec": {**tpl["spec"], "schedulerName": "default-scheduler"}}
                pods.append(client.create_pod("default", pod))
        assert len(pods) == 4
        for pod in pods:
            placed = []                                        # the extender's informer catches up
            assert D.wait_for(lambda: placed.append(sched.schedule(pod, [NODE])) or placed[-1] == NODE, 10, 0.1), \
                O.name(pod)
            bound = client.get_pod("default", O.name(pod))
            adm = kubelet.admit(bound)
            assert adm.error is None, adm.error
            envs = adm.responses[0].envs
            assert envs[const.ENV_RESOURCE_INDEX] == O.annotations(bound)[const.ENV_RESOURCE_INDEX]
            assert int(envs["ALIYUN_COM_GPU_MEM_CONTAINER"]) == 2
            # the shim the DaemonSet installed is what the container gets mounted and preloaded
            mounts = {m.container_path: m.host_path for m in adm.responses[0].mounts}
            assert any(h.startswith(ct.host_path("/var/lib/gpushare/lib")) for h in mounts.values()), mounts
            assert "LD_PRELOAD" in envs
        # best fit packs all four 2 GiB pods onto one GPU
        gpus = {O.annotations(client.get_pod("default", O.name(p)))[const.ENV_RESOURCE_INDEX] for p in pods}
        assert len(gpus) == 1

        # ---- a 64 GiB pod (deploy/demo/llama-colocate.yaml) takes its HBM from its GPU's broker
        from aliyun_gpushare_device_plugin_amd.quota import hbmbroker as hb

        hdir = ct.host_path("/var/run/gpushare/hbm")
        dep = next(d for d in D.load(os.path.join(ROOT, "deploy", "demo", "llama-colocate.yaml")) if d["kind"] == "Deployment")
        tpl = D.pod_template(dep)
        big = client.create_pod("default", {"apiVersion": "v1", "kind": "Pod",
                                            "metadata": {"name": "llama-0", "namespace": "default"},
                                            "spec": {**tpl["spec"], "schedulerName": "default-scheduler"}})
        placed = []
        assert D.wait_for(lambda: placed.append(sched.schedule(big, [NODE])) or placed[-1] == NODE, 10, 0.1)
        adm = kubelet.admit(client.get_pod("default", "llama-0"))
        assert adm.error is None, adm.error
        r = adm.responses[0]
        gi = int(r.envs[const.ENV_RESOURCE_INDEX])
        tok = r.envs[const.ENV_HBM_TOKEN]
        mounts = {m.container_path: m for m in r.mounts}
        assert mounts[const.HBM_BROKER_CONTAINER_DIR].host_path == hb.pod_dir(hdir, gi)   # its GPU's sockets only
        assert mounts[const.HBM_BROKER_CONTAINER_DIR].read_only
        assert not any(m.host_path.startswith(hb.admin_dir(hdir)) for m in r.mounts)
        # the init container's comgr cache, read-only, with comgr pointed at it
        assert mounts[const.COMGR_CACHE_CONTAINER_DIR].host_path == cache and mounts[const.COMGR_CACHE_CONTAINER_DIR].read_only
        assert r.envs[const.ENV_COMGR_CACHE_DIR] == const.COMGR_CACHE_CONTAINER_DIR and r.envs[const.ENV_COMGR_CACHE] == "1"
        st = {}
        assert D.wait_for(lambda: st.update(hb.HBMBroker.attach(hb.pod_socket(hdir, gi), hb.admin_socket(hdir, gi))
                                            .list()) or tok in st.get("grants", {}), 30, 0.2), \
            open(os.path.join(hostroot, "brokers.log")).read()[-3000:]
        # the container's process: the answer's env with its mounts resolved to host paths
        env = dict(r.envs)

        def host(v):
            for cpath, m in sorted(mounts.items(), key=lambda x: -len(x[0])):
                if v == cpath or v.startswith(cpath.rstrip("/") + "/"):
                    return m.host_path + v[len(cpath.rstrip("/")):]
            return v
        for k, v in list(env.items()):
            env[k] = ":".join(host(x) for x in v.split(":")) if k == "LD_PRELOAD" else host(v)
        # the shim, then the comgr action cache the plugin installed next to it (with the cache mounted)
        pre = env["LD_PRELOAD"].split(":")
        assert [os.path.basename(x) for x in pre] == [const.SHIM_LIB_NAME, const.COMGR_ACTION_LIB_NAME]
        assert all(os.path.isfile(x) for x in pre)
        assert env[const.ENV_COMGR_ACTION_CACHE] == cache
        env.update(LD_LIBRARY_PATH=stub_runtime, FAKE_HIP_TOTAL_GIB="288")
        p = subprocess.run([os.path.join(stub_runtime, "shim_driver"), "alloc", str(32 << 30), "arena"],
                           env=dict(os.environ, **env), capture_output=True, text=True, timeout=60)
        out = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
        assert '"op":"arena","on":1,"size":64424509440' in out[-1], (out, p.stderr[-2000:])   # 60 GiB: 94 % of 64

        # ---- kubectl-inspect-gpushare against the same apiserver
        r = subprocess.run([sys.executable, "-m", D.ENTRY_POINTS["kubectl-inspect-gpushare"], "--apiserver", api.url],
                           capture_output=True, text=True, timeout=60,
                           env=dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", "")))
        assert r.returncode == 0, r.stdout + r.stderr
        assert NODE in r.stdout and "72/576" in r.stdout.replace(" ", ""), r.stdout   # 4 x 2 + 64 GiB

        # ---- the node is labelled cgpu.disable.isolation=true while running. The
        # brokers (--start-empty: sized by the plugin) give their HBM back to the driver, answers carry
        # CGPU_DISABLE and no shim; the label removed, the brokers take the GPU again
        adm_b = hb.HBMBroker.attach(hb.pod_socket(hdir, gi), hb.admin_socket(hdir, gi))
        assert adm_b.stat()["target"] == adm_b.stat()["granules_max"] == 276        # 288 less the 12 GiB reserve
        client.patch_node(NODE, {"metadata": {"labels": {const.NODE_LABEL_DISABLE_CGPU: "true"}}})
        assert D.wait_for(lambda: adm_b.stat()["target"] == 0 and adm_b.stat()["granules"] == 0, 40, 0.2), adm_b.stat()
        assert adm_b.list()["grants"] == {}                                          # every grant revoked
        off = client.create_pod("default", {"apiVersion": "v1", "kind": "Pod",
                                            "metadata": {"name": "llama-1", "namespace": "default"},
                                            "spec": {**tpl["spec"], "schedulerName": "default-scheduler"}})
        placed = []
        assert D.wait_for(lambda: placed.append(sched.schedule(off, [NODE])) or placed[-1] == NODE, 10, 0.1)
        adm = kubelet.admit(client.get_pod("default", "llama-1"))
        assert adm.error is None, adm.error
        envs = adm.responses[0].envs
        assert envs[const.ENV_CGPU_DISABLE] == "true" and "LD_PRELOAD" not in envs and const.ENV_HBM_TOKEN not in envs
        client.patch_node(NODE, {"metadata": {"labels": {const.NODE_LABEL_DISABLE_CGPU: None}}})
        assert D.wait_for(lambda: adm_b.stat()["target"] == 276 and adm_b.stat()["granules"] == 276, 40, 0.2), \
            adm_b.stat()
    finally:
        _stop(ext)
        _stop(brokers)
        _stop(plugin)
        kubelet.stop()
        api.stop()


def test_rehearsal_overrides_are_only_the_documented_ones():
    """Nothing but the SMI backend, the apiserver and the listening address/port differs from the
    manifests: every other flag reaches the process as written (paths remapped)."""
    ds = next(d for d in D.load(os.path.join(ROOT, "deploy", "device-plugin-ds.yaml")) if d["kind"] == "DaemonSet")
    root = tempfile.mkdtemp(prefix="gsd-", dir="/tmp")
    try:
        ct = D.resolve(ds, root, {"spec.nodeName": NODE},
                       {"--smi-backend": "fake:2x288G", "--metrics-addr": "127.0.0.1:1", "--apiserver": "http://x"},
                       skip_volumes=("sys",))
        cmd = ds["spec"]["template"]["spec"]["containers"][0]["command"]
        want = [D._rewrite(a, ct.mounts) for a in cmd[1:]
                if a.partition("=")[0] not in ("--smi-backend", "--metrics-addr")]
        got = ct.argv[3:]
        assert [a for a in got if a.partition("=")[0] not in ("--smi-backend", "--metrics-addr", "--apiserver")] == want
        assert all(not a.startswith("/var/lib/gpushare") for a in got)   # every hostPath remapped
    finally:
        shutil.rmtree(root, ignore_errors=True)
