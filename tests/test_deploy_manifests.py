"""Deployment manifests stay in step with the code: every YAML parses, the DaemonSet's flags are
accepted by the plugin's CLI, and demo pods use the resource / annotation names the plugin reads."""
import glob
import os

import yaml

from aliyun_gpushare_device_plugin_amd import const
from aliyun_gpushare_device_plugin_amd.cli.main import build_parser, config_from_args

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _docs():
    for path in sorted(glob.glob(os.path.join(ROOT, "deploy", "**", "*.yaml"), recursive=True)):
        with open(path) as f:
            for d in yaml.safe_load_all(f):
                if d:
                    yield path, d


def _pod_specs(d):
    spec = d.get("spec", {})
    if d["kind"] == "Pod":
        yield d["metadata"], spec
    elif "template" in spec:
        yield spec["template"].get("metadata", {}), spec["template"]["spec"]


def test_manifests_parse_and_have_kinds():
    docs = list(_docs())
    assert len(docs) >= 6
    assert all("kind" in d and "apiVersion" in d for _, d in docs)


def test_daemonset_flags_are_accepted_by_the_cli():
    cmd = _ds()["containers"][0]["command"]
    cfg = config_from_args(build_parser().parse_args([a for a in cmd[1:] if a.startswith("--")]))
    assert cfg.memory_unit == const.GIB and cfg.hbm_broker_dir == "/var/run/gpushare/hbm"
    # the commented-out isolation flag is valid too
    assert config_from_args(build_parser().parse_args(["--compute-isolation=cu"])).compute_isolation == "cu"


def test_demo_pods_use_the_plugin_contract():
    seen = 0
    for path, d in _docs():
        for meta, spec in _pod_specs(d):
            for c in spec.get("containers", []):
                lim = c.get("resources", {}).get("limits", {})
                if const.RESOURCE_NAME in lim:
                    assert int(lim[const.RESOURCE_NAME]) > 0
                    seen += 1
            ann = meta.get("annotations") or {}
            for k in ann:
                if k.startswith("gpushare.amd.com/"):
                    assert k == const.POD_ANNOTATION_CU_SLOTS_REQUEST, (path, k)
    assert seen >= 4


def _ds(name="gpushare-device-plugin-ds"):
    ds = [d for _, d in _docs() if d["kind"] == "DaemonSet" and d["metadata"]["name"] == name]
    assert len(ds) == 1
    return ds[0]["spec"]["template"]["spec"]


def test_hbm_brokers_ship_on_by_default_with_the_plugin():
    """The default deployment runs what the bench measures: the brokers are a container of the
    plugin's own DaemonSet (no opt-in), the plugin's --hbm-broker-dir names the directory they
    serve, both containers mount it from the same hostPath, and the broker container is privileged
    for /dev/kfd. Only the plugin and the brokers mount the whole directory: a shared container
    gets its GPU's gpu<i>/ only (tests/test_allocate_engine.py), never admin/."""
    from aliyun_gpushare_device_plugin_amd.cli import hbmbroker

    ds = [d for _, d in _docs() if d["kind"] == "DaemonSet"]
    assert [d["metadata"]["name"] for d in ds] == ["gpushare-device-plugin-ds"]   # one DaemonSet: the product
    spec = _ds()
    plugin, brokers = spec["containers"]
    assert brokers["name"] == "hbm-brokers" and brokers["command"][0] == "gpushare-hbm-brokers"
    assert brokers["securityContext"]["privileged"] is True
    a = hbmbroker.build_parser().parse_args(brokers["command"][1:])
    cfg = config_from_args(build_parser().parse_args([x for x in plugin["command"][1:] if x.startswith("--")]))
    assert cfg.hbm_broker_dir == a.dir == "/var/run/gpushare/hbm"
    vols = {v["name"]: v for v in spec["volumes"]}
    for c in (plugin, brokers):
        m = {x["mountPath"]: x for x in c["volumeMounts"]}[a.dir]
        assert vols[m["name"]]["hostPath"]["path"] == a.dir and not m.get("readOnly")


def test_daemonset_can_open_kfd_and_render_nodes():
    """Round-2 review item 3: a hostPath mount of /dev/kfd without a device-cgroup grant is
    refused at open(), so SMI event notification could never arm in a cluster. The plugin
    container must be privileged (AMD's own device plugin does the same) — and then the
    security context must not contradict it — and /readyz must gate readiness on it."""
    spec = _ds()
    c = spec["containers"][0]
    sc = c.get("securityContext") or {}
    assert sc.get("privileged") is True
    # the API server rejects privileged + allowPrivilegeEscalation=false; dropping all
    # capabilities would also defeat the KFD SMI-event ioctl
    assert sc.get("allowPrivilegeEscalation") is not False
    assert "ALL" not in ((sc.get("capabilities") or {}).get("drop") or [])
    assert c["readinessProbe"]["httpGet"]["path"] == "/readyz"
    assert c["livenessProbe"]["httpGet"]["path"] == "/healthz"
    port = int(next(a for a in c["command"] if a.startswith("--metrics-addr=")).rsplit(":", 1)[1])
    assert c["readinessProbe"]["httpGet"]["port"] == port


def test_daemonset_mounts_match_the_flags():
    """Every host path a flag names is mounted: the device-plugin dir (kubelet.sock + our
    socket), the kubelet pod-resources socket (placement truth), the shim/ledger/journal dir
    and /sys (read-only, SMI + KFD topology)."""
    spec = _ds()
    c = spec["containers"][0]
    mounts = {m["mountPath"]: m for m in c["volumeMounts"]}
    vols = {v["name"]: v for v in spec["volumes"]}
    for path in ("/var/lib/kubelet/device-plugins", "/var/lib/kubelet/pod-resources", "/var/lib/gpushare", "/sys"):
        assert path in mounts, path
        assert vols[mounts[path]["name"]]["hostPath"]["path"] == path
    assert mounts["/sys"].get("readOnly") is True
    cfg = config_from_args(build_parser().parse_args([a for a in c["command"][1:] if a.startswith("--")]))
    assert os.path.dirname(cfg.pod_resources_socket) == "/var/lib/kubelet/pod-resources"
    for p in (cfg.ledger_dir, cfg.journal_path):
        assert p.startswith("/var/lib/gpushare/")
    assert spec.get("hostNetwork") is True and spec["nodeSelector"] == {"gpushare": "true"}
    # the quota watchdog reads every GPU process's DRM fdinfo and pod cgroup
    assert spec.get("hostPID") is True
    # round-3 review item 4: non-cooperative tenants are enforced by default — kill where the
    # kernel has no dmem controller (the pod-resources mount above is what kill mode needs)
    assert cfg.quota_enforcement in ("auto", "kill")
    # kernel dmem limits write the HOST cgroup hierarchy (the container's own is namespaced)
    assert cfg.dmem_limits == "auto" and cfg.cgroup_root in mounts and not mounts[cfg.cgroup_root].get("readOnly")
    assert vols[mounts[cfg.cgroup_root]["name"]]["hostPath"]["path"] == "/sys/fs/cgroup"


def test_dockerfile_recipe_builds_and_installs(tmp_path):
    """Round-2 review: the image was never built. No container runtime here, so the image's
    own steps are replayed from the Dockerfile: the COPY sources exist, the build stage's RUN
    compiles the native pieces from a clean copy, and the runtime stage's pip install yields
    the reference's binary names, which start and parse the DaemonSet's command line."""
    import re
    import shutil
    import subprocess
    import sys

    text = open(os.path.join(ROOT, "deploy", "Dockerfile")).read()
    copies = [c for ln in text.splitlines() if ln.startswith("COPY ") and "--from" not in ln
              for c in ln.split()[1:-1]]
    assert copies and all(os.path.exists(os.path.join(ROOT, c)) for c in copies), copies
    src = tmp_path / "src"
    for c in copies:
        s, d = os.path.join(ROOT, c), src / c
        if os.path.isdir(s):
            shutil.copytree(s, d, ignore=shutil.ignore_patterns("_native", "__pycache__", "*.so", "*.o"))
        else:
            d.parent.mkdir(parents=True, exist_ok=True)
            shutil.copy(s, d)
    build = re.search(r"RUN (python3 native/build\.py [^\n]+)", text).group(1)
    r = subprocess.run(build.replace("python3", sys.executable).split(), cwd=src, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    native = src / "aliyun_gpushare_device_plugin_amd" / "_native"
    assert (native / "libgpushare_gpuinfo.so").exists() and (native / "libgpushare_hipquota.so").exists()
    assert (native / "gpushare-smi").exists()
    assert (native / "libgpushare_dpserver.so").exists()       # the native DevicePlugin server
    assert (native / "gpushare-hbm-broker").exists()           # the per-GPU HBM broker
    site = tmp_path / "site"
    r = subprocess.run([sys.executable, "-m", "pip", "install", "--no-deps", "--no-build-isolation", "--no-index",
                        "--target", str(site), str(src)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    for name in ("gpushare-device-plugin", "kubectl-inspect-gpushare"):
        assert (site / "bin" / name).exists(), name
    ds = _ds()["containers"][0]["command"]
    assert ds[0] == "gpushare-device-plugin-v2"          # the symlink the runtime stage adds
    env = dict(os.environ, PYTHONPATH=str(site), GPUSHARE_NO_AUTOBUILD="1")
    r = subprocess.run([sys.executable, str(site / "bin" / "gpushare-device-plugin"), "--help"], env=env,
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "--quota-enforcement" in r.stdout
    probe = ("import sys; from aliyun_gpushare_device_plugin_amd.cli.main import build_parser, config_from_args; "
             "cfg = config_from_args(build_parser().parse_args(sys.argv[1:])); "
             "import aliyun_gpushare_device_plugin_amd.utils.native as n; print(n.lib_path('hipshim'))")
    r = subprocess.run([sys.executable, "-c", probe, *[a for a in ds[1:] if a.startswith("-")]], env=env, cwd=tmp_path,
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().startswith(str(site)) and os.path.exists(r.stdout.strip())


def test_scheduler_extender_manifest_matches_the_cli():
    """The extender Deployment's flags parse, its Service port is the one it listens on, and
    the KubeSchedulerConfiguration points filter/bind at the routes it serves."""
    import yaml as _yaml

    from aliyun_gpushare_device_plugin_amd.cli import extender as X

    docs = [d for p, d in _docs() if p.endswith("scheduler-extender.yaml")]
    dep = next(d for d in docs if d["kind"] == "Deployment")
    cmd = dep["spec"]["template"]["spec"]["containers"][0]["command"]
    a = X.build_parser().parse_args(cmd[1:])
    svc = next(d for d in docs if d["kind"] == "Service")
    assert svc["spec"]["ports"][0]["targetPort"] == a.port
    cm = next(d for d in docs if d["kind"] == "ConfigMap")
    cfg = _yaml.safe_load(cm["data"]["scheduler-config.yaml"])
    ext = cfg["extenders"][0]
    assert ext["urlPrefix"].endswith(f":{a.port}/gpushare-scheduler")
    assert (ext["filterVerb"], ext["bindVerb"]) == ("filter", "bind")
    assert ext["managedResources"][0]["name"] == const.RESOURCE_NAME
    rules = next(d for d in docs if d["kind"] == "ClusterRole")["rules"]
    assert any("pods/binding" in r["resources"] and "create" in r["verbs"] for r in rules)
