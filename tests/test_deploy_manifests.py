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
    ds = [d for _, d in _docs() if d["kind"] == "DaemonSet"]
    assert ds
    cmd = ds[0]["spec"]["template"]["spec"]["containers"][0]["command"]
    cfg = config_from_args(build_parser().parse_args([a for a in cmd[1:] if a.startswith("--")]))
    assert cfg.memory_unit == const.GIB
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


def _ds():
    ds = [d for _, d in _docs() if d["kind"] == "DaemonSet"]
    assert len(ds) == 1
    return ds[0]["spec"]["template"]["spec"]


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
    assert spec.get("hostPID") is True and cfg.quota_enforcement in ("report", "kill")
