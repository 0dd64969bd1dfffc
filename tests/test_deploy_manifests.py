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
