"""Deployment rehearsal: run the shipped manifests the way a node would, without a cluster.

``deploy/device-plugin-ds.yaml`` and ``deploy/scheduler-extender.yaml`` are read as written; each
container is started as a local process with the manifest's own command and environment, and
every hostPath volume is bind-"mounted" by rewriting the container paths in its arguments and
environment to a host directory (what the container runtime's mount namespace does). The
kube-scheduler side uses the KubeSchedulerConfiguration in the extender's ConfigMap — its
``urlPrefix`` / ``filterVerb`` / ``bindVerb`` — and the workloads come from ``deploy/demo``.

Only what a CPU-only container cannot provide is overridden, and each override is listed in
``Rehearsal.overrides``: the SMI backend (no GPU here: a fake MI355X node), the apiserver
address (no in-cluster service account: the fake apiserver), listening ports (free ones instead
of the fixed 9400 / 39999), and the service DNS name in the scheduler config (127.0.0.1).
The reference ships the same two pieces (``device-plugin-ds.yaml``, and the extender from its
sister project); this is the closest this repository can come to ``kubectl apply`` on a node.
"""
from __future__ import annotations

import dataclasses
import json
import os
import socket
import subprocess
import sys
import time
import urllib.parse
import urllib.request

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# console entry points (setup.cfg) -> modules, for running a manifest's command without installing
ENTRY_POINTS = {
    "gpushare-device-plugin-v2": "aliyun_gpushare_device_plugin_amd.cli.main",
    "gpushare-scheduler-extender": "aliyun_gpushare_device_plugin_amd.cli.extender",
    "kubectl-inspect-gpushare": "aliyun_gpushare_device_plugin_amd.cli.inspect",
    "gpushare-hbm-brokers": "aliyun_gpushare_device_plugin_amd.cli.hbmbroker",
    "gpushare-comgr-cache": "aliyun_gpushare_device_plugin_amd.cli.comgrcache",
}


def load(path: str) -> list[dict]:
    with open(path) as f:
        return [d for d in yaml.safe_load_all(f) if d]


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def pod_template(doc: dict) -> dict:
    spec = doc["spec"]
    return spec["template"] if "template" in spec else {"metadata": doc.get("metadata", {}), "spec": spec}


@dataclasses.dataclass
class Container:
    """One manifest container, resolved for a local run."""
    argv: list
    env: dict
    mounts: dict            # container path -> host path

    def host_path(self, cpath: str) -> str:
        for c in sorted(self.mounts, key=len, reverse=True):
            if cpath == c or cpath.startswith(c.rstrip("/") + "/"):
                return self.mounts[c] + cpath[len(c.rstrip("/")):]
        return cpath


def _rewrite(value: str, mounts: dict) -> str:
    """Container paths inside one argument (``--flag=/path`` or ``/path``) -> host paths."""
    flag, eq, rest = value.partition("=")
    target = rest if eq else value
    for c in sorted(mounts, key=len, reverse=True):
        if target == c or target.startswith(c.rstrip("/") + "/"):
            target = mounts[c] + target[len(c.rstrip("/")):]
            break
    return f"{flag}={target}" if eq else target


def resolve(doc: dict, host_root: str, field_refs: dict, overrides: dict, skip_volumes=(),
            container: str | None = None) -> Container:
    """A container of a DaemonSet / Deployment (the first, or the one named ``container``, which
    may be an init container):
    command with hostPath volumes mapped under ``host_root`` (one directory per volume, shared by
    the pod's containers as a hostPath is), env with downward-API ``fieldRef`` values from
    ``field_refs``, and ``overrides`` ({flag: value or None to drop}) applied to the flags."""
    spec = pod_template(doc)["spec"]
    c = spec["containers"][0] if container is None else next(
        x for x in spec["containers"] + spec.get("initContainers", []) if x["name"] == container)
    vols = {v["name"]: v for v in spec.get("volumes", [])}
    mounts = {}
    for m in c.get("volumeMounts", []):
        v = vols[m["name"]]
        if "hostPath" not in v or m["name"] in skip_volumes:
            continue
        host = os.path.join(host_root, m["name"])
        os.makedirs(host, exist_ok=True)
        mounts[m["mountPath"]] = host
    argv = list(c.get("command", [])) + list(c.get("args", []))
    if argv and argv[0] in ENTRY_POINTS:
        argv = [sys.executable, "-m", ENTRY_POINTS[argv[0]]] + argv[1:]
    out, seen = [], set()
    for a in argv:
        flag = a.partition("=")[0]
        if flag in overrides:
            seen.add(flag)
            if overrides[flag] is not None:
                out.append(f"{flag}={overrides[flag]}")
            continue
        out.append(_rewrite(a, mounts) if a.startswith(("/", "-")) else a)
    out += [f"{f}={v}" for f, v in overrides.items() if f not in seen and v is not None]
    env = {}
    for e in c.get("env", []):
        if "value" in e:
            env[e["name"]] = _rewrite(e["value"], mounts)
        elif "valueFrom" in e and "fieldRef" in e["valueFrom"]:
            env[e["name"]] = field_refs[e["valueFrom"]["fieldRef"]["fieldPath"]]
    return Container(out, env, mounts)


def start(ct: Container, log_path: str) -> subprocess.Popen:
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""), **ct.env)
    return subprocess.Popen(ct.argv, env=env, stdout=subprocess.PIPE, stderr=open(log_path, "w"), text=True)


def http_get(url: str, timeout: float = 5.0) -> tuple[int, str]:
    try:
        with urllib.request.urlopen(url, timeout=timeout) as r:
            return r.status, r.read().decode()
    except urllib.error.HTTPError as e:
        return e.code, e.read().decode()


class Scheduler:
    """The kube-scheduler half of the extender contract, driven by the ConfigMap's
    KubeSchedulerConfiguration (extenders[0]: urlPrefix, filterVerb, bindVerb)."""

    def __init__(self, config_yaml: str, host_port: str):
        ext = yaml.safe_load(config_yaml)["extenders"][0]
        u = urllib.parse.urlsplit(ext["urlPrefix"])
        self.prefix = urllib.parse.urlunsplit((u.scheme, host_port, u.path, "", ""))
        self.filter_verb, self.bind_verb = ext["filterVerb"], ext["bindVerb"]
        self.managed = [r["name"] for r in ext.get("managedResources", [])]

    def _post(self, verb: str, body: dict) -> dict:
        req = urllib.request.Request(f"{self.prefix}/{verb}", json.dumps(body).encode(),
                                     {"Content-Type": "application/json"})
        with urllib.request.urlopen(req, timeout=10) as r:
            return json.loads(r.read())

    def schedule(self, pod: dict, nodes: list[str]) -> str | None:
        f = self._post(self.filter_verb, {"Pod": pod, "NodeNames": nodes})
        if not f.get("NodeNames"):
            return None
        md = pod["metadata"]
        b = self._post(self.bind_verb, {"PodName": md["name"], "PodNamespace": md.get("namespace", "default"),
                                        "PodUID": md["uid"], "Node": f["NodeNames"][0]})
        if b.get("Error"):
            raise RuntimeError(b["Error"])
        return f["NodeNames"][0]


def wait_for(pred, timeout: float = 20.0, step: float = 0.05) -> bool:
    t = time.monotonic() + timeout
    while time.monotonic() < t:
        if pred():
            return True
        time.sleep(step)
    return False
