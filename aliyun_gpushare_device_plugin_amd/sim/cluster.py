"""Composable fake cluster: apiserver + N nodes (fake kubelet + real plugin) + extender.

"Multi-node without a real cluster" (SURVEY §4): every node runs the real plugin code
(``SharedGPUManager`` — in a thread, or as a separate ``gpushare-device-plugin`` process for
honest IPC timing) against a shared fake apiserver, and pods flow through the same path as
in production: create → extender filter/bind (annotations) → kubelet admission → plugin
``Allocate`` over gRPC/UDS → ``ASSIGNED=true`` patch → Running.
"""
from __future__ import annotations

import dataclasses
import itertools
import os
import shutil
import signal
import subprocess
import sys
import tempfile
import threading
import time

from .. import const
from ..cluster import objects as O
from ..cluster.client import APIClient, KubeConfig
from ..plugin.manager import PluginConfig, SharedGPUManager
from ..utils import log
from .apiserver import FakeAPIServer, make_node
from ..extender import TP_GROUP_LABEL, TP_SIZE_LABEL, Extender
from .kubelet import Admission, FakeKubelet
from .kubelet_proc import KubeletProcess


def pod_spec(name: str, gpu_mem, namespace: str = "default", labels: dict | None = None,
             image: str = "rocm/pytorch:latest", annotations: dict | None = None) -> dict:
    """A pod with one container per entry of ``gpu_mem`` (int → single container)."""
    mems = [gpu_mem] if isinstance(gpu_mem, int) else list(gpu_mem)
    ctrs = [{"name": f"c{i}", "image": image,
             "resources": {"limits": {const.RESOURCE_NAME: str(m)}} if m else {}} for i, m in enumerate(mems)]
    return {"apiVersion": "v1", "kind": "Pod",
            "metadata": {"name": name, "namespace": namespace, "labels": dict(labels or {}),
                         **({"annotations": dict(annotations)} if annotations else {})},
            "spec": {"containers": ctrs, "schedulerName": "default-scheduler"}}


@dataclasses.dataclass
class SimNode:
    name: str
    smi_spec: str
    plugin_dir: str
    kubelet: "FakeKubelet | KubeletProcess"
    manager: SharedGPUManager | None = None
    thread: threading.Thread | None = None
    proc: subprocess.Popen | None = None


class SimCluster:
    def __init__(self, nodes: list[tuple[str, str]], workdir: str | None = None, plugin_mode: str = "thread",
                 pod_source: str = "watch", apiserver_latency_s: float = 0.0, shim_host_dir: str | None = None,
                 gpu_indices: list[int] | None = None, health_poll_s: float = 1.0, round_policy: str = "nearest",
                 extra_plugin_args: list[str] | None = None, apiserver: str = "thread",
                 preferred_allocation: bool = False, compute_isolation: str = "none", kubelet: str = "thread",
                 placement_truth: bool = True, node_overrides: dict | None = None,
                 admission_identity: bool = True, grpc_server: str = "auto", daemon_cpus: dict | None = None):
        self.node_specs = nodes
        # process-mode children's CPUs, by role ("plugin", "apiserver", "kubelet": "3" / "6-7"), as a
        # node reserves CPUs for its daemons (the package import applies GPUSHARE_CPUS)
        self.daemon_cpus = dict(daemon_cpus or {})
        # kubelet: "thread" (FakeKubelet in this interpreter) or "process" (its own interpreter,
        # sim/kubelet_proc.py, so kubelet-side Allocate timing is not inflated by this process's GIL)
        self.kubelet_mode = kubelet
        # per-node plugin settings: {node: {"pod_source": ..., "extra_args": [...]}} (e.g. a second
        # node running the reference's cost model next to the default one, bench.py)
        self.node_overrides = node_overrides or {}
        self.grpc_server = grpc_server
        # the fake kubelet serves pod-resources; the plugin uses it for placement truth
        self.placement_truth = placement_truth
        self.admission_identity = admission_identity
        self.compute_isolation = compute_isolation
        self._own_dir = workdir is None
        # short paths: UDS paths are limited to 108 bytes
        self.workdir = workdir or tempfile.mkdtemp(prefix="gs-", dir="/tmp")
        self.plugin_mode = plugin_mode
        self.pod_source = pod_source
        # apiserver: "thread" (in-process) or "process" (separate interpreter, so the
        # control-plane latency is not inflated by this process's GIL)
        self.api_mode = apiserver
        self.api = FakeAPIServer(latency_s=apiserver_latency_s) if apiserver == "thread" else None
        self.api_proc = None
        self.api_url = None
        self.apiserver_latency_s = apiserver_latency_s
        self.client: APIClient | None = None
        self.extender: Extender | None = None
        self.nodes: dict[str, SimNode] = {}
        self.shim_host_dir = shim_host_dir
        self.gpu_indices = gpu_indices
        self.health_poll_s = health_poll_s
        self.round_policy = round_policy
        self.extra_plugin_args = extra_plugin_args or []
        self.preferred_allocation = preferred_allocation
        self._seq = itertools.count(1)
        import concurrent.futures as cf
        self._bg = cf.ThreadPoolExecutor(max_workers=1, thread_name_prefix="status")   # ordered

    # -- lifecycle ------------------------------------------------------------------------
    def _start_apiserver(self):
        if self.api is not None:
            self.api.start()
            self.api_url = self.api.url
            return
        self.api_proc = subprocess.Popen(
            [sys.executable, "-m", "aliyun_gpushare_device_plugin_amd.sim.apiserver", "--port", "0",
             "--latency-ms", str(self.apiserver_latency_s * 1e3)],
            env=self._child_env("apiserver"), stdout=subprocess.PIPE, text=True)
        self.api_url = self.api_proc.stdout.readline().strip()
        if not self.api_url.startswith("http"):
            raise RuntimeError("fake apiserver process failed to start")

    def _child_env(self, role: str = ""):
        env = dict(os.environ)
        if self.daemon_cpus.get(role):
            env["GPUSHARE_CPUS"] = str(self.daemon_cpus[role])
        env.setdefault("GPUSHARE_DEBUG", "1")      # simulator children: debug endpoints on
        # SIGTERM the child when the simulator dies (a killed test or bench leaves no fake
        # apiserver / kubelet / plugin behind); armed by the package import, after exec
        env["GPUSHARE_DIE_WITH_PARENT"] = str(os.getpid())
        env["PYTHONPATH"] = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))) + \
            os.pathsep + env.get("PYTHONPATH", "")
        return env

    def start(self, timeout: float = 30.0):
        self._start_apiserver()
        self.client = APIClient(KubeConfig(self.api_url))
        for name, spec in self.node_specs:
            self.client.create_node(make_node(name))
            pdir = os.path.join(self.workdir, name)
            if self.kubelet_mode == "process" and self.pod_source != "kubelet":
                kl = KubeletProcess(pdir, self.api_url, name, env=self._child_env("kubelet")).start()
            else:
                kl = FakeKubelet(pdir, APIClient(KubeConfig(self.api_url)), name).start()
                if self.pod_source == "kubelet":
                    kl.serve_pods()
            node = SimNode(name, spec, pdir, kl)
            self.nodes[name] = node
            self._start_plugin(node)
        for node in self.nodes.values():
            if not node.kubelet.registered.wait(timeout):
                raise TimeoutError(f"plugin on {node.name} did not register{self._plugin_log_tail(node)}")
            if node.manager is not None and not node.manager.started.wait(timeout):
                raise TimeoutError(f"plugin manager on {node.name} did not finish starting")
            self._wait_capacity(node.name, timeout)
        self.extender = Extender(self.client)
        self.extender.sync()
        return self

    def _pod_source(self, node: SimNode) -> str:
        return self.node_overrides.get(node.name, {}).get("pod_source", self.pod_source)

    def _plugin_cfg(self, node: SimNode) -> PluginConfig:
        return PluginConfig(node_name=node.name, smi_backend=node.smi_spec, device_plugin_dir=node.plugin_dir,
                            apiserver=self.api_url, pod_source=self._pod_source(node),
                            shim_host_dir=self.shim_host_dir, gpu_indices=self.gpu_indices,
                            health_poll_s=self.health_poll_s, round_policy=self.round_policy,
                            preferred_allocation=self.preferred_allocation,
                            compute_isolation=self.compute_isolation, pod_resources_socket=self._podres(node),
                            admission_identity=self.admission_identity, grpc_server=self.grpc_server,
                            **self._kubelet_cfg(node))

    def _thread_cfg(self, node: SimNode) -> PluginConfig:
        """The in-process plugin's config: ``_plugin_cfg`` plus whatever the extra plugin
        arguments (the command-line flags a process-mode plugin gets) set away from their
        defaults, so both modes run the same plugin."""
        cfg = self._plugin_cfg(node)
        ov = self.node_overrides.get(node.name, {})
        extra = list(ov["extra_args"] if "extra_args" in ov else self.extra_plugin_args)
        if extra:
            import dataclasses

            from ..cli.main import build_parser, config_from_args

            base = config_from_args(build_parser().parse_args([]))
            over = config_from_args(build_parser().parse_args(extra))
            for f in dataclasses.fields(cfg):
                v = getattr(over, f.name)
                if v != getattr(base, f.name):
                    setattr(cfg, f.name, v)
        return cfg

    def _podres(self, node: SimNode) -> str:
        return os.path.join(node.plugin_dir, "pod-resources.sock") if self.placement_truth else "none"

    def _kubelet_cfg(self, node: SimNode) -> dict:
        if self.pod_source != "kubelet":
            return {}
        return {"kubelet_address": "127.0.0.1", "kubelet_port": node.kubelet.pods_port, "kubelet_scheme": "http",
                "token": node.kubelet.pods_token}

    def _start_plugin(self, node: SimNode):
        if self.plugin_mode == "process":
            args = [sys.executable, "-m", "aliyun_gpushare_device_plugin_amd.cli.main",
                    "--node-name", node.name, "--smi-backend", node.smi_spec,
                    "--device-plugin-dir", node.plugin_dir, "--apiserver", self.api_url,
                    "--pod-source", self._pod_source(node), "--round", self.round_policy,
                    "--health-poll", str(self.health_poll_s)]
            if self.shim_host_dir:
                args += ["--shim-path", self.shim_host_dir]
            if self.gpu_indices:
                args += ["--gpu-indices", ",".join(map(str, self.gpu_indices))]
            if self.preferred_allocation:
                args += ["--preferred-allocation"]
            if self.compute_isolation != "none":
                args += ["--compute-isolation", self.compute_isolation]
            args += ["--pod-resources-socket", self._podres(node),
                     "--admission-identity", "true" if self.admission_identity else "false",
                     "--grpc-server", self.grpc_server]
            for k, v in self._kubelet_cfg(node).items():
                args += ["--" + k.replace("_", "-"), str(v)]
            ov = self.node_overrides.get(node.name, {})
            args += ov["extra_args"] if "extra_args" in ov else self.extra_plugin_args
            role = f"plugin:{node.name}" if f"plugin:{node.name}" in self.daemon_cpus else "plugin"
            node.proc = subprocess.Popen(args, env=self._child_env(role), stdout=subprocess.DEVNULL,
                                         stderr=open(os.path.join(self.workdir, f"{node.name}.plugin.log"), "w"))
        else:
            node.manager = SharedGPUManager(self._thread_cfg(node), client=APIClient(KubeConfig(self.api_url)))
            node.thread = threading.Thread(target=node.manager.run, kwargs={"install_signals": False},
                                           name=f"plugin-{node.name}", daemon=True)
            node.thread.start()

    def kill_plugin(self, node: str, sig: int = signal.SIGKILL):
        """Fault injection: kill a process-mode plugin outright (no shutdown path runs)."""
        n = self.nodes[node]
        if n.proc is None:
            raise RuntimeError("kill_plugin needs plugin_mode='process'")
        n.proc.send_signal(sig)
        n.proc.wait(timeout=10)

    def restart_plugin(self, node: str, timeout: float = 30.0):
        """Start the plugin of ``node`` again (after ``kill_plugin``) and wait until it has
        re-registered with the fake kubelet and re-opened ListAndWatch."""
        n = self.nodes[node]
        n.kubelet.registered.clear()
        self._start_plugin(n)
        if not n.kubelet.registered.wait(timeout):
            if n.proc is not None and n.proc.poll() is None:
                n.proc.send_signal(signal.SIGUSR2)       # every thread's stack into its log
                time.sleep(1.0)
            raise TimeoutError(f"plugin on {node} did not re-register{self._plugin_log_tail(n, 20000)}")

    def _plugin_log_tail(self, node, n: int = 3000) -> str:
        """The end of a process-mode plugin's log, for timeout messages."""
        try:
            with open(os.path.join(self.workdir, f"{node.name}.plugin.log")) as f:
                return "; plugin log tail:\n" + f.read()[-n:]
        except OSError:
            return ""

    def _wait_capacity(self, node: str, timeout: float):
        t = time.monotonic() + timeout
        while time.monotonic() < t:
            n = self.client.get_node(node)
            if O.node_allocatable(n, const.RESOURCE_COUNT) > 0 and O.node_allocatable(n, const.RESOURCE_NAME) > 0:
                return n
            time.sleep(0.02)
        raise TimeoutError(f"node {node} never reported gpu capacity")

    def stop(self):
        self._bg.shutdown(wait=True)
        if self.extender is not None:
            self.extender.stop_watch()
        for node in self.nodes.values():
            if node.manager is not None:
                node.manager.stop()
                if node.thread is not None:
                    node.thread.join(timeout=5)
            if node.proc is not None:
                node.proc.terminate()
                try:
                    node.proc.wait(timeout=10)
                except subprocess.TimeoutExpired:
                    node.proc.kill()
            node.kubelet.stop()
        if self.api is not None:
            self.api.stop()
        if self.api_proc is not None:
            self.api_proc.terminate()
            try:
                self.api_proc.wait(timeout=10)
            except subprocess.TimeoutExpired:
                self.api_proc.kill()
        if self._own_dir:
            shutil.rmtree(self.workdir, ignore_errors=True)

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()

    # -- pod flow -------------------------------------------------------------------------
    def create_pod(self, gpu_mem, name: str | None = None, labels: dict | None = None,
                   annotations: dict | None = None) -> dict:
        pod = self.client.create_pod("default", pod_spec(name or f"pod-{next(self._seq)}", gpu_mem, labels=labels,
                                                         annotations=annotations))
        if self.extender is not None:
            self.extender.note_pending(pod)       # what the extender's pod informer sees
        return pod

    def schedule(self, pod: dict, node_names: list | None = None):
        return self.extender.schedule(pod, node_names)

    def admit(self, pod: dict, async_status: bool = False) -> Admission:
        """Kubelet admission. ``pod`` may be the bound object the caller already holds (the
        kubelet gets it from its own watch); otherwise it is fetched. With ``async_status`` the
        Running status is posted off the admission path, as the kubelet's status manager does."""
        if not O.node_name(pod):
            pod = self.client.get_pod(O.namespace(pod), O.name(pod))
        node = self.nodes[O.node_name(pod)]
        self._watch_delivered(node, pod)
        adm = node.kubelet.admit(pod)
        if adm.error is None:
            ns, nm = O.namespace(pod), O.name(pod)
            if async_status:
                self._bg.submit(self.client.patch_pod_status, ns, nm, {"status": {"phase": "Running"}})
            else:
                self.client.patch_pod_status(ns, nm, {"status": {"phase": "Running"}})
        return adm

    @staticmethod
    def _watch_delivered(node, pod: dict, timeout: float = 2.0) -> None:
        """The kubelet admits a pod once its own apiserver watch delivered the binding — the
        same event stream the plugin's pod informer reads, so the plugin has (nearly always)
        seen it too. The harness hands the kubelet the bound object straight from the bind
        call; with the plugin in this process, wait until its informer has the binding as well
        (a kubelet that outruns the informer is the watch-lag case, covered by the full path's
        fresh LIST and by placement truth)."""
        src = getattr(getattr(node.manager, "allocator", None), "pods", None)
        if src is None or not hasattr(src, "pending_version"):
            return
        u = O.uid(pod)
        t = time.monotonic() + timeout
        while time.monotonic() < t:
            p = src.get(u)
            if p is not None and O.node_name(p):
                return
            time.sleep(0.0005)

    def wait_assigned(self, pod: dict, timeout: float = 10.0) -> dict:
        """Wait until the plugin's (write-behind) ASSIGNED=true patch is visible."""
        t = time.monotonic() + timeout
        while True:
            got = self.client.get_pod(O.namespace(pod), O.name(pod))
            if O.annotations(got).get(const.ENV_ASSIGNED_FLAG) == "true" or time.monotonic() > t:
                return got
            time.sleep(0.005)

    def flush(self):
        """Wait for asynchronous status updates."""
        self._bg.submit(lambda: None).result()

    def run_pod(self, gpu_mem, name: str | None = None, labels: dict | None = None,
                annotations: dict | None = None, node_names: list | None = None):
        pod = self.create_pod(gpu_mem, name, labels, annotations)
        placed = self.schedule(pod, node_names)
        if placed is None:
            return pod, None, None
        return pod, placed, self.admit(pod)

    def run_tp_group(self, group: str, size: int, gpu_mem: int):
        pods = [self.create_pod(gpu_mem, labels={TP_GROUP_LABEL: group, TP_SIZE_LABEL: str(size)})
                for _ in range(size)]
        placed = self.extender.schedule_group(pods)
        if placed is None:
            return pods, None, []
        return pods, placed, [self.admit(p) for p in pods]

    def delete_pod(self, pod: dict):
        if not O.node_name(pod):
            pod = self.client.get_pod(O.namespace(pod), O.name(pod))
        nn = O.node_name(pod)
        if nn in self.nodes:
            self.nodes[nn].kubelet.release(O.uid(pod))
        self.extender.forget(pod)
        self.client.delete_pod(O.namespace(pod), O.name(pod))

    def manager(self, node: str) -> SharedGPUManager | None:
        return self.nodes[node].manager


def quiet():
    log.setup(verbosity=0)
