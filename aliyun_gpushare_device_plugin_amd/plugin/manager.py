"""Lifecycle supervisor (component C9; reference ``pkg/gpu/nvidia/gpumanager.go:16-111``).

Same state machine as the reference:
* init the SMI layer; if it fails or finds no GPU, park (the reference ``select{}``s forever
  so the DaemonSet does not crash-loop) — here parking still honours SIGTERM;
* watch the device-plugin directory; re-creation of ``kubelet.sock`` (kubelet restart) or
  SIGHUP rebuilds the plugin: re-enumerate, re-patch ``gpu-count``, re-register;
* SIGQUIT dumps all stacks; SIGINT/SIGTERM stop cleanly;
* construction failure exits 1, serve/register failure exits 2 (``:71-77``).
Additions: topology export, the live health monitor, the metrics endpoint, and a choice of
pod source (watch cache by default).
"""
from __future__ import annotations

import dataclasses
import os
import queue
import signal
import threading
import time

from .. import const
from ..alloc.engine import Allocator, AllocatorOptions
from ..cluster import nodestatus, objects as O
from ..cluster.client import APIClient, build_client
from ..cluster.kubelet import KubeletClient
from ..cluster.podcache import KubeletSource, ListSource, PrebindWatch, WatchCache
from ..device import smi as S
from ..device.health import HealthMonitor
from ..device.model import DeviceConfigError, DeviceModel
from ..parallel import topology as T
from ..quota import ShimConfig
from ..utils import log, metrics as M, stackdump
from .server import DevicePluginServer
from .watchers import FSWatcher, watch_signals

# the plugin's cyclic-GC collections by generation and the time they took (the debug view; the
# bench line reports them for its timed window). Measured: none lands in a churn bench's timed
# window at CPython's default thresholds (profiles/r6/allocate_tail.md), so they are left alone.
GC_STATS = {"collections": [0, 0, 0], "ns": [0, 0, 0], "max_ns": 0}
_gc_t0 = [0]


def _gc_timer(phase: str, info: dict) -> None:
    if phase == "start":
        _gc_t0[0] = time.monotonic_ns()
        return
    dt = time.monotonic_ns() - _gc_t0[0]
    g = info.get("generation", 0)
    GC_STATS["collections"][g] += 1
    GC_STATS["ns"][g] += dt
    GC_STATS["max_ns"] = max(GC_STATS["max_ns"], dt)


def time_gc() -> None:
    import gc

    if _gc_timer not in gc.callbacks:
        gc.callbacks.append(_gc_timer)


@dataclasses.dataclass
class PluginConfig:
    node_name: str = ""
    memory_unit: str = const.GIB
    round_policy: str = "nearest"
    homogeneous: bool = True
    health_check: bool = True
    health_poll_s: float = 5.0
    pod_source: str = "watch"            # watch | list | kubelet
    query_kubelet: bool = False          # reference flag; implies pod_source=kubelet
    kubelet_address: str = "0.0.0.0"
    kubelet_port: int = 10250
    kubelet_scheme: str = "https"
    client_cert: str = ""
    client_key: str = ""
    token: str = ""
    timeout: float = 10.0
    smi_backend: str = "auto"
    device_plugin_dir: str = const.DEVICE_PLUGIN_PATH
    kubeconfig: str | None = None
    apiserver: str | None = None
    gpu_indices: list | None = None
    shim_host_dir: str | None = None     # None = do not inject the quota shim
    strict_allocate: bool = False
    preferred_allocation: bool = False   # opt-in: costs the kubelet one extra RPC per container
    export_topology: bool = True
    expose_devices: bool = True          # DeviceSpecs for /dev/kfd + the GPU's render node
    cdi_kind: str = ""                   # e.g. "amd.com/gpu": also answer CDI device names
    rocr_visible: bool = False
    metrics_addr: str | None = None
    async_patch: bool = True             # write-behind ASSIGNED patch (see AllocatorOptions)
    complete_swaps: bool = True          # match a swapped equal-size pod (see alloc/engine.py)
    partition_aware: bool = True         # divide NPS1-shared HBM among compute partitions
    ledger_dir: str | None = None        # host dir for file-backed shim ledgers (usage metrics)
    hbm_broker_dir: str | None = None    # host dir of the per-GPU HBM broker sockets (quota/hbmbroker.py)
    hbm_broker_fraction: float = 0.94
    comgr_cache_dir: str | None = None   # host dir of the node's read-only comgr cache (quota/comgr_cache.py)
    hbm_granter_args: dict = dataclasses.field(default_factory=dict)   # HBMGranter timing (tests)
    ledger_scan_s: float = 10.0
    journal_path: str | None = None      # persisted allocation journal (alloc/journal.py)
    compute_isolation: str = "none"      # "cu": per-pod CU-slot masks (alloc/cuslots.py)
    # kubelet pod-resources socket for placement truth (alloc/placement.py): "auto" = the
    # standard path when it exists, "none"/"" = off
    pod_resources_socket: str = "auto"
    placement_s: float = 2.0
    admission_identity: bool = True      # which pod is being admitted, from pod-resources (engine)
    # quota/watchdog.py: off | report | kill | auto (kill where the kernel has no dmem limits
    # and placement truth is on, so the share holds for a tenant that drops the shim)
    quota_enforcement: str = "auto"
    quota_watch_s: float = 10.0
    quota_slack_mib: int = 256
    dmem_limits: str = "auto"            # quota/dmem.py: kernel dmem.max per pod cgroup when available | off
    cgroup_root: str = "/sys/fs/cgroup"
    mps: bool = False                    # accepted for flag compatibility; ignored
    # DevicePlugin gRPC server: "native" (libgpushare_dpserver, Allocate fast path in C++),
    # "python" (grpcio), "auto" = native when the library loads
    grpc_server: str = "auto"
    native_fast_wait_us: int = 300       # native server: wait for a republished table (see native_server.py)
    prebind_watch: bool = True           # prepare answers of pods the extender placed here, before their bind
    native_spin_us: int = 0              # native server: busy-poll this long after a pod is published (0 = off)
    # re-read the node's cgpu.disable.isolation label this often (0 = only at start, as the
    # reference does): a flip re-prepares answers and sizes the HBM brokers to nothing / back
    label_poll_s: float = 10.0


class SharedGPUManager:
    def __init__(self, cfg: PluginConfig, client: APIClient | None = None, smi: S.SMI | None = None):
        self.cfg = cfg
        if cfg.query_kubelet:
            cfg.pod_source = "kubelet"
        if cfg.mps:
            log.warning("--mps is accepted for compatibility and ignored (no MPS on MI355X)")
        self.client = client
        self.smi = smi
        self.events: "queue.Queue" = queue.Queue()
        self.metrics = M.PluginMetrics()
        self._prebind = None
        self.metrics.registry.add_collector(lambda: M.native_server_exposition(self._debug_view().get("native_server")))
        self.plugin: DevicePluginServer | None = None
        self.health: HealthMonitor | None = None
        self.pod_source = None
        self.allocator: Allocator | None = None
        self.model: DeviceModel | None = None
        self.started = threading.Event()
        self.restarts = 0
        self._metrics_srv = None
        self._ledger_thread = None
        self._ledger_stop = threading.Event()
        self.watchdog = None
        self.dmem = None
        self.enforcement = "off"             # effective HBM-share enforcement (see _enforcement)
        self._cgpu_disabled = False
        self._label_thread = None

    # ------------------------------------------------------------------------------------
    def _kubelet_socket(self) -> str:
        return os.path.join(self.cfg.device_plugin_dir, const.KUBELET_SOCKET_NAME)

    def _plugin_socket(self) -> str:
        return os.path.join(self.cfg.device_plugin_dir, const.PLUGIN_SOCKET_NAME)

    def _export_topology(self):
        if not (self.cfg.export_topology and self.client and self.smi):
            return
        try:
            self.smi.refresh()                  # link state may have changed since enumeration
            topo = T.build_topology(self.smi, self.cfg.gpu_indices)
            nodestatus.export_topology(self.client, self.cfg.node_name, topo)
        except Exception as e:  # noqa: BLE001 - best effort, never blocks Allocate
            log.warning("topology export failed: %s", e)

    def _export_health(self, *_a):
        if not (self.client and self.model):
            return
        try:
            nodestatus.export_health(self.client, self.cfg.node_name, {
                str(g.index): {"uuid": g.uuid, "healthy": g.healthy and g.present, "reason": g.reason}
                for g in self.model.gpus})
        except Exception as e:  # noqa: BLE001
            log.warning("health export failed: %s", e)

    def build_plugin(self) -> DevicePluginServer:
        """``NewNvidiaDevicePlugin`` (``server.go:43-78``)."""
        cfg = self.cfg
        self.smi.refresh()
        model = DeviceModel(self.smi.devices(), cfg.memory_unit, cfg.round_policy, cfg.homogeneous,
                            cfg.gpu_indices, partition_aware=cfg.partition_aware)
        self.metrics.unit_fallback.set(1 if model.unit_fallback else 0)
        for g in model.gpus:
            self.metrics.units_per_gpu.set(g.units, gpu=str(g.index))
            self.metrics.device_health.set(1 if g.healthy else 0, gpu=str(g.index))
        disable_cgpu = False
        if self.client is not None:
            nodestatus.patch_gpu_count(self.client, cfg.node_name, model.count())
            nodestatus.export_memory_unit(self.client, cfg.node_name, model.unit)
            disable_cgpu = nodestatus.cgpu_isolation_disabled(self.client, cfg.node_name)
        if self.pod_source is not None:
            self.pod_source.stop()
        if self._prebind is not None:
            self._prebind.stop()
            self._prebind = None
        fallback = ListSource(self.client, cfg.node_name) if self.client else None
        if cfg.pod_source == "watch" and self.client is not None:
            src = WatchCache(self.client, cfg.node_name,
                             on_event=lambda t: self.metrics.cache_events.inc(type=t)).start()
            src.wait_synced(5.0)
        elif cfg.pod_source == "kubelet":
            kc = KubeletClient.from_flags(cfg.kubelet_address, cfg.kubelet_port, cfg.client_cert, cfg.client_key,
                                          cfg.token, cfg.timeout, cfg.kubelet_scheme)
            src = KubeletSource(kc, fallback)
        else:
            src = fallback
        self.pod_source = src
        shim = ShimConfig(cfg.shim_host_dir) if cfg.shim_host_dir else None
        opts = AllocatorOptions(unit=model.unit, disable_cgpu=disable_cgpu, shim=shim,
                                strict=cfg.strict_allocate, expose_devices=cfg.expose_devices,
                                cdi_kind=cfg.cdi_kind or None,
                                rocr_visible=cfg.rocr_visible, async_patch=cfg.async_patch,
                                complete_swaps=cfg.complete_swaps,
                                ledger_dir=cfg.ledger_dir if shim else None,
                                hbm_broker_dir=cfg.hbm_broker_dir if shim else None,
                                hbm_broker_fraction=cfg.hbm_broker_fraction,
                                comgr_cache_dir=cfg.comgr_cache_dir,
                                hbm_granter_args=dict(cfg.hbm_granter_args),
                                journal_path=cfg.journal_path,
                                compute_isolation=cfg.compute_isolation, placement_s=cfg.placement_s,
                                identify=cfg.admission_identity)
        if self.allocator is None:
            if cfg.async_patch and not cfg.journal_path:
                log.warning("write-behind ASSIGNED patches without --journal-path: a patch still queued when "
                            "the plugin process dies is lost (the reconcile pass only covers restarts in-process)")
            self.allocator = Allocator(model, src, self.client, cfg.node_name, opts, self.metrics)
        else:
            # rebuild: keep claims, assigned pods, queued patches and the patcher thread
            self.allocator.reconfigure(model, src, self.client, opts)
        self._cgpu_disabled = disable_cgpu
        allocator = self.allocator
        if allocator.podres is None:
            allocator.set_pod_resources(self._pod_resources())
        if cfg.prebind_watch and cfg.pod_source == "watch" and self.client is not None:
            self._prebind = PrebindWatch(self.client, cfg.node_name, allocator.precompute,
                                         on_gone=allocator.prebind_gone, trace=allocator._mark).start()
        self.model = model
        cls = self._server_class()
        kw = ({"fast_wait_us": cfg.native_fast_wait_us, "spin_us": cfg.native_spin_us}
              if cls is not DevicePluginServer else {})
        return cls(model, allocator, self._plugin_socket(), const.RESOURCE_NAME, cfg.preferred_allocation,
                   self.metrics, **kw)

    def _server_class(self):
        mode = self.cfg.grpc_server
        if mode == "python":
            return DevicePluginServer
        from .native_server import NativeDevicePluginServer, load

        try:
            load()
        except Exception as e:  # noqa: BLE001
            if mode == "native":
                raise
            log.warning("native device-plugin server unavailable (%s): serving with grpcio", e)
            return DevicePluginServer
        return NativeDevicePluginServer

    def readiness(self) -> tuple[bool, str]:
        """``/readyz``: serving and registered, with health detection at full strength (SMI
        event notification armed on every GPU). A DaemonSet pod that cannot open /dev/kfd shows
        NotReady instead of silently degrading to polling."""
        if self.plugin is None or self.plugin.stopped.is_set():
            return False, "device plugin not serving"
        if self.health is not None and not self.health.ready:
            return False, self.health.degraded
        if self.enforcement in ("report", "off") and not self._cgpu_disabled and self.cfg.shim_host_dir:
            return False, (f"HBM shares are not enforced on a tenant that drops the quota shim: no dmem cgroup "
                           f"controller and the watchdog is in {self.enforcement!r} mode")
        return True, "ok"

    def _enforcement(self) -> str:
        """Effective enforcement of the HBM shares on non-cooperative tenants: "dmem" (kernel
        limit per pod cgroup), "kill" (watchdog SIGKILL), "report" or "off". ``auto`` picks
        kill when the kernel cannot limit; kill needs placement truth (pod-resources), because
        without it a swapped admission leaves the annotations crossed and a pod inside its real
        share would be killed — it is downgraded to report then."""
        mode = self.cfg.quota_enforcement
        dmem_on = self.dmem is not None and self.dmem.available()
        podres = self.allocator is not None and self.allocator.podres is not None
        if mode == "auto":
            mode = "report" if dmem_on else "kill" if podres else "report"
        elif mode == "kill" and not podres:
            log.warning("--quota-enforcement=kill needs the kubelet pod-resources API (placement truth): without "
                        "it pod annotations can be crossed after a swapped admission; reporting only")
            mode = "report"
        eff = "dmem" if dmem_on and mode != "off" else mode
        for m in ("dmem", "kill", "report", "off"):
            self.metrics.enforcement_mode.set(1 if m == eff else 0, mode=m)
        if eff in ("report", "off") and self.cfg.shim_host_dir:
            log.warning("HBM shares are enforced by the quota shim only (%s): a tenant that drops LD_PRELOAD is "
                        "not limited", eff)
        self.enforcement = eff
        return mode

    def _debug_view(self) -> dict:
        stats = getattr(self.plugin, "stats", None)
        if not stats:
            return {}
        skipped = {dict(k).get("why", ""): v for k, v in self.metrics.table_publish_skipped._v.items()}
        out = {"native_server": dict(stats(), table_hook_skipped=skipped,
                                     gen_bumps=self.allocator.gen_bump_counts()
                                     if hasattr(self.allocator, "gen_bump_counts") else {},
                                     gc=dict(GC_STATS, collections=list(GC_STATS["collections"]),
                                             ns=list(GC_STATS["ns"])))}
        trace = getattr(self.allocator, "pod_trace", None)
        if trace is not None:
            out["pod_trace"] = trace()
        return out

    def _pod_resources(self):
        from ..api.podresources import SOCKET, PodResourcesClient

        path = self.cfg.pod_resources_socket
        if not path or path == "none":
            return None
        if path == "auto":
            path = SOCKET
            if not os.path.exists(path):
                log.warning("kubelet pod-resources socket %s not found: placement truth is off, so a swapped "
                            "admission of two equal-size pods leaves their IDX annotations crossed", path)
                return None
        log.info("placement truth from the kubelet pod-resources API at %s", path)
        return PodResourcesClient(path, const.RESOURCE_NAME)

    def _start_health(self):
        if self.health:
            self.health.stop()
            self.health = None
        if self.cfg.health_check and self.model is not None:
            def changed(idx, healthy, reason):
                self.metrics.device_health.set(1 if healthy else 0, gpu=str(idx))
                self._export_health()

            def sample(idx, d):
                self.metrics.hbm_used.set(d.vram_used, gpu=str(idx))

            self.health = HealthMonitor(self.smi, self.model, self.cfg.health_poll_s, on_change=changed,
                                        on_topology_change=lambda ev: self._export_topology(),
                                        on_sample=sample).start()
            st = self.health.status
            self.metrics.health_events_armed.set(st.get("events_armed", 0))
            self.metrics.health_ecc_readable.set(st.get("ecc_reads_ok", 0))
            self.metrics.health_degraded.set(0 if self.health.ready else 1)

    def _start_watchdog(self):
        """The node-side quota watchdog (quota/watchdog.py), re-pointed at the current device
        model and pod source after every rebuild."""
        from ..quota.watchdog import QuotaWatchdog

        cfg = self.cfg
        mode = self._enforcement()
        if mode == "off" or self.model is None or self.pod_source is None:
            return
        alloc = self.allocator
        if self.watchdog is None:
            self.watchdog = QuotaWatchdog(self.model, self.pod_source, self.metrics, mode,
                                          cfg.quota_watch_s, cfg.quota_slack_mib << 20,
                                          disabled=lambda: self._cgpu_disabled,
                                          view=alloc.view if alloc else None,
                                          settled=alloc.settled if alloc else None).start()
        else:
            self.watchdog.model, self.watchdog.pods, self.watchdog.mode = self.model, self.pod_source, mode

    def _start_dmem(self):
        """Kernel HBM limits (quota/dmem.py): applied before each container start and on the
        watchdog's period, so they follow re-homed placements."""
        from ..quota.dmem import DmemLimits

        cfg = self.cfg
        if cfg.dmem_limits == "off" or self.model is None or self.pod_source is None or self.allocator is None:
            return
        if self.dmem is None:
            self.dmem = DmemLimits(self.model, self.pod_source, self.metrics, cfg.cgroup_root, cfg.dmem_limits,
                                   disabled=lambda: self._cgpu_disabled)

            def loop():
                while not self._ledger_stop.wait(cfg.quota_watch_s):
                    try:
                        self.dmem.sync()
                    except Exception as e:  # noqa: BLE001 - never take the plugin down
                        log.warning("dmem limit pass failed: %s", e)
            threading.Thread(target=loop, name="dmem-limits", daemon=True).start()
        else:
            self.dmem.model, self.dmem.pods = self.model, self.pod_source
        if self.dmem.available():
            log.info("dmem cgroup controller present: shared pods get a kernel HBM limit (dmem.max) on their cgroup")
            if self.dmem.sync not in self.allocator.prestart_hooks:
                self.allocator.prestart_hooks.append(self.dmem.sync)
        else:
            self.dmem.sync()                        # logs once that it is inactive

    def _start_label_watch(self):
        """Follow the node's ``cgpu.disable.isolation`` label while the plugin runs (the
        reference reads it once, at start: ``podmanager.go:62-75``, ``server.go:43-78``)."""
        if self.cfg.label_poll_s <= 0 or self.client is None or self._label_thread is not None:
            return

        def loop():
            while not self._ledger_stop.wait(self.cfg.label_poll_s):
                try:
                    v = nodestatus.cgpu_isolation_disabled(self.client, self.cfg.node_name, quiet=True)
                except Exception as e:  # noqa: BLE001 - the next poll tries again
                    log.V(2).info("node label poll: %s", e)
                    continue
                if v != self._cgpu_disabled and self.allocator is not None:
                    log.warning("node label %s=%s: %s", const.NODE_LABEL_DISABLE_CGPU, "true" if v else "(unset)",
                                "quota isolation off, HBM brokers hold nothing" if v else "quota isolation back on")
                    self._cgpu_disabled = v
                    self.allocator.set_cgpu_disabled(v)

        self._label_thread = threading.Thread(target=loop, name="node-label-watch", daemon=True)
        self._label_thread.start()

    def _start_ledger_collector(self):
        """Export the quota shim's per-container ledgers (--ledger-dir) every ledger_scan_s and
        remove the ledger directories of containers whose pods no longer exist on this node."""
        d = self.cfg.ledger_dir
        if not d or self._ledger_thread is not None:
            return
        from ..quota import ledger as L

        # layout and permissions: quota/ledger.py (the root stays plugin-owned, 0755; each
        # container gets its own subdirectory)
        try:
            L.LedgerDir(d).prepare()
        except OSError as e:
            log.warning("cannot prepare ledger dir %s: %s", d, e)

        def loop():
            while not self._ledger_stop.wait(self.cfg.ledger_scan_s):
                try:
                    live = None
                    src = self.pod_source
                    if isinstance(src, WatchCache) and src.wait_synced(0):
                        live = {O.uid(p) for p in src.snapshot()}
                    L.collect(d, self.metrics, live)
                except Exception as e:  # noqa: BLE001
                    log.warning("ledger scan failed: %s", e)

        self._ledger_thread = threading.Thread(target=loop, name="ledger-collector", daemon=True)
        self._ledger_thread.start()

    def stop(self):
        self.events.put(("signal", signal.SIGTERM))

    def _park(self):
        log.info("parking: no usable GPU on this node (waiting for SIGTERM)")
        while True:
            kind, val = self.events.get()
            if kind == "signal" and val in (signal.SIGINT, signal.SIGTERM):
                return 0

    def run(self, install_signals: bool | None = None) -> int:
        cfg = self.cfg
        if install_signals is None:
            install_signals = threading.current_thread() is threading.main_thread()
        if install_signals:
            watch_signals(self.events)
        log.V(1).info("Loading SMI backend %s", cfg.smi_backend)
        if self.smi is None:
            try:
                self.smi = S.SMI(cfg.smi_backend)
            except Exception as e:  # noqa: BLE001
                log.warning("Failed to initialize SMI: %s", e)
                return self._park()
        if self.smi.count() == 0:
            log.V(1).info("No devices found. Waiting indefinitely.")
            return self._park()
        if self.client is None and (cfg.apiserver or cfg.kubeconfig or os.environ.get(const.ENV_KUBECONFIG)
                                    or os.environ.get("KUBERNETES_SERVICE_HOST")):
            self.client = build_client(cfg.kubeconfig, cfg.apiserver, cfg.timeout)
        if cfg.metrics_addr:
            self._metrics_srv = M.serve(self.metrics.registry, cfg.metrics_addr,
                                        lambda: self.plugin is not None and not self.plugin.stopped.is_set(),
                                        ready_fn=self.readiness, debug_fn=self._debug_view)
        os.makedirs(cfg.device_plugin_dir, exist_ok=True)
        watcher = FSWatcher(cfg.device_plugin_dir, self.events)
        log.V(1).info("Starting FS watcher (%s).", watcher.mode)
        restart = True
        rc = 0
        try:
            while True:
                if restart:
                    if self.plugin is not None:
                        self.plugin.stop()
                        self.restarts += 1
                    try:
                        self.plugin = self.build_plugin()
                    except DeviceConfigError as e:
                        # a configuration the node can never satisfy: exiting would only
                        # crash-loop the DaemonSet pod
                        log.error("cannot advertise this node: %s", e)
                        self.metrics.config_error.set(1)
                        self.plugin = None
                        return self._park()
                    except Exception as e:  # noqa: BLE001
                        log.warning("Failed to get device plugin due to %s", e)
                        return 1
                    # the topology is on the node before the kubelet advertises capacity, so a
                    # TP-aware extender never schedules against a node without it
                    self._export_topology()
                    try:
                        self.plugin.serve(self._kubelet_socket())
                    except Exception as e:  # noqa: BLE001
                        log.warning("Failed to start device plugin due to %s", e)
                        return 2
                    self._start_health()
                    self._start_label_watch()
                    self._start_ledger_collector()
                    self._start_dmem()
                    self._start_watchdog()
                    restart = False
                    if install_signals:           # the plugin owns this process
                        time_gc()
                    self.started.set()
                kind, val = self.events.get()
                if kind == "fs":
                    if val.name == self._kubelet_socket() and val.op == "create":
                        log.V(1).info("inotify: %s created, restarting.", val.name)
                        restart = True
                elif kind == "signal":
                    if val == signal.SIGHUP:
                        log.V(1).info("Received SIGHUP, restarting.")
                        restart = True
                    elif val == signal.SIGQUIT:
                        log.info("generate core dump: %s", stackdump.coredump())
                    else:
                        log.V(1).info('Received signal "%s", shutting down.', val)
                        break
        finally:
            watcher.close()
            self._ledger_stop.set()
            if self.watchdog is not None:
                self.watchdog.stop()
            if self.health:
                self.health.stop()
            if self.plugin is not None:
                self.plugin.stop()
            if self.pod_source is not None:
                self.pod_source.stop()
            if self._prebind is not None:
                self._prebind.stop()
            if self.allocator is not None:
                self.allocator.flush_patches(2.0)
                self.allocator.close()
            if self._metrics_srv is not None:
                self._metrics_srv.shutdown()
        return rc
