"""``gpushare-device-plugin`` entry point (components C5/C12; reference ``cmd/nvidia/main.go``).

Reference flags are kept with the same names and defaults (``main.go:15-26``) so existing
DaemonSet manifests work unchanged; glog's ``-logtostderr`` and ``--v`` are accepted.
New flags select the SMI backend, rounding policy, pod source, quota shim, topology export
and metrics endpoint.
"""
from __future__ import annotations

import argparse
import os
import sys

from .. import const
from ..plugin.manager import PluginConfig, SharedGPUManager
from ..utils import log, units


def _bool(v: str) -> bool:
    return str(v).lower() in ("1", "true", "t", "yes", "y", "")


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="gpushare-device-plugin",
                                description="MI355X GPU-sharing device plugin (aliyun.com/gpu-mem)")
    # --- reference flags (cmd/nvidia/main.go:15-26) ---
    p.add_argument("--mps", nargs="?", const="true", default="false", help="accepted and ignored")
    p.add_argument("--health-check", nargs="?", const="true", default="true",
                   help="enable GPU health monitoring (SMI events + polling)")
    p.add_argument("--memory-unit", default=const.GIB, help="GiB or MiB")
    p.add_argument("--query-kubelet", nargs="?", const="true", default="false",
                   help="source pending pods from the kubelet /pods endpoint")
    p.add_argument("--kubelet-address", default="0.0.0.0")
    p.add_argument("--kubelet-port", type=int, default=10250)
    p.add_argument("--kubelet-scheme", default="https", choices=("https", "http"),
                   help="kubelet /pods scheme (http only for the read-only port or tests)")
    p.add_argument("--client-cert", default="")
    p.add_argument("--client-key", default="")
    p.add_argument("--token", default="")
    p.add_argument("--timeout", type=int, default=10, help="kubelet/apiserver HTTP timeout (s)")
    # --- glog compatibility ---
    p.add_argument("-logtostderr", "--logtostderr", nargs="?", const="true", default="true")
    p.add_argument("-v", "--v", type=int, default=int(os.environ.get("GPUSHARE_V", "0")))
    p.add_argument("--log-json", action="store_true")
    # --- MI355X additions ---
    p.add_argument("--smi-backend", default="auto", help="auto | amdsmi | rocm_smi | sysfs[:root] | fake:<N>x<SIZE> | fake:<json>")
    p.add_argument("--round", dest="round_policy", choices=units.ROUND_POLICIES, default="nearest",
                   help="bytes->units rounding (nearest advertises the nominal 288 GiB of an MI355X)")
    p.add_argument("--heterogeneous", action="store_true",
                   help="advertise each GPU's own units instead of the node minimum")
    p.add_argument("--pod-source", choices=("watch", "list", "kubelet"), default="watch")
    p.add_argument("--device-plugin-dir", default=const.DEVICE_PLUGIN_PATH)
    p.add_argument("--kubeconfig", default=None)
    p.add_argument("--apiserver", default=None, help="apiserver URL (overrides kubeconfig/in-cluster)")
    p.add_argument("--node-name", default=os.environ.get(const.ENV_NODE_NAME, ""))
    p.add_argument("--gpu-indices", default="", help="comma-separated subset of GPUs to manage")
    p.add_argument("--shim-path", default=os.environ.get("GPUSHARE_SHIM_HOST_DIR", ""),
                   help="host directory containing libgpushare_hipquota.so to inject (empty: no shim)")
    p.add_argument("--install-shim", default="",
                   help="copy the bundled libgpushare_hipquota.so into this host directory at startup and "
                        "inject it from there (DaemonSet hostPath, e.g. /var/lib/gpushare/lib)")
    p.add_argument("--strict-allocate", action="store_true",
                   help="fail Allocate with a gRPC error instead of an error-shaped response")
    p.add_argument("--preferred-allocation", action="store_true",
                   help="advertise GetPreferredAllocation: the kubelet then picks fake IDs of the GPU the "
                        "extender chose (accurate device checkpoint, one extra RPC per container)")
    p.add_argument("--partition-aware", type=_bool, nargs="?", const=True, default=True,
                   help="treat same-socket compute partitions (CPX/DPX/QPX under NPS1) as sharing the socket's "
                        "HBM and advertise each its share (default true; false = every partition reports full HBM)")
    p.add_argument("--ledger-dir", default=None,
                   help="host directory for file-backed quota-shim ledgers, mounted into every shared "
                        "container; the plugin exports per-container HBM used/peak/denials from it")
    p.add_argument("--ledger-scan-interval", type=float, default=10.0)
    p.add_argument("--hbm-broker-dir", default=None,
                   help="host directory of the per-GPU HBM brokers' sockets (hbm<index>.sock, gpushare-hbm-broker): "
                        "every shared container gets a grant of broker granules and its quota shim serves hipMalloc "
                        "from them, so admissions do not wait for amdgpu to wipe a retired pod's HBM")
    p.add_argument("--comgr-cache-dir", default=None,
                   help="host directory of the node's comgr cache (filled by the DaemonSet's init container, "
                        "gpushare-comgr-cache): mounted read-only into shared containers with AMD_COMGR_CACHE set, "
                        "so their HIP runtime loads its blit kernels instead of compiling them at the first stream")
    p.add_argument("--hbm-broker-fraction", type=float, default=0.94,
                   help="share of a container's quota granted as broker granules (whole GiB, rounded down); the "
                        "rest of the quota is borrowed from granules no grant claims, or from the driver")
    p.add_argument("--label-poll-interval", type=float, default=10.0,
                   help="re-read the node's cgpu.disable.isolation label this often while running (0 = at start "
                        "only, as the reference): a flip re-prepares answers and sizes the HBM brokers")
    p.add_argument("--journal-path", default=None,
                   help="persist recent Allocate decisions (JSON lines) so a retried admission of an "
                        "already-assigned, still-Pending pod is answered identically across plugin restarts")
    p.add_argument("--compute-isolation", default="none", choices=("none", "cu"),
                   help="cu: give every shared pod its own run of CU slots (one CU per XCD each, sized by "
                        "its HBM share) through HSA_CU_MASK / ROC_GLOBAL_CU_MASK; none: time-slice the whole GPU")
    p.add_argument("--no-swap-completion", action="store_true",
                   help="reference behaviour: fail a pod whose equal-size twin was admitted first "
                        "under its reservation instead of exchanging their GPUs")
    p.add_argument("--pod-resources-socket", default="auto",
                   help="kubelet pod-resources socket (v1.PodResourcesLister); with it the plugin requests "
                        "PreStartContainer and rewrites IDX/allocation annotations to the GPU each container "
                        "really got (swapped admissions). 'auto' = /var/lib/kubelet/pod-resources/kubelet.sock "
                        "when present; 'none' disables placement truth")
    p.add_argument("--admission-identity", type=_bool, nargs="?", const=True, default=True,
                   help="when several pending pods could own an Allocate request, ask the kubelet's "
                        "pod-resources List which pod is being admitted (it holds no IDs yet) instead of "
                        "guessing by assume time (default true; needs --pod-resources-socket)")
    p.add_argument("--cdi-kind", default="",
                   help="also answer the GPU as a CDI device '<kind>=<index>' (e.g. amd.com/gpu, the spec AMD's "
                        "container toolkit generates); empty = DeviceSpecs only")
    p.add_argument("--device-specs", type=_bool, nargs="?", const=True, default=True,
                   help="answer /dev/kfd and the GPU's render node as DeviceSpecs (false with --cdi-kind: CDI only)")
    p.add_argument("--grpc-server", default="auto", choices=("auto", "native", "python"),
                   help="DevicePlugin gRPC server: native = libgpushare_dpserver (HTTP/2 in C++, the common "
                        "Allocate answered without entering Python), python = grpcio; auto = native when it loads")
    p.add_argument("--native-fast-wait-us", type=int, default=300,
                   help="native server: how long an Allocate that finds the prepared answers one pod-cache "
                        "change behind waits for them to be rebuilt before the engine's full path answers it")
    p.add_argument("--native-spin-us", type=int, default=0,
                   help="native server: busy-poll the kubelet connection this long after a pod joined the "
                        "Pending set (keeps the answering core awake; costs a core meanwhile and, on a "
                        "small VM, can delay the kubelet itself: off by default)")
    p.add_argument("--prebind-watch", default="true",
                   help="watch pods the scheduler extender placed on this node (label gpushare.amd.com/node) "
                        "and prepare their Allocate answers before the bind reaches the node")
    p.add_argument("--quota-enforcement", default="auto", choices=("auto", "off", "report", "kill"),
                   help="node-side quota watchdog over the kernel's per-process HBM (DRM fdinfo): report "
                        "pods above their share, or also SIGKILL their largest GPU process (the shim cannot be "
                        "bypassed this way; needs hostPID). auto = kill when the kernel has no dmem limits and "
                        "the kubelet pod-resources API is available, else report; kill without pod-resources "
                        "is downgraded to report")
    p.add_argument("--dmem-limits", default="auto", choices=("auto", "off"),
                   help="kernel-enforced HBM shares: write each shared pod's share as dmem.max on its cgroup "
                        "when the kernel has the dmem cgroup controller with amdgpu VRAM regions (auto), else "
                        "rely on the shim and the watchdog")
    p.add_argument("--cgroup-root", default="/sys/fs/cgroup", help="cgroup v2 mount (dmem limits)")
    p.add_argument("--quota-watch-interval", type=float, default=10.0)
    p.add_argument("--quota-slack-mib", type=int, default=256,
                   help="HBM above a pod's share tolerated by the watchdog (runtime overhead)")
    p.add_argument("--placement-interval", type=float, default=2.0,
                   help="seconds between periodic placement-truth passes (besides PreStartContainer)")
    p.add_argument("--sync-patch", action="store_true",
                   help="PATCH ASSIGNED=true inside Allocate (reference behaviour) instead of write-behind")
    p.add_argument("--export-topology", nargs="?", const="true", default="true")
    p.add_argument("--rocr-visible-devices", action="store_true",
                   help="also set ROCR_VISIBLE_DEVICES=<uuid> in containers")
    p.add_argument("--metrics-addr", default=None, help="host:port for /metrics and /healthz")
    p.add_argument("--health-poll", type=float, default=5.0)
    return p


def config_from_args(a) -> PluginConfig:
    return PluginConfig(
        node_name=a.node_name, memory_unit=units.normalize_unit(a.memory_unit), round_policy=a.round_policy,
        homogeneous=not a.heterogeneous, health_check=_bool(a.health_check), health_poll_s=a.health_poll,
        pod_source=a.pod_source, query_kubelet=_bool(a.query_kubelet), kubelet_address=a.kubelet_address,
        kubelet_port=a.kubelet_port, kubelet_scheme=a.kubelet_scheme, client_cert=a.client_cert,
        client_key=a.client_key, token=a.token,
        timeout=float(a.timeout), smi_backend=a.smi_backend, device_plugin_dir=a.device_plugin_dir,
        kubeconfig=a.kubeconfig, apiserver=a.apiserver,
        gpu_indices=[int(x) for x in a.gpu_indices.split(",") if x.strip()] or None,
        shim_host_dir=a.shim_path or None, strict_allocate=a.strict_allocate,
        preferred_allocation=a.preferred_allocation, export_topology=_bool(a.export_topology),
        rocr_visible=a.rocr_visible_devices, metrics_addr=a.metrics_addr, mps=_bool(a.mps),
        async_patch=not a.sync_patch, complete_swaps=not a.no_swap_completion,
        partition_aware=a.partition_aware, ledger_dir=a.ledger_dir, ledger_scan_s=a.ledger_scan_interval,
        hbm_broker_dir=a.hbm_broker_dir, hbm_broker_fraction=a.hbm_broker_fraction, comgr_cache_dir=a.comgr_cache_dir, label_poll_s=a.label_poll_interval,
        journal_path=a.journal_path, compute_isolation=a.compute_isolation,
        pod_resources_socket=a.pod_resources_socket, placement_s=a.placement_interval,
        admission_identity=a.admission_identity, quota_enforcement=a.quota_enforcement,
        grpc_server=a.grpc_server, native_fast_wait_us=a.native_fast_wait_us, prebind_watch=_bool(a.prebind_watch),
        native_spin_us=a.native_spin_us,
        cdi_kind=a.cdi_kind, expose_devices=a.device_specs,
        quota_watch_s=a.quota_watch_interval, quota_slack_mib=a.quota_slack_mib,
        dmem_limits=a.dmem_limits, cgroup_root=a.cgroup_root)


def install_shim(dest_dir: str) -> str:
    """Atomically place the quota shim where containers can bind-mount it from the host."""
    import shutil
    import tempfile

    from ..utils.native import ensure_built

    from ..utils.native import NativeUnavailable

    libs = [(ensure_built("hipshim"), const.SHIM_LIB_NAME)]
    try:      # the comgr action cache goes next to it (answers preload it when the cache is mounted)
        libs.append((ensure_built("comgrcache"), const.COMGR_ACTION_LIB_NAME))
    except NativeUnavailable as e:
        log.warning("comgr action cache not installed: %s", e)
    os.makedirs(dest_dir, exist_ok=True)
    for src, name in libs:
        fd, tmp = tempfile.mkstemp(dir=dest_dir, prefix=".shim-")
        os.close(fd)
        shutil.copyfile(src, tmp)
        os.chmod(tmp, 0o755)
        os.replace(tmp, os.path.join(dest_dir, name))
    log.info("installed quota shim into %s", dest_dir)
    return dest_dir


def main(argv=None) -> int:
    a = build_parser().parse_args(argv)
    # Allocate runs on a gRPC thread while the informer thread decodes watch events of the very
    # pod being admitted: with CPython's default 5 ms GIL switch interval the handler can sit
    # behind a whole decode. A 0.25 ms interval bounds that wait (the kubelet blocks on it).
    sys.setswitchinterval(float(os.environ.get("GPUSHARE_SWITCH_INTERVAL", "0.00025")))
    log.setup(verbosity=a.v, json_lines=a.log_json, buffered=os.environ.get("GPUSHARE_LOG_UNBUFFERED") != "1")
    # SIGUSR2: every thread's stack to stderr straight from the signal handler — works even when
    # the interpreter is wedged (SIGQUIT's dump needs the main thread to run Python)
    import faulthandler
    import signal as _signal

    faulthandler.register(_signal.SIGUSR2, all_threads=True)
    log.V(1).info("Start gpushare device plugin")
    cfg = config_from_args(a)
    if a.install_shim:
        cfg.shim_host_dir = install_shim(a.install_shim)
    if not cfg.node_name:
        log.error("Please set env NODE_NAME (or --node-name)")
        return 1
    prof_path = os.environ.get("GPUSHARE_PROFILE")
    if not prof_path:
        return SharedGPUManager(cfg).run()
    # opt-in: profile every plugin thread (gRPC handlers, informer, patcher) until shutdown
    import cProfile
    import threading

    prof = cProfile.Profile()
    profs = [prof]

    def _thread_hook(*_a):   # first profile event of a new thread: swap in its own profiler
        p = cProfile.Profile()
        profs.append(p)
        p.enable()

    threading.setprofile(_thread_hook)
    prof.enable()
    try:
        return SharedGPUManager(cfg).run()
    finally:
        prof.disable()
        import pstats
        st = pstats.Stats(prof)
        for p in profs[1:]:
            p.disable()
            st.add(p)
        st.dump_stats(prof_path)


if __name__ == "__main__":
    sys.exit(main())
