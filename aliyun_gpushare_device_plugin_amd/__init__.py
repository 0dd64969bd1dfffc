"""MI355X-native GPU-sharing Kubernetes device plugin (aliyun.com/gpu-mem compatible).

Layer map (re-designed for MI355X):
  L0 device/smi.py       -> native/gpuinfo (C++: librocm_smi64 + amdgpu/KFD sysfs)
  L1 device/model.py     physical GPU -> fake memory-unit devices
  L2 cluster/            apiserver client, node status, pod watch cache, kubelet client
  L3 plugin/native_server.py -> native/dpserver (C++ HTTP/2 + gRPC: the kubelet v1beta1
                         DevicePlugin service, Allocate answered from the engine's prepared
                         table); plugin/server.py (grpcio alternative); alloc/ Allocate engine
  L4 plugin/manager.py   lifecycle (inotify, signals, restart), device/health.py
  L5 cli/main.py         flags / entry point
  L6 cli/inspect.py      kubectl-inspect-gpushare; cli/podgetter.py
  quota/ + native/hipshim    per-container HBM quota (LD_PRELOAD shim at the KFD boundary),
                             watchdog, dmem limits
  quota/hbmbroker.py + native/hbmbroker   per-GPU HBM broker (VMM granules lent to pods) and
                             the plugin's granter
  extender/ + cli/extender.py  gpushare-scheduler-extender (filter / bind, HA leader election)
  ops/ + models/           HIP/CDNA4 kernels and the PyTorch-ROCm demo workloads
  parallel/                xGMI topology export, TP-group placement, RCCL demo
  sim/                     fake apiserver / kubelet and the multi-node harness for CPU-only runs
"""
import os as _os

__version__ = "0.1.0"


def _lifeline() -> None:
    """Simulator children (``sim/cluster.py``: fake apiserver, kubelet, plugin processes) die with
    the process that started them. Armed here, after exec: in a ``preexec_fn`` (between fork and
    exec) the child imports ctypes and dlopens, and a loader or import lock another thread of the
    multi-threaded parent (gRPC pollers) held at fork time deadlocks it (seen as a plugin process
    that never registered)."""
    ppid = _os.environ.pop("GPUSHARE_DIE_WITH_PARENT", None)      # not inherited any further
    if not ppid:
        return
    import ctypes
    import signal

    ctypes.CDLL(None, use_errno=True).prctl(1, signal.SIGTERM)    # PR_SET_PDEATHSIG
    if _os.getppid() != int(ppid):                                # the parent is already gone
        _os._exit(0)


def _cpus() -> None:
    """``GPUSHARE_CPUS=3,7-8``: run this process on those CPUs (set here, before any thread
    starts, so every thread keeps it). A node's daemons on CPUs of their own — the kubelet's
    ``reservedSystemCPUs`` — keep the plugin's watch and Allocate path off the cores pod start-ups
    saturate (sim/cluster.py ``daemon_cpus``, bench.py ``--reserved-cpus``)."""
    spec = _os.environ.pop("GPUSHARE_CPUS", None)
    if not spec:
        return
    cpus = set()
    for part in spec.split(","):
        lo, _, hi = part.partition("-")
        if lo.strip():
            cpus.update(range(int(lo), int(hi or lo) + 1))
    try:
        _os.sched_setaffinity(0, cpus)
    except (OSError, ValueError):
        pass


_lifeline()
_cpus()
