"""Node-side HBM quota watchdog: enforcement a tenant cannot opt out of.

The reference delegates the per-container share to Alibaba's kernel-level cGPU module
(``allocate.go:119-127``): every allocation path is covered and nothing inside the container
can switch it off. The quota shim (``native/hipshim``) is in-process: it sees the KFD and
render-node ioctls of every process that keeps it preloaded, but a process that drops
``LD_PRELOAD`` or issues raw syscalls is not charged. This watchdog closes that gap from
outside the container, with what the kernel itself reports:

* amdgpu's DRM fdinfo (``/proc/<pid>/fdinfo/<fd>`` of a render-node fd): ``drm-total-vram``
  (``drm-memory-vram`` on older kernels) per DRM client, ``drm-pdev`` the GPU's PCI address.
  Measured on MI355X (``tools/kfd_proc_probe.py``): it includes the buffers KFD allocated for
  the process (ROCr binds its KFD VM to a render-node file), so HIP, HSA and raw GEM use all
  show up; clients are de-duplicated by ``drm-client-id`` (dup'ed fds share one);
* the pod a process belongs to, from ``/proc/<pid>/cgroup`` (``.../pod<uid>/...`` or the
  systemd ``...-pod<uid_with_underscores>.slice`` form) — the DaemonSet runs with ``hostPID``;
* the pod's share per GPU, from its (truthful, ``alloc/placement.py``) placement annotations.

Every ``period_s`` the watchdog sums each pod's HBM per GPU and compares it with its share
plus ``slack_bytes`` (runtime overhead the quota does not model). A violation is exported
(``gpushare_quota_violation_bytes{pod_uid,gpu}``), logged, and — with ``mode="kill"`` — ended
the way the kernel ends a cgroup over its memory limit: the pod's largest GPU process on that
GPU is SIGKILLed, then the next, until the pod is back within its share. ``mode="report"``
only reports. Processes on a GPU that belong to no pod are exported as
``gpushare_unaccounted_hbm_bytes{gpu}``.

Kill mode acts only on a settled placement, so a pod that stays within its real share is never
killed for a stale annotation: the pods are read through the allocator's view (placement
fixes queued but not landed yet, ``view``), a pod whose answer or placement patch is still in
flight is reported but not killed (``settled``), and a violation must be seen on
``confirm_scans`` consecutive scans (the placement pass runs every 2 s while answers are in
flight, the watchdog every 10 s) before the first SIGKILL.
"""
from __future__ import annotations

import dataclasses
import os
import re
import signal
import threading

from ..alloc import placement as PL
from ..cluster import objects as O
from ..utils import log, units as U

_UNITS = {"": 1, "B": 1, "KiB": 1 << 10, "MiB": 1 << 20, "GiB": 1 << 30}
_POD_RE = re.compile(r"pod([0-9a-fA-F]{8}[-_][0-9a-fA-F]{4}[-_][0-9a-fA-F]{4}[-_][0-9a-fA-F]{4}[-_][0-9a-fA-F]{12})")


def _bytes(v: str) -> int:
    parts = v.split()
    try:
        return int(parts[0]) * _UNITS.get(parts[1] if len(parts) > 1 else "", 1)
    except (ValueError, IndexError):
        return 0


def drm_usage(pid: int, proc: str = "/proc") -> dict[str, tuple[int, str]]:
    """HBM a process holds per DRM client: {client id: (bytes, pci address)} (amdgpu only)."""
    base = f"{proc}/{pid}/fdinfo"
    out: dict[str, tuple[int, str]] = {}
    try:
        fds = os.listdir(base)
    except OSError:
        return out
    for fd in fds:
        try:
            with open(f"{base}/{fd}") as f:
                text = f.read()
        except OSError:
            continue
        if "drm-driver:" not in text:
            continue
        kv = {}
        for ln in text.splitlines():
            k, _, v = ln.partition(":")
            if k.startswith("drm-"):
                kv[k] = v.strip()
        if kv.get("drm-driver") != "amdgpu":
            continue
        cid = kv.get("drm-client-id", f"fd{fd}")
        vram = kv.get("drm-total-vram") or kv.get("drm-memory-vram") or "0"
        out[cid] = (_bytes(vram), kv.get("drm-pdev", ""))
    return out


def pod_of_pid(pid: int, proc: str = "/proc") -> str | None:
    """Kubernetes pod UID of a process, from its cgroup path (cgroupfs or systemd driver)."""
    try:
        with open(f"{proc}/{pid}/cgroup") as f:
            text = f.read()
    except OSError:
        return None
    m = _POD_RE.search(text)
    return m.group(1).replace("_", "-") if m else None


def gpu_pids(proc: str = "/proc", kfd_proc: str = "/sys/class/kfd/kfd/proc") -> set[int]:
    """Processes that may hold HBM: those KFD knows (``kfd_proc``) plus those with a render
    node open (a ``/proc`` scan of fd links)."""
    pids: set[int] = set()
    try:
        pids.update(int(p) for p in os.listdir(kfd_proc) if p.isdigit())
    except OSError:
        pass
    try:
        entries = [p for p in os.listdir(proc) if p.isdigit()]
    except OSError:
        return pids
    for p in entries:
        d = f"{proc}/{p}/fd"
        try:
            for fd in os.listdir(d):
                try:
                    if os.readlink(f"{d}/{fd}").startswith("/dev/dri/renderD"):
                        pids.add(int(p))
                        break
                except OSError:
                    continue
        except OSError:
            continue
    return pids


@dataclasses.dataclass
class Violation:
    pod_uid: str
    pod: str
    gpu: int
    used: int
    allowed: int
    pids: list                 # (pid, bytes) on that GPU, largest first
    killed: list = dataclasses.field(default_factory=list)


class QuotaWatchdog:
    def __init__(self, model, pods, metrics=None, mode: str = "report", period_s: float = 10.0,
                 slack_bytes: int = 256 << 20, proc: str = "/proc", kfd_proc: str = "/sys/class/kfd/kfd/proc",
                 pid_pod=None, pids=None, disabled=lambda: False, view=None, settled=None,
                 confirm_scans: int = 2):
        """``pods``: a PodSource (this node's pods). ``pid_pod`` / ``pids`` override the
        cgroup lookup / process discovery (tests, the simulator). ``view(pods)`` /
        ``settled(uid)``: the allocator's annotation overlay and in-flight test (see above)."""
        if mode not in ("off", "report", "kill"):
            raise ValueError(f"quota enforcement mode {mode!r}")
        self.model, self.pods, self.metrics = model, pods, metrics
        self.mode, self.period_s, self.slack = mode, period_s, slack_bytes
        self.proc, self.kfd_proc = proc, kfd_proc
        self.pid_pod = pid_pod or (lambda pid: pod_of_pid(pid, self.proc))
        self.pids = pids or (lambda: gpu_pids(self.proc, self.kfd_proc))
        self.disabled = disabled          # node label cgpu.disable.isolation=true
        self.view = view or (lambda pods: pods)
        self.settled = settled or (lambda uid: True)
        self.confirm_scans = max(1, confirm_scans)
        self._strikes: dict[tuple[str, int], int] = {}   # (pod uid, gpu) -> consecutive violating scans
        self.violations_total = 0
        self._stop = threading.Event()
        self._thread = None

    def _gpu_of_bdf(self) -> dict[str, int]:
        return {g.bdf.lower(): g.index for g in self.model.gpus if getattr(g, "bdf", "")}

    def allowed(self, pod: dict) -> dict[int, int]:
        """Bytes per GPU index the pod may hold: its units there, as the shim computes it."""
        out = {}
        for gi, units in PL.annotated_usage(pod).items():
            g = self.model.gpu(gi)
            if g is not None:
                out[gi] = U.quota_bytes(units, g.units, g.vram_bytes)
        return out

    def scan(self) -> list[Violation]:
        if self.mode == "off" or self.disabled():
            return []
        by_bdf = self._gpu_of_bdf()
        pods = {O.uid(p): p for p in self.view(self.pods.node_pods())}
        usage: dict[tuple[str, int], list] = {}
        unaccounted: dict[int, int] = {}
        seen: set[str] = set()           # a DRM client inherited across fork is counted once
        for pid in sorted(self.pids()):
            per_gpu: dict[int, int] = {}
            for cid, (nbytes, bdf) in drm_usage(pid, self.proc).items():
                if cid in seen:
                    continue
                seen.add(cid)
                gi = by_bdf.get(bdf.lower(), 0 if self.model.count() == 1 else -1)
                if gi >= 0 and nbytes:
                    per_gpu[gi] = per_gpu.get(gi, 0) + nbytes
            if not per_gpu:
                continue
            uid = self.pid_pod(pid)
            for gi, n in per_gpu.items():
                if uid in pods:
                    usage.setdefault((uid, gi), []).append((pid, n))
                else:
                    unaccounted[gi] = unaccounted.get(gi, 0) + n
        out = []
        if self.metrics is not None:
            self.metrics.quota_violation.clear()
            self.metrics.pod_hbm_used.clear()
            for (uid, gi), procs in usage.items():
                self.metrics.pod_hbm_used.set(sum(n for _, n in procs), pod_uid=uid, gpu=str(gi))
            for g in self.model.gpus:
                self.metrics.unaccounted_hbm.set(unaccounted.get(g.index, 0), gpu=str(g.index))
        strikes: dict[tuple[str, int], int] = {}
        for (uid, gi), procs in usage.items():
            pod = pods[uid]
            if O.gpu_mem_of_pod(pod) <= 0:
                continue                  # not a shared pod: whole-GPU or foreign workloads
            allowed = self.allowed(pod).get(gi, 0)
            used = sum(n for _, n in procs)
            if used <= allowed + self.slack:
                continue
            procs.sort(key=lambda x: -x[1])
            v = Violation(uid, O.name(pod), gi, used, allowed, procs)
            self.violations_total += 1
            strikes[(uid, gi)] = n_seen = self._strikes.get((uid, gi), 0) + 1
            if self.metrics is not None:
                self.metrics.quota_violation.set(used - allowed, pod_uid=uid, gpu=str(gi))
                self.metrics.quota_violations_total.inc()
            act = self.mode == "kill" and n_seen >= self.confirm_scans and self.settled(uid)
            log.warning("quota violation: pod %s/%s holds %.2f GiB on GPU %d, its share is %.2f GiB (%s)",
                        O.namespace(pod), O.name(pod), used / (1 << 30), gi, allowed / (1 << 30),
                        "killing its largest process" if act else
                        "report only" if self.mode != "kill" else
                        f"seen {n_seen}/{self.confirm_scans} scans" if self.settled(uid) else "placement in flight")
            if act:
                left = used
                for pid, n in procs:
                    if left <= allowed + self.slack:
                        break
                    try:
                        os.kill(pid, signal.SIGKILL)
                        v.killed.append(pid)
                        left -= n
                        if self.metrics is not None:
                            self.metrics.quota_kills.inc()
                    except OSError as e:
                        log.warning("quota enforcement: cannot kill pid %d: %s", pid, e)
            out.append(v)
        self._strikes = strikes
        return out

    def start(self) -> "QuotaWatchdog":
        if self.mode == "off" or self._thread is not None:
            return self

        def loop():
            while not self._stop.wait(self.period_s):
                try:
                    self.scan()
                except Exception as e:  # noqa: BLE001 - never take the plugin down
                    log.warning("quota watchdog scan failed: %s", e)
        self._thread = threading.Thread(target=loop, name="quota-watchdog", daemon=True)
        self._thread.start()
        return self

    def stop(self):
        self._stop.set()
