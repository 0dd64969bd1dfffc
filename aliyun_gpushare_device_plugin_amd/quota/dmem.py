"""Kernel-enforced HBM limits through the cgroup v2 device-memory controller (``dmem``), where the
node's kernel has it.

The reference hands the per-container share to Alibaba's cGPU kernel module
(``pkg/gpu/nvidia/allocate.go:119-127``): the limit lives in the kernel, so nothing inside the
container can lift it. Upstream Linux has a kernel-side equivalent for device memory since 6.14:
the ``dmem`` cgroup controller. A DRM driver registers its VRAM as a region (listed at the cgroup
root in ``dmem.capacity`` as ``drm/<pci address>/<name> <bytes>``); ``dmem.max`` of a cgroup caps
what the processes under it may allocate in each region, and TTM refuses allocations beyond it.

This module applies each shared pod's HBM share as ``dmem.max`` on the pod's cgroup:

* the share per GPU comes from the pod's (truthful, ``alloc/placement.py``) placement annotations,
  converted exactly as the quota shim and the watchdog convert units to bytes (``units.quota_bytes``);
  the pod's other regions are left at the kernel default (``max``; the device cgroup already keeps
  it off GPUs it was not given, and a pod may hold whole GPUs from another plugin), and a region
  whose share moved away with a re-homed placement goes back to ``max``;
* the pod's cgroup is found under the kubelet's hierarchy (cgroupfs ``kubepods/<qos>/pod<uid>`` or
  systemd ``kubepods-<qos>-pod<uid_with_underscores>.slice``); the controller is switched on down
  the path (``+dmem`` in every ancestor's ``cgroup.subtree_control``), which the kubelet does not
  do for a controller it does not know;
* it runs when a container is about to start (``PreStartContainer``: the pod cgroup exists by then)
  and on the watchdog's period, so limits follow re-homed placements.

Where the kernel has no ``dmem`` controller, or the GPU driver registers no VRAM region for a GPU of
this node, it is inactive and says so once; the shim (in-process) and the watchdog (DRM fdinfo,
report/kill) remain the enforcement. ``mode``: ``auto`` (apply when available) or ``off``.
"""
from __future__ import annotations

import os
import re
import threading

from ..alloc import placement as PL
from ..cluster import objects as O
from ..utils import log, units as U


def _read(path: str) -> str:
    try:
        with open(path) as f:
            return f.read()
    except OSError:
        return ""


class DmemLimits:
    def __init__(self, model, pods, metrics=None, cgroup_root: str = "/sys/fs/cgroup", mode: str = "auto",
                 disabled=lambda: False):
        if mode not in ("auto", "off"):
            raise ValueError(f"dmem limit mode {mode!r}")
        self.model, self.pods, self.metrics = model, pods, metrics
        self.root, self.mode, self.disabled = cgroup_root, mode, disabled
        self.applied: dict[str, dict[str, int]] = {}      # pod uid -> {region: bytes} last written
        self._mu = threading.Lock()
        self._said = False

    # ---- what the kernel offers -----------------------------------------------------------------
    def controller_present(self) -> bool:
        return "dmem" in _read(os.path.join(self.root, "cgroup.controllers")).split()

    def regions(self) -> dict[int, str]:
        """GPU index -> its VRAM region name (``dmem.capacity`` at the cgroup root)."""
        names = [ln.split()[0] for ln in _read(os.path.join(self.root, "dmem.capacity")).splitlines() if ln.split()]
        out = {}
        for g in self.model.gpus:
            bdf = (getattr(g, "bdf", "") or "").lower()
            if not bdf:
                continue
            cand = [n for n in names if n.startswith("drm/") and f"/{bdf}/" in n.lower() and "vram" in n.lower()]
            if cand:
                out[g.index] = sorted(cand)[0]
        return out

    def available(self) -> bool:
        return self.mode != "off" and self.controller_present() and bool(self.regions())

    # ---- where a pod lives ------------------------------------------------------------------------
    def pod_cgroup(self, uid: str) -> str | None:
        """The pod-level cgroup directory of ``uid`` under the kubelet's hierarchy, or None."""
        pats = (re.compile(rf"^pod{re.escape(uid)}$"),
                re.compile(rf"^kubepods(-[a-z]+)?-pod{re.escape(uid.replace('-', '_'))}\.slice$"))
        frontier = [os.path.join(self.root, d) for d in ("kubepods.slice", "kubepods")
                    if os.path.isdir(os.path.join(self.root, d))]
        for _ in range(3):                                 # kubepods / <qos> / pod<uid>
            nxt = []
            for d in frontier:
                try:
                    entries = os.listdir(d)
                except OSError:
                    continue
                for e in entries:
                    p = os.path.join(d, e)
                    if not os.path.isdir(p):
                        continue
                    if any(r.match(e) for r in pats):
                        return p
                    nxt.append(p)
            frontier = nxt
        return None

    def _enable_down_to(self, path: str) -> None:
        """``+dmem`` in the subtree_control of every ancestor of ``path`` (root included)."""
        rel = os.path.relpath(path, self.root)
        cur = self.root
        for part in [""] + rel.split(os.sep)[:-1]:
            cur = os.path.join(cur, part) if part else cur
            ctl = os.path.join(cur, "cgroup.subtree_control")
            if "dmem" not in _read(ctl).split():
                with open(ctl, "w") as f:
                    f.write("+dmem")

    # ---- the limits -------------------------------------------------------------------------------
    def limits_for(self, pod: dict, regions: dict[int, str]) -> dict[str, int]:
        """Region -> bytes the pod may hold, for the GPUs it is placed on."""
        out = {}
        for gi, units in PL.annotated_usage(pod).items():
            g = self.model.gpu(gi)
            if g is not None and gi in regions:
                out[regions[gi]] = U.quota_bytes(units, g.units, g.vram_bytes)
        return out

    def apply(self, pod: dict, regions: dict[int, str] | None = None) -> bool:
        """Write the pod's limits to its cgroup's ``dmem.max`` (only what changed). False when the
        pod has no placement yet, no cgroup on this node, or the write is refused."""
        regions = self.regions() if regions is None else regions
        uid = O.uid(pod)
        if not regions or not PL.annotated_usage(pod):
            return False
        want = self.limits_for(pod, regions)
        if not want:
            return False
        with self._mu:
            before = self.applied.get(uid, {})
            if before == want:
                return True
            cg = self.pod_cgroup(uid)
            if cg is None:
                return False
            lines = [f"{name} {nbytes}" for name, nbytes in sorted(want.items())]
            lines += [f"{name} max" for name in sorted(before) if name not in want]    # share moved away
            try:
                self._enable_down_to(cg)
                with open(os.path.join(cg, "dmem.max"), "w") as f:    # one "region limit" line each
                    f.write("\n".join(lines) + "\n")
            except OSError as e:
                log.warning("dmem limit for pod %s/%s not applied: %s", O.namespace(pod), O.name(pod), e)
                return False
            self.applied[uid] = want
        log.V(2).info("dmem.max of pod %s/%s: %s", O.namespace(pod), O.name(pod), want)
        return True

    def sync(self) -> int:
        """Apply every live shared pod's limits; forget pods that are gone. Returns pods limited."""
        if self.mode == "off" or self.disabled():
            return 0
        if not self.available():
            if not self._said:
                log.info("dmem cgroup controller with amdgpu VRAM regions not available on this node: HBM shares "
                         "are enforced by the quota shim and the watchdog only")
                self._said = True
            return 0
        regions = self.regions()
        live = [p for p in self.pods.node_pods()
                if O.gpu_mem_of_pod(p) > 0 and not O.deleting(p) and not O.is_terminated(p)]
        n = sum(1 for p in live if self.apply(p, regions))
        uids = {O.uid(p) for p in live}
        with self._mu:
            for u in [u for u in self.applied if u not in uids]:
                del self.applied[u]
        if self.metrics is not None:
            self.metrics.dmem_limited_pods.set(n)
        return n
