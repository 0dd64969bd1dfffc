"""Physical MI355X → fake "memory-unit" devices (component C2).

Reference behaviour (``nvidia.go:23-29,50-86``): every physical GPU becomes ``gpuMemory``
fake devices with IDs ``"<UUID>-_-<j>"``, all Healthy, no topology; ``gpuMemory`` is set
once from the first GPU and cached globally across plugin restarts. The kubelet only ever
counts these IDs; which IDs it picks is ignored (``allocate.go:55-57``).

Differences here:
* units are computed from *bytes* with an explicit rounding policy (utils/units.py);
* per-GPU units are computed per device; when the node is heterogeneous the advertised
  units per GPU default to the minimum across GPUs so the extender's homogeneous
  ``allocatable / gpu-count`` arithmetic never over-commits a smaller GPU;
* each fake device carries its GPU's NUMA node in ``Device.topology``;
* health is tracked per physical GPU and can recover (the reference could not:
  ``server.go:188``); indices stay stable across hot-unplug so extender ``IDX``
  annotations keep meaning the same GPU;
* partition awareness (MI355X compute partitioning, SPX/DPX/QPX/CPX x NPS1/NPS2): in a
  non-SPX mode every partition enumerates as its own HIP device and is advertised as its own
  GPU, but under NPS1 the partitions of one socket all report the socket's whole HBM. With
  ``partition_aware`` (default) such a group of same-socket partitions (same unique id, or
  same BDF) that reports identical totals is treated as sharing that HBM, and each partition
  is advertised ``total / partitions`` — without it every partition would claim the full
  288 GB and the node would be over-committed by the partition count. Partitions that report
  their own (NPS-split) memory are taken as reported. Each GPU records its socket so the
  topology export can tell partitions of one package apart from xGMI peers.
"""
from __future__ import annotations

import dataclasses
import threading

from .. import const
from ..api import v1beta1 as api
from ..utils import log, units as U
from .smi import GPU


def fake_device_id(real_id: str, j: int) -> str:
    return f"{real_id}{const.FAKE_ID_SEP}{j}"


def real_device_id(fake_id: str) -> str:
    return fake_id.split(const.FAKE_ID_SEP)[0]


@dataclasses.dataclass
class PhysicalGPU:
    index: int
    uuid: str
    vram_bytes: int
    units: int
    numa_node: int
    render_minor: int
    bdf: str
    name: str
    healthy: bool = True
    present: bool = True
    reason: str = ""
    socket: int = -1        # physical package (same-socket partitions share it)
    partition: int = 0      # partition index within the socket
    num_xcc: int = 1        # XCDs in this (partition of the) device: 8 on an SPX MI355X
    num_cu: int = 0         # active compute units (256 on an SPX MI355X)

    @property
    def render_node(self) -> str | None:
        return const.DRI_RENDER_FMT.format(minor=self.render_minor) if self.render_minor >= 0 else None


def socket_key(g: GPU) -> str:
    """Identity of the physical package a (possibly partitioned) device belongs to."""
    return f"uid:{g.unique_id:x}" if g.unique_id else f"bdf:{g.bdf}" if g.bdf else f"idx:{g.index}"


def partition_layout(gpus: list[GPU], partition_aware: bool = True) -> tuple[dict, dict, dict]:
    """Returns ``({index: socket}, {index: partition}, {index: usable bytes})``."""
    groups: dict[str, list[GPU]] = {}
    for g in gpus:
        groups.setdefault(socket_key(g), []).append(g)
    sockets, parts, vram = {}, {}, {}
    for s, (_, members) in enumerate(groups.items()):
        members = sorted(members, key=lambda g: g.index)
        shared = (partition_aware and len(members) > 1 and len({m.vram_total for m in members}) == 1
                  and all(m.memory_partition in (0, 1) for m in members))
        if shared:
            log.info("socket %s: %d compute partitions share %d bytes of HBM (NPS1); %d bytes each",
                     socket_key(members[0]), len(members), members[0].vram_total,
                     members[0].vram_total // len(members))
        for p, m in enumerate(members):
            sockets[m.index], parts[m.index] = s, p
            vram[m.index] = m.vram_total // len(members) if shared else m.vram_total
    return sockets, parts, vram


class DeviceConfigError(ValueError):
    """The node cannot be advertised under this configuration; the supervisor parks instead of
    exiting (an exit would only crash-loop the DaemonSet pod)."""


class DeviceModel:
    """Thread-safe device table; ``generation`` bumps on every health change.

    ``--memory-unit=MiB`` on an MI355X would mean 294,912 fake devices per GPU (2.36 M per
    node, a >100 MB ListAndWatch message the kubelet rejects). When the MiB count
    exceeds ``MAX_FAKE_DEVICES_PER_NODE`` the model falls back to GiB with a warning
    (``unit_fallback`` records why; the plugin exports the unit it actually advertises as a
    node annotation and a metric), the same way the reference falls back to GiB for a unit it
    cannot use (``cmd/nvidia/main.go:67-78``)."""

    def __init__(self, gpus: list[GPU], unit: str = const.GIB, round_policy: str = "nearest",
                 homogeneous: bool = True, gpu_indices: list[int] | None = None, partition_aware: bool = True):
        self.unit = unit
        self.round_policy = round_policy
        self._lock = threading.Lock()
        self._cond = threading.Condition(self._lock)
        self.generation = 0
        self.unit_fallback = ""
        sel = [g for g in gpus if gpu_indices is None or g.index in set(gpu_indices)]
        sockets, part_idx, vram = partition_layout(gpus, partition_aware)
        per = [U.units_for_bytes(vram[g.index], unit, round_policy) for g in sel]
        if sum(per) > U.MAX_FAKE_DEVICES_PER_NODE and unit == const.MIB:
            self.unit_fallback = (f"{sum(per)} MiB devices exceed the ListAndWatch limit "
                                  f"({U.MAX_FAKE_DEVICES_PER_NODE}); advertising GiB")
            log.warning("--memory-unit=MiB: %s. Pods must request aliyun.com/gpu-mem in GiB on this node.",
                        self.unit_fallback)
            unit = self.unit = const.GIB
            per = [U.units_for_bytes(vram[g.index], unit, round_policy) for g in sel]
        if homogeneous and per and len(set(per)) > 1:
            log.warning("heterogeneous GPU memory %s %s; advertising the minimum (%d) per GPU",
                        per, unit, min(per))
            per = [min(per)] * len(per)
        self.gpus: list[PhysicalGPU] = []
        for new_idx, (g, u) in enumerate(zip(sel, per)):
            self.gpus.append(PhysicalGPU(index=new_idx, uuid=g.uuid, vram_bytes=vram[g.index], units=u,
                                         numa_node=g.numa_node, render_minor=g.render_minor, bdf=g.bdf,
                                         name=g.name, healthy=g.health == 0, socket=sockets[g.index],
                                         partition=part_idx[g.index], num_xcc=max(1, g.num_xcc),
                                         num_cu=g.num_cu))
        total = sum(g.units for g in self.gpus)
        if total > U.MAX_FAKE_DEVICES_PER_NODE:
            raise DeviceConfigError(f"{total} fake devices exceed the ListAndWatch limit "
                             f"({U.MAX_FAKE_DEVICES_PER_NODE}); use --memory-unit=GiB on this node")
        self._by_uuid = {g.uuid: g for g in self.gpus}
        self._devs_cache = None
        for g in self.gpus:
            log.info("GPU %d %s %s %s: %d bytes -> %d %s", g.index, g.uuid, g.bdf, g.name, g.vram_bytes,
                     g.units, unit)

    # -- queries ------------------------------------------------------------------------
    def count(self) -> int:
        return len(self.gpus)

    def total_units(self) -> int:
        return sum(g.units for g in self.gpus)

    def units_of(self, index: int) -> int:
        return self.gpus[index].units

    def dev_units(self) -> int:
        """Per-GPU units as the extender sees them (``ALIYUN_COM_GPU_MEM_DEV``)."""
        return self.gpus[0].units if self.gpus else 0

    def gpu(self, index: int) -> PhysicalGPU | None:
        return self.gpus[index] if 0 <= index < len(self.gpus) else None

    def by_uuid(self, uuid: str) -> PhysicalGPU | None:
        return self._by_uuid.get(uuid)

    def uuid_by_index(self, index: int) -> str | None:
        """``GetDeviceNameByIndex`` (``server.go:80-91``) without the lazy racy map."""
        g = self.gpu(index)
        return g.uuid if g else None

    def fake_ids(self, index: int) -> list[str]:
        g = self.gpus[index]
        return [fake_device_id(g.uuid, j) for j in range(g.units)]

    def device_list(self) -> list:
        """Immutable snapshot of every fake device (rebuilt only when health changes)."""
        with self._lock:
            if self._devs_cache is None:
                devs = []
                for g in self.gpus:
                    health = const.HEALTHY if (g.healthy and g.present) else const.UNHEALTHY
                    topo = api.TopologyInfo(nodes=[api.NUMANode(ID=g.numa_node)]) if g.numa_node >= 0 else None
                    for j in range(g.units):
                        d = api.Device(ID=fake_device_id(g.uuid, j), health=health)
                        if topo is not None:
                            d.topology.CopyFrom(topo)
                        devs.append(d)
                self._devs_cache = devs
            return self._devs_cache

    def healthy_indices(self) -> list[int]:
        return [g.index for g in self.gpus if g.healthy and g.present]

    # -- mutation -----------------------------------------------------------------------
    def set_health(self, index: int, healthy: bool, reason: str = "", present: bool | None = None) -> bool:
        """Returns True if anything changed (and wakes ListAndWatch streams)."""
        with self._cond:
            g = self.gpus[index]
            new_present = g.present if present is None else present
            if g.healthy == healthy and g.present == new_present:
                g.reason = reason or g.reason   # e.g. an ECC mark now waiting for its reset
                return False
            g.healthy, g.present, g.reason = healthy, new_present, reason
            self._devs_cache = None
            self.generation += 1
            self._cond.notify_all()
        log.warning("GPU %d (%s) -> %s%s", index, g.uuid, "Healthy" if healthy and new_present else "Unhealthy",
                    f" ({reason})" if reason else "")
        return True

    def wait_change(self, generation: int, timeout: float) -> int:
        with self._cond:
            if self.generation == generation:
                self._cond.wait(timeout)
            return self.generation

    def notify_all(self):
        with self._cond:
            self._cond.notify_all()
