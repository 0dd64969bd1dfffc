"""Compute isolation for pods sharing one MI355X: CU slots laid out symmetrically over the XCDs.

The reference leaves isolation to an external module (cGPU, toggled by the
``cgpu.disable.isolation`` node label: ``pkg/gpu/nvidia/podmanager.go:62``, ``allocate.go:125-126``) and only hands
out memory. Here memory is enforced by the HIP quota shim and, with
``--compute-isolation=cu``, compute by a queue CU mask the plugin injects.

What the hardware accepts (measured on MI355X, ``profiles/cu_mask/README.md``): in SPX mode
(8 XCDs x 32 CUs) the KFD applies a queue CU mask identically on every XCD. Bit ``b`` of the
256-bit mask is CU ``b // 8`` of XCD ``b % 8``, and a mask that does not give every XCD the
same CU set ("all of XCD 0") is silently not applied. A pod therefore cannot be pinned to
whole XCDs (CPX compute partitions do that; ``device/model.py`` handles them). What it can
get is a run of CU *slots*: slot ``s`` = CU ``s`` of every XCD = mask bits ``[8s, 8s + 8)``.
A pod holding slots ``[a, b)`` owns ``(b - a) x 8`` CUs spread evenly over all XCDs, keeps
all eight L2s and HBM paths, and no other masked pod issues work to its CUs.

Policy: a pod of ``u`` units on a GPU of ``U`` units wants ``k = clamp(floor(S * u / U), 1, S)``
slots (``S`` = CUs per XCD; floor, so pods whose memory fits the GPU also fit its slots unless
several are smaller than one slot), or the count in its ``gpushare.amd.com/cu-slots-request``
annotation. The plugin takes the best-fit free contiguous run among the slots held by the
GPU's other pods (read from their ``gpushare.amd.com/cu-slots`` annotation, so the plugin stays
stateless), falls back to the least-loaded run when the GPU's slots are oversubscribed, records
its choice on the pod in the ASSIGNED patch, and answers with

* ``HSA_CU_MASK=<dev>:<8a>-<8b-1>`` — ROCr applies it to every queue of every process in the
  container (HIP, RCCL, hipBLASLt alike);
* ``ROC_GLOBAL_CU_MASK=0x<hex>`` (only when the container sees exactly one GPU) — HIP then
  reports ``(b - a) x 8`` compute units, so grid sizing in PyTorch, hipBLASLt and the kernels
  here follows the slice instead of launching for 256 CUs.
"""
from __future__ import annotations

import dataclasses

from .. import const
from ..cluster import objects as O

POLICIES = ("none", "cu")


@dataclasses.dataclass(frozen=True)
class SlotRun:
    start: int
    count: int

    @property
    def end(self) -> int:
        return self.start + self.count

    def annotation(self) -> str:
        return f"{self.start}-{self.end - 1}"

    @staticmethod
    def parse(s: str | None) -> SlotRun | None:
        """``"a-b"`` (inclusive, cpuset style) or ``"a"``; None on anything malformed."""
        if not s:
            return None
        try:
            lo, _, hi = s.strip().partition("-")
            a, b = int(lo), int(hi) if hi else int(lo)
        except ValueError:
            return None
        return SlotRun(a, b - a + 1) if 0 <= a <= b else None


def mask_bits(run: SlotRun, num_xcc: int) -> range:
    """Queue-mask bit indices of a slot run: slot s -> bits [s * num_xcc, (s + 1) * num_xcc)."""
    return range(run.start * num_xcc, run.end * num_xcc)


def hsa_cu_mask(run: SlotRun, num_xcc: int, device: int = 0) -> str:
    bits = mask_bits(run, num_xcc)
    return f"{device}:{bits.start}-{bits.stop - 1}"


def roc_cu_mask(run: SlotRun, num_xcc: int) -> str:
    m = 0
    for b in mask_bits(run, num_xcc):
        m |= 1 << b
    return f"0x{m:x}"


def wanted_slots(pod_units: int, dev_units: int, slots: int, request: str | None = None) -> int:
    if request:
        try:
            return max(1, min(slots, int(request)))
        except ValueError:
            pass
    if dev_units <= 0:
        return slots
    return max(1, min(slots, slots * pod_units // dev_units))


def choose(held: list[SlotRun], k: int, slots: int) -> tuple[SlotRun, bool]:
    """Best-fit contiguous run of ``k`` slots given the runs other pods hold.

    Returns ``(run, exclusive)``. Exclusive runs come from the smallest free gap that fits (ties:
    lowest start) so large requests keep finding room; when no gap fits, the run with the least
    summed load (then lowest start) is shared and ``exclusive`` is False."""
    load = [0] * slots
    for r in held:
        for s in range(max(0, r.start), min(slots, r.end)):
            load[s] += 1
    gaps, s = [], 0
    while s < slots:
        if load[s]:
            s += 1
            continue
        e = s
        while e < slots and not load[e]:
            e += 1
        gaps.append((s, e - s))
        s = e
    fit = [(n, a) for a, n in gaps if n >= k]
    if fit:
        n, a = min(fit)
        return SlotRun(a, k), True
    best = min(range(slots - k + 1), key=lambda a: (sum(load[a:a + k]), a))
    return SlotRun(best, k), False


def held_runs(pods: list[dict], gpu_index: int, exclude_uid: str | None = None) -> list[SlotRun]:
    """Slot runs recorded on the live pods of one GPU (terminal pods hold nothing)."""
    out = []
    for p in pods:
        if O.uid(p) == exclude_uid or O.phase(p) in ("Succeeded", "Failed"):
            continue
        ann = O.annotations(p)
        r = SlotRun.parse(ann.get(const.POD_ANNOTATION_CU_SLOTS))
        if r is None:
            continue
        try:
            if int(ann.get(const.ENV_RESOURCE_INDEX, "-1")) != gpu_index:
                continue
        except ValueError:
            continue
        out.append(r)
    return out
