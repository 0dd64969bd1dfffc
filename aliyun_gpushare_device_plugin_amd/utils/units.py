"""Memory units and the advertised-capacity math.

Reference: ``translatememoryUnits`` (``cmd/nvidia/main.go:67-78``) accepts ``GiB``/``MiB``
and warns + falls back to GiB otherwise; ``setGPUMemory`` (``nvidia.go:31-38``) divides the
NVML total by 1024 for GiB. NVML reports *bytes*, so the reference over-advertises by 1024×
(SURVEY §2.4.1). Here capacity is computed from bytes explicitly, per device, with a
documented rounding policy:

* ``floor``   — ``bytes // unit``: never advertises memory that is not there.
* ``nearest`` — ``round(bytes / unit)``: MI355X reports 309,220,868,096 B = 287.98 GiB, so
  ``floor`` gives 287 and ``nearest`` gives the nominal 288. Safe because the HIP quota shim
  enforces ``container_units / device_units × real_bytes`` (proportional), never
  ``units × 2^30``: a pod holding every unit of a GPU gets exactly the whole GPU.
"""
from __future__ import annotations

from .. import const
from . import log

ROUND_POLICIES = ("nearest", "floor")

# Above this many fake devices per node the ListAndWatch message approaches gRPC's default
# 4 MiB limit (≈60 B/device); the reference would silently fail in MiB mode on MI355X
# (SURVEY §3.2 sizing note: 8 × 294,912 MiB ≈ 2.36 M devices).
MAX_FAKE_DEVICES_PER_NODE = 60_000


def normalize_unit(value: str) -> str:
    if value in (const.GIB, const.MIB):
        return value
    log.warning("Unsupported memory unit: %s, use memoryUnit Gi as default", value)
    return const.GIB


def units_for_bytes(nbytes: int, unit: str = const.GIB, policy: str = "nearest") -> int:
    if nbytes <= 0:
        return 0
    ub = const.UNIT_BYTES[unit]
    if policy == "floor":
        return nbytes // ub
    if policy == "nearest":
        return max(1, (nbytes + ub // 2) // ub)
    raise ValueError(f"unknown rounding policy {policy!r}; expected one of {ROUND_POLICIES}")


def quota_bytes(container_units: int, device_units: int, device_bytes: int) -> int:
    """Bytes a container may allocate: its share of the *real* device memory."""
    if device_units <= 0 or container_units <= 0:
        return 0
    return min(device_bytes, device_bytes * container_units // device_units)


def parse_quantity(q) -> int:
    """Parse a Kubernetes resource quantity ("2", "64", "1k", "2Gi", "500m") to an int value.

    Extended resources such as ``aliyun.com/gpu-mem`` are integers in practice, but the API
    accepts any quantity syntax; ``Quantity.Value()`` rounds up (ceil) like Go does.
    """
    if isinstance(q, bool):
        raise ValueError("bad quantity")
    if isinstance(q, (int, float)):
        return int(-(-q // 1))
    if isinstance(q, str) and q.isdigit():      # the common case for extended resources: "64"
        return int(q)
    s = str(q).strip()
    if not s:
        return 0
    suffixes = {"Ki": 2**10, "Mi": 2**20, "Gi": 2**30, "Ti": 2**40, "Pi": 2**50, "Ei": 2**60,
                "k": 10**3, "M": 10**6, "G": 10**9, "T": 10**12, "P": 10**15, "E": 10**18, "m": None}
    for suf in ("Ki", "Mi", "Gi", "Ti", "Pi", "Ei", "k", "M", "G", "T", "P", "E", "m"):
        if s.endswith(suf):
            num = s[: -len(suf)]
            if suf == "m":
                from fractions import Fraction
                v = Fraction(num) / 1000
                return int(-(-v.numerator // v.denominator))
            from fractions import Fraction
            v = Fraction(num) * suffixes[suf]
            return int(-(-v.numerator // v.denominator))
    if "e" in s.lower():
        from fractions import Fraction
        mant, _, exp = s.lower().partition("e")
        v = Fraction(mant) * (Fraction(10) ** int(exp))
        return int(-(-v.numerator // v.denominator))
    from fractions import Fraction
    v = Fraction(s)
    return int(-(-v.numerator // v.denominator))
