#!/usr/bin/env python3
"""Quota-shim granule probe on a real MI355X (run it under rocprofv3 --memory-allocation-trace).

For each requested size it calls hipMalloc through the shim (libgpushare_hipquota.so, loaded
with ctypes in front of /opt/rocm's libamdhip64) and records three views of the same
allocation:
  * ``device_bytes``  — how much the runtime's free HBM dropped (hipMemGetInfo, real runtime),
  * ``shim_charge``   — what the shim's ledger charged against the container quota,
  * the rocprofv3 memory-allocation trace row (collected by the profiler, joined afterwards).
The shim is correct when ``shim_charge == device_bytes`` for every size: CDNA4's 2 MiB
allocation granule is what a container really consumes, so quotas are enforced in the same
currency the GPU spends. Then it shows the over-quota denial. Prints one JSON document.
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MIB = 1 << 20


def main():
    quota = int(os.environ.get("PROBE_QUOTA", str(64 * MIB)))
    os.environ.setdefault("GPUSHARE_QUOTA_BYTES", str(quota))
    hip = ctypes.CDLL(os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib", "libamdhip64.so"),
                      mode=ctypes.RTLD_GLOBAL)
    shim = ctypes.CDLL(os.path.join(ROOT, "aliyun_gpushare_device_plugin_amd", "_native", "libgpushare_hipquota.so"))
    for lib in (hip, shim):
        lib.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
        lib.hipFree.argtypes = [ctypes.c_void_p]
        lib.hipMemGetInfo.argtypes = [ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t)]
    shim.gpushare_shim_stats.argtypes = [ctypes.POINTER(ctypes.c_uint64)] * 4
    shim.gpushare_shim_granule.restype = ctypes.c_uint64

    def real_free():
        f, t = ctypes.c_size_t(), ctypes.c_size_t()
        assert hip.hipMemGetInfo(ctypes.byref(f), ctypes.byref(t)) == 0
        return f.value, t.value

    def shim_used():
        u, q, d, p = (ctypes.c_uint64() for _ in range(4))
        shim.gpushare_shim_stats(ctypes.byref(u), ctypes.byref(q), ctypes.byref(d), ctypes.byref(p))
        return u.value, q.value, d.value

    # warm the runtime (first hipMalloc creates pools) so deltas measure only the probe sizes
    p0 = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(p0), 1) == 0
    hip.hipFree(p0)

    rows = []
    for size in (1, 4096, 65536, 2 * MIB - 1, 2 * MIB, 2 * MIB + 1, 3 * MIB, 6 * MIB + 4096):
        f0, _ = real_free()
        u0, _, _ = shim_used()
        p = ctypes.c_void_p()
        rc = shim.hipMalloc(ctypes.byref(p), size)
        f1, _ = real_free()
        u1, _, _ = shim_used()
        rows.append({"requested": size, "rc": rc, "device_bytes": f0 - f1, "shim_charge": u1 - u0,
                     "ptr": hex(p.value or 0)})
        shim.hipFree(p)
    # over-quota: the shim refuses before the runtime is asked
    big = ctypes.c_void_p()
    rc_over = shim.hipMalloc(ctypes.byref(big), quota + MIB)
    used, q, denied = shim_used()
    free_shim, tot_shim = ctypes.c_size_t(), ctypes.c_size_t()
    shim.hipMemGetInfo(ctypes.byref(free_shim), ctypes.byref(tot_shim))
    out = {"granule": shim.gpushare_shim_granule(), "quota": q, "rows": rows,
           "over_quota": {"requested": quota + MIB, "rc": rc_over, "denied": denied},
           "container_view": {"total": tot_shim.value, "free": free_shim.value},
           "device_total": real_free()[1],
           "consistent": all(r["rc"] == 0 and r["shim_charge"] == r["device_bytes"] for r in rows)}
    print(json.dumps(out, indent=1))
    return 0 if out["consistent"] and rc_over == 2 else 1


if __name__ == "__main__":
    sys.exit(main())
