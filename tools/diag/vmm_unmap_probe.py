"""Does HIP unmap several mappings with one hipMemUnmap over their whole range, and what does
one unmap per mapping cost? PyTorch's HIP runtime, 1 GiB physical handles, N of them mapped
back to back into one reservation. One JSON line. Run on the GPU box:
python tools/diag/vmm_unmap_probe.py [N]
"""
import ctypes
import json
import sys
import time

import torch

N = int(sys.argv[1]) if len(sys.argv) > 1 else 16
GIB = 1 << 30
torch.cuda.init()
lib = next(ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln)
hip = ctypes.CDLL(lib)
hip.hipMemAddressReserve.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_size_t,
                                     ctypes.c_void_p, ctypes.c_ulonglong]
hip.hipMemMap.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_ulonglong]
hip.hipMemUnmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
hip.hipMemAddressFree.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
hip.hipMemRelease.argtypes = [ctypes.c_void_p]


class Loc(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("id", ctypes.c_int)]


class Prop(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("requestedHandleType", ctypes.c_int), ("location", Loc),
                ("win32HandleMetaData", ctypes.c_void_p), ("allocFlags", ctypes.c_ubyte * 8)]


class Access(ctypes.Structure):
    _fields_ = [("location", Loc), ("flags", ctypes.c_int)]


prop = Prop()
prop.type = 1                      # hipMemAllocationTypePinned
prop.location = Loc(1, 0)          # hipMemLocationTypeDevice, device 0
acc = Access(Loc(1, 0), 3)         # hipMemAccessFlagsProtReadWrite
out = {"n": N}


def setup():
    hs = []
    for _ in range(N):
        h = ctypes.c_void_p()
        assert hip.hipMemCreate(ctypes.byref(h), ctypes.c_size_t(GIB), ctypes.byref(prop), ctypes.c_ulonglong(0)) == 0
        hs.append(h)
    base = ctypes.c_void_p()
    assert hip.hipMemAddressReserve(ctypes.byref(base), N * GIB, 0, None, 0) == 0
    for i, h in enumerate(hs):
        assert hip.hipMemMap(base.value + i * GIB, GIB, 0, h, 0) == 0
    assert hip.hipMemSetAccess(ctypes.c_void_p(base.value), ctypes.c_size_t(N * GIB), ctypes.byref(acc),
                               ctypes.c_size_t(1)) == 0
    torch.cuda.synchronize()
    return base.value, hs


def teardown(base, hs):
    hip.hipMemAddressFree(base, N * GIB)
    for h in hs:
        hip.hipMemRelease(h)


# A: one unmap per mapping
base, hs = setup()
t = time.perf_counter()
rcs = [hip.hipMemUnmap(base + i * GIB, GIB) for i in range(N)]
out["per_mapping_ms"] = round((time.perf_counter() - t) * 1e3, 3)
out["per_mapping_rcs"] = sorted(set(rcs))
teardown(base, hs)

# B: one unmap over the whole range, then: is each mapping gone? (mapping it again succeeds only
# where nothing is mapped; a second unmap of one mapping fails where it is gone)
base, hs = setup()
t = time.perf_counter()
out["whole_rc"] = hip.hipMemUnmap(base, N * GIB)
out["whole_ms"] = round((time.perf_counter() - t) * 1e3, 3)
again = [hip.hipMemUnmap(base + i * GIB, GIB) for i in range(N)]
out["after_whole_second_unmap_rcs"] = again          # 0 = that mapping was still there
teardown(base, hs)
print(json.dumps(out))
