"""Where a fresh process's GPU start-up time goes: the runtime's init (the first HIP call), the rest
of torch.cuda.init, and the first memory operation (the device's lazy setup). One JSON line.

Run on the GPU box: python tools/diag/cuda_init_split.py [first-op]
first-op: malloc (default) | memset | ctx (hipSetDevice + hipDeviceSynchronize only)
"""
import ctypes
import json
import sys
import time

t0 = time.perf_counter()
import torch  # noqa: E402

t1 = time.perf_counter()
# the runtime torch loaded (PyTorch's bundled libamdhip64), not another copy on the library path
lib = next(ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln)
hip = ctypes.CDLL(lib)
n = ctypes.c_int(0)
t2 = time.perf_counter()
rc = hip.hipGetDeviceCount(ctypes.byref(n))
t3 = time.perf_counter()
torch.cuda.init()
t4 = time.perf_counter()
op = sys.argv[1] if len(sys.argv) > 1 else "malloc"
if op == "ctx":
    hip.hipSetDevice(0)
    hip.hipDeviceSynchronize()
    t5 = time.perf_counter()
    x = torch.empty(1 << 20, device="cuda")
else:
    x = torch.empty(1 << 20, device="cuda")
    if op == "memset":
        x.zero_()
    t5 = time.perf_counter()
torch.cuda.synchronize()
t6 = time.perf_counter()
y = torch.empty(1 << 20, device="cuda")
y.zero_()
torch.cuda.synchronize()
t7 = time.perf_counter()
ms = lambda a, b: round((b - a) * 1e3, 3)  # noqa: E731
print(json.dumps({"op": op, "import_torch_ms": ms(t0, t1), "hip_get_device_count_ms": ms(t2, t3), "rc": rc,
                  "devices": n.value, "torch_cuda_init_rest_ms": ms(t3, t4), "first_op_ms": ms(t4, t5),
                  "first_sync_ms": ms(t5, t6), "second_alloc_zero_sync_ms": ms(t6, t7),
                  "hip_version": torch.version.hip, "lib": lib}))
