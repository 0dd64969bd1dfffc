"""What a fresh process's first GPU work pays for, step by step: the runtime's own memset
(its blit kernel, no PyTorch code object), then a PyTorch elementwise kernel, then a GEMM.
Markers go to stderr, so they interleave with the runtime's own log (AMD_LOG_LEVEL).
One JSON line on stdout. Run on the GPU box: python tools/diag/first_kernel_split.py
"""
import ctypes
import json
import os
import time

import torch

lib = next(ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln)
hip = ctypes.CDLL(lib)
out, last = {}, [time.perf_counter()]


def mark(name):
    t = time.perf_counter()
    out[name] = round((t - last[0]) * 1e3, 3)
    last[0] = t
    os.write(2, f"=== MARK {name} {out[name]} ms\n".encode())


n = ctypes.c_int(0)
hip.hipGetDeviceCount(ctypes.byref(n))
mark("runtime_init")
hip.hipSetDevice(0)
mark("set_device")
p = ctypes.c_void_p()
assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(64 << 20)) == 0
mark("hip_malloc")
s = ctypes.c_void_p()
assert hip.hipStreamCreate(ctypes.byref(s)) == 0
mark("stream_create")
assert hip.hipMemsetAsync(p, 0, ctypes.c_size_t(64 << 20), s) == 0
mark("memset_enqueue")
assert hip.hipStreamSynchronize(s) == 0
mark("memset_sync")
assert hip.hipMemsetAsync(p, 0, ctypes.c_size_t(64 << 20), None) == 0
assert hip.hipStreamSynchronize(None) == 0
mark("memset_null_stream")
x = torch.empty(1 << 20, device="cuda")
x.zero_()
torch.cuda.synchronize()
mark("torch_first_kernel")
x.add_(1)
torch.cuda.synchronize()
mark("torch_second_kernel")
a = torch.randn(1024, 1024, device="cuda", dtype=torch.bfloat16)
(a @ a).sum().item()
mark("torch_first_gemm")
hip.hipFree(p)
out["env"] = {k: v for k, v in os.environ.items() if k.startswith(("HIP_", "HSA_", "GPU_", "AMD_", "ROC"))}
print(json.dumps(out))
