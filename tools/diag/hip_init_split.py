"""Where a pod's HIP runtime start-up (torch.cuda.init: ~60-70 ms alone on MI355X) goes: ROCr's
hsa_init against the runtime's own device set-up, in the library set PyTorch bundles (the pods'
runtime). One JSON line per run; run on the GPU box:
    python tools/diag/hip_init_split.py [ENV=VALUE ...]
Each ENV=VALUE is set before anything loads (a knob to compare)."""
import ctypes
import glob
import json
import os
import sys
import time

for kv in sys.argv[1:]:
    k, v = kv.split("=", 1)
    os.environ[k] = v
t_imp = time.perf_counter()
import torch  # noqa: E402  (the pods' runtime: torch's bundled libamdhip64 / libhsa-runtime64)

out = {"torch_import_ms": round((time.perf_counter() - t_imp) * 1e3, 1), "env": sys.argv[1:]}
lib = os.path.join(os.path.dirname(torch.__file__), "lib")
hsa_path = (glob.glob(os.path.join(lib, "libhsa-runtime64.so*")) or ["libhsa-runtime64.so.1"])[0]
t = time.perf_counter()
hsa = ctypes.CDLL(hsa_path)
out["hsa_dlopen_ms"] = round((time.perf_counter() - t) * 1e3, 2)
prof = os.environ.get("GS_WALLPROF")     # sample what hsa_init's thread is doing (syscall or user)
samples: list = []
if prof:
    import threading

    tid = threading.get_native_id()
    stop = threading.Event()

    def sampler():
        path = f"/proc/self/task/{tid}/syscall"
        while not stop.is_set():
            try:
                with open(path) as f:
                    samples.append((time.perf_counter(), f.read().split()[:3]))
            except OSError:
                pass
            time.sleep(0.0001)

    th = threading.Thread(target=sampler, daemon=True)
    th.start()
    time.sleep(0.01)
import resource  # noqa: E402

r0 = resource.getrusage(resource.RUSAGE_THREAD)
t = time.perf_counter()
rc = hsa.hsa_init()
t_end = time.perf_counter()
r1 = resource.getrusage(resource.RUSAGE_THREAD)
out["hsa_init_ms"] = round((t_end - t) * 1e3, 2)
out["hsa_init_user_ms"] = round((r1.ru_utime - r0.ru_utime) * 1e3, 2)
out["hsa_init_sys_ms"] = round((r1.ru_stime - r0.ru_stime) * 1e3, 2)
out["hsa_init_minflt"] = r1.ru_minflt - r0.ru_minflt
if prof:
    stop.set()
    th.join()
    # syscall numbers (x86-64): 16 ioctl, 0 read, 257 openat, 9 mmap, 11 munmap, 3 close, 202 futex
    names = {"16": "ioctl", "0": "read", "257": "openat", "9": "mmap", "11": "munmap", "3": "close",
             "202": "futex", "10": "mprotect", "4": "stat", "5": "fstat", "262": "newfstatat", "17": "pread64",
             "89": "readlink", "217": "getdents64", "8": "lseek", "7": "poll", "1": "write"}
    hist: dict = {}
    n = 0
    for ts, f in samples:
        if not (t <= ts <= t_end) or not f:
            continue
        n += 1
        if f[0] == "running":
            k = "user"
        else:
            k = names.get(f[0], "sys" + f[0])
            if k == "ioctl" and len(f) > 2:
                k += " " + f[2]
        hist[k] = hist.get(k, 0) + 1
    out["samples"] = n
    out["where_pct"] = {k: round(100.0 * v / max(1, n), 1) for k, v in sorted(hist.items(), key=lambda x: -x[1])}
    with open(prof, "w") as fo:
        json.dump(out["where_pct"], fo)
hip_path = next(ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln)
hip = ctypes.CDLL(hip_path)
n = ctypes.c_int(0)
t = time.perf_counter()
hip.hipGetDeviceCount(ctypes.byref(n))
out["hip_device_count_ms"] = round((time.perf_counter() - t) * 1e3, 2)
t = time.perf_counter()
torch.cuda.init()
out["torch_cuda_init_rest_ms"] = round((time.perf_counter() - t) * 1e3, 2)
out["devices"] = n.value
out["kfd_nodes"] = len(glob.glob("/sys/class/kfd/kfd/topology/nodes/*"))
out["hsa_lib"] = hsa_path
print(json.dumps(out))
