"""Which part of a retiring ROCm process's teardown slows the next process's runtime start-up.

A tenant (torch, 6 GiB, GEMMs) ends in one of several ways; a starter that already imported
torch then times ``torch.cuda.init()`` and its first allocation. ``--when reaped``: the starter
goes once the tenant was reaped (the kubelet's order); ``--when ack``: as soon as the tenant says
it is leaving (the bench's cooperative stop). One JSON line per trial.

    python tools/diag/exit_overlap_modes.py --trials 3
"""
import argparse
import json
import subprocess
import sys
import time

TENANT = r"""
import ctypes, json, os, sys
if os.environ.get("GS_CPU"): os.sched_setaffinity(0, {int(os.environ["GS_CPU"])})
import torch
kind = os.environ.get("GS_TENANT", "full")     # what the tenant did with the GPU before it leaves
if kind == "initonly":
    torch.cuda.init()
elif kind == "small":
    x = torch.ones(1 << 20, device="cuda"); x.add_(1); torch.cuda.synchronize()
else:
    x = torch.full((6 << 30,), 7, dtype=torch.uint8, device="cuda")
    y = torch.randn(4096, 4096, device="cuda")
    for _ in range(20):
        y = y @ y.T / 4096.0
    torch.cuda.synchronize()
print(json.dumps({"ready": True}), flush=True)
mode = sys.stdin.readline().strip()
if mode in ("free", "reset") and kind == "full":
    del x, y
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
if mode == "reset":
    lib = next(ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln)
    ctypes.CDLL(lib).hipDeviceReset()
if mode in ("shimfast", "shimfastall"):   # the quota shim's fast exit: queues (and buffers) freed here
    torch.cuda.synchronize()
    ctypes.CDLL(None).gpushare_shim_fast_exit_release()
print(json.dumps({"leaving": True}), flush=True)
os._exit(0)
"""

STARTER = r"""
import json, os, sys, threading, time
if os.environ.get("GS_CPU"): os.sched_setaffinity(0, {int(x) for x in os.environ["GS_CPU"].split(",")})
import torch
NAMES = {"16": "ioctl", "0": "read", "257": "openat", "9": "mmap", "11": "munmap", "3": "close", "202": "futex",
         "10": "mprotect", "262": "newfstatat", "17": "pread64", "89": "readlink", "217": "getdents64", "7": "poll"}
tid = threading.get_native_id()
samples, stop = [], threading.Event()
def sampler():                     # what the starting thread is doing, every 100 us: on a CPU or in a syscall
    path = f"/proc/self/task/{tid}/syscall"
    while not stop.is_set():
        try:
            with open(path) as f:
                samples.append(f.read().split()[:3])
        except OSError:
            pass
        time.sleep(0.0001)
sys.stdout.write("go\n"); sys.stdout.flush()
sys.stdin.readline()
import resource
def cg():                          # the job's cgroup CPU accounting (throttling under a CPU quota)
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            return {k: int(v) for k, v in (ln.split() for ln in f)}
    except OSError:
        return {}
def cpustat():                     # system-wide jiffies: irq, softirq, steal (a VM's host takes the vCPUs)
    with open("/proc/stat") as f:
        v = [int(x) for x in f.readline().split()[1:]]
    return {"user": v[0], "system": v[2], "idle": v[3], "iowait": v[4], "irq": v[5], "softirq": v[6], "steal": v[7]}
th = threading.Thread(target=sampler, daemon=True); th.start()
s0 = cpustat()
c0, r0 = cg(), resource.getrusage(resource.RUSAGE_THREAD)
# ROCr's hsa_init through ctypes (the interpreter lock is released, so the sampler runs during it;
# torch.cuda.init() keeps the lock), then the rest of torch.cuda.init()
import ctypes, glob
hsa = ctypes.CDLL((glob.glob(os.path.join(os.path.dirname(torch.__file__), "lib", "libhsa-runtime64.so*")) or ["libhsa-runtime64.so.1"])[0])
t2 = time.perf_counter()
hsa.hsa_init()
t_hsa = time.perf_counter()
torch.cuda.init()
t3 = time.perf_counter()
c1, r1 = cg(), resource.getrusage(resource.RUSAGE_THREAD)
s1 = cpustat()
stop.set(); th.join()
where = {}
for f in samples:
    if f and f[0] == "257" and len(f) > 2:          # openat: the path, read from this process's memory
        try:
            f = ["257", "", ctypes.string_at(int(f[2], 16), 120).split(b"\0")[0].decode(errors="replace")]
        except (ValueError, OSError):
            pass
    k = "runnable" if f and f[0] == "running" else (NAMES.get(f[0], "sys" + f[0]) + (" " + f[2] if f[0] in ("16", "257") and len(f) > 2 else "")) if f else "?"
    where[k] = where.get(k, 0) + 1
z = torch.zeros(1 << 20, device="cuda")
torch.cuda.synchronize()
t4 = time.perf_counter()
n = max(1, sum(where.values()))
print(json.dumps({"cuda_init_ms": round((t3 - t2) * 1e3, 1), "hsa_init_ms": round((t_hsa - t2) * 1e3, 1), "first_alloc_ms": round((t4 - t3) * 1e3, 1),
                  "init_where_pct": {k: round(100 * v / n, 1) for k, v in sorted(where.items(), key=lambda x: -x[1])},
                  "init_thread_cpu_ms": round((r1.ru_utime + r1.ru_stime - r0.ru_utime - r0.ru_stime) * 1e3, 1),
                  "system_jiffies_during_init": {k: s1[k] - s0[k] for k in s1},
                  "init_nvcsw": r1.ru_nvcsw - r0.ru_nvcsw, "init_nivcsw": r1.ru_nivcsw - r0.ru_nivcsw,
                  "cgroup_during_init": {k: c1[k] - c0.get(k, 0) for k in c1 if k in ("usage_usec", "nr_throttled", "throttled_usec", "nr_periods")}}), flush=True)
"""


def trial(mode: str, when: str, pause_s: float, cpus: tuple = ("", "")) -> dict:
    import os
    st = subprocess.Popen([sys.executable, "-c", STARTER], stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True,
                          env=dict(os.environ, GS_CPU=cpus[1]))
    assert st.stdout.readline().strip() == "go"
    tenv = dict(os.environ, GS_CPU=cpus[0])
    if mode.startswith("shim"):                # the tenant under the quota shim (kfd mode)
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        tenv.update(LD_PRELOAD=os.path.join(root, "aliyun_gpushare_device_plugin_amd", "_native", "libgpushare_hipquota.so"),
                    GPUSHARE_QUOTA_BYTES=str(200 << 30), GPUSHARE_SHIM_FREE_ALLOCS_AT_EXIT="1" if mode == "shimfastall" else "0")
    t = subprocess.Popen([sys.executable, "-c", TENANT], stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True,
                         env=tenv)
    assert json.loads(t.stdout.readline())["ready"]
    t0 = time.perf_counter()
    t.stdin.write(mode + "\n")
    t.stdin.flush()
    assert json.loads(t.stdout.readline())["leaving"]
    t_ack = time.perf_counter()
    if when == "reaped":
        t.wait(60)
    time.sleep(pause_s)
    t_go = time.perf_counter()
    st.stdin.write("\n")
    st.stdin.flush()
    r = json.loads(st.stdout.readline())
    st.wait(60)
    t.wait(60)
    return dict(r, mode=mode, when=when, pause_s=pause_s, cpus=list(cpus), leave_ms=round((t_ack - t0) * 1e3, 1),
                go_after_ack_ms=round((t_go - t_ack) * 1e3, 1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=3)
    ap.add_argument("--modes", default="exit,free,reset")
    ap.add_argument("--whens", default="ack,reaped")
    ap.add_argument("--tenants", default="", help="tenant kinds to compare (initonly,small,full): reaped order")
    ap.add_argument("--pin", default="", help="'T/S' CPU lists for tenant / starter, ';'-separated variants")
    a = ap.parse_args()
    if a.tenants:
        import os
        for i in range(a.trials):
            for k in a.tenants.split(","):
                os.environ["GS_TENANT"] = k
                print(json.dumps(dict(trial("exit", "reaped", 0.0), tenant=k, trial=i)), flush=True)
        return
    if a.pin:                      # placement variants only: reaped order, no pause
        for i in range(a.trials):
            for v in a.pin.split(";"):
                tc, sc = v.split("/")
                print(json.dumps(dict(trial("exit", "reaped", 0.0, (tc, sc)), trial=i)), flush=True)
        return
    for i in range(a.trials):
        for mode in a.modes.split(","):
            for when in a.whens.split(","):
                print(json.dumps(dict(trial(mode, when, 0.0), trial=i)), flush=True)
        print(json.dumps(dict(trial("exit", "reaped", 1.0), trial=i)), flush=True)


if __name__ == "__main__":
    main()
