"""Where a HIP process's normal exit spends its time: libc exit(0) after a kernel, timed from the
parent (blocking waitpid), with the runtime's log (AMD_LOG_LEVEL=4: microsecond timestamps) of the
teardown. Prints one JSON line per run; the logs go to <out>/exit_<n>.log.
``--shim``: the same under the quota shim, with its exit-time skip of code-object unloads on and
off (GPUSHARE_SHIM_SKIP_UNLOAD_AT_EXIT), no logs."""
import json
import os
import subprocess
import sys
import time

CODE = r"""
import ctypes, sys, time, torch
x = torch.ones(1 << 20, device="cuda"); x.add_(1); torch.cuda.synchronize()
print("ready", flush=True)
sys.stdin.readline()
sys.stderr.write("=== EXIT CALLED %d us\n" % (time.clock_gettime_ns(time.CLOCK_REALTIME) // 1000)); sys.stderr.flush()
ctypes.CDLL(None).exit(0)
"""

args = [a for a in sys.argv[1:] if a != "--shim"]
shim = "--shim" in sys.argv
out = args[0] if args else "/tmp"
os.makedirs(out, exist_ok=True)
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
runs = [(False, s) for s in ("1", "0", "1", "0", "1", "0")] if shim else [(lg, None) for lg in (False, True, False, True)]
for n, (log, skip) in enumerate(runs):
    env = dict(os.environ)
    if log:
        env["AMD_LOG_LEVEL"] = "4"
    if skip is not None:
        env.update(LD_PRELOAD=os.path.join(ROOT, "aliyun_gpushare_device_plugin_amd", "_native", "libgpushare_hipquota.so"),
                   GPUSHARE_QUOTA_BYTES=str(64 << 30), GPUSHARE_SHIM_SKIP_UNLOAD_AT_EXIT=skip)
    with open(os.path.join(out, f"exit_{n}.log"), "w") as err:
        p = subprocess.Popen([sys.executable, "-c", CODE], stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                             stderr=err, text=True, env=env)
        assert p.stdout.readline().strip() == "ready"
        time.sleep(0.3)
        t0 = time.perf_counter()
        p.stdin.write("\n")
        p.stdin.flush()
        p.wait()
        print(json.dumps({"run": n, "log": log, "shim_skip_unload": skip,
                          "exit_ms": round((time.perf_counter() - t0) * 1e3, 2), "rc": p.returncode}), flush=True)
    time.sleep(1.0)
