"""Where a HIP process's normal exit spends its time: libc exit(0) after a kernel, timed from the
parent (blocking waitpid), with the runtime's log (AMD_LOG_LEVEL=4: microsecond timestamps) of the
teardown. Prints one JSON line per run; the logs go to <out>/exit_<n>.log."""
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

out = sys.argv[1] if len(sys.argv) > 1 else "/tmp"
os.makedirs(out, exist_ok=True)
for n, log in enumerate((False, True, False, True)):
    env = dict(os.environ)
    if log:
        env["AMD_LOG_LEVEL"] = "4"
    with open(os.path.join(out, f"exit_{n}.log"), "w") as err:
        p = subprocess.Popen([sys.executable, "-c", CODE], stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                             stderr=err, text=True, env=env)
        assert p.stdout.readline().strip() == "ready"
        time.sleep(0.3)
        t0 = time.perf_counter()
        p.stdin.write("\n")
        p.stdin.flush()
        p.wait()
        print(json.dumps({"run": n, "log": log, "exit_ms": round((time.perf_counter() - t0) * 1e3, 2),
                          "rc": p.returncode}), flush=True)
    time.sleep(1.0)
