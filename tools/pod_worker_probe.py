#!/usr/bin/env python3
"""Probe the pod-worker lifecycle on one MI355X: spawn standby processes under the quota shim,
start them as 4 pods (64+64+96+64 GiB, fill 0.85), run traffic for a few seconds, stop.
Prints one JSON document (standby spawn time, ready latency, aggregate TFLOP/s, HBM held)."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SHIM = os.path.join(ROOT, "aliyun_gpushare_device_plugin_amd", "_native", "libgpushare_hipquota.so")


def spawn():
    env = dict(os.environ, LD_PRELOAD=":".join(x for x in (SHIM, os.environ.get("LD_PRELOAD", "")) if x), PYTHONPATH=ROOT)
    t = time.perf_counter()
    p = subprocess.Popen([sys.executable, "-m", "aliyun_gpushare_device_plugin_amd.models.pod_worker"], env=env,
                         stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, bufsize=1)
    ev = json.loads(p.stdout.readline())
    assert ev["event"] == "standby"
    return p, time.perf_counter() - t


def main():
    sizes = [64, 64, 96, 64]
    total = int(os.environ.get("DEV_BYTES", "309220868096"))
    out = {"spawn_s": [], "ready": []}
    procs = []
    for s in sizes:
        p, dt = spawn()
        out["spawn_s"].append(round(dt, 3))
        procs.append((p, s))
    for i, (p, s) in enumerate(procs):
        env = {"GPUSHARE_QUOTA_BYTES": str(total * s // 288), "ALIYUN_COM_GPU_MEM_CONTAINER": str(s),
               "ALIYUN_COM_GPU_MEM_DEV": "288", "GPUSHARE_LEDGER": f"/gs-probe-{os.getpid()}-{i}"}
        t = time.perf_counter()
        p.stdin.write(json.dumps({"cmd": "start", "env": env, "gemm": 4096, "burst": 8, "fill": 0.85}) + "\n")
        ev = json.loads(p.stdout.readline())
        ev["wall_ms"] = round((time.perf_counter() - t) * 1e3, 1)
        out["ready"].append(ev)
    def stats():
        r = []
        for p, _ in procs:
            p.stdin.write('{"cmd":"stats"}\n')
        for p, _ in procs:
            r.append(json.loads(p.stdout.readline()))
        return r
    s0 = stats()
    time.sleep(float(os.environ.get("SECONDS_RUN", "5")))
    s1 = stats()
    dt = max(b["t"] for b in s1) - min(a["t"] for a in s0)
    n = sum(b["gemms"] - a["gemms"] for a, b in zip(s0, s1))
    out["tflops_aggregate"] = round(2 * 4096 ** 3 * n / dt / 1e12, 1)
    out["per_pod_gemms"] = [b["gemms"] - a["gemms"] for a, b in zip(s0, s1)]
    t = time.perf_counter()
    for p, _ in procs:
        p.stdin.write('{"cmd":"stop"}\n')
    out["done"] = [json.loads(p.stdout.readline()) for p, _ in procs]
    for p, _ in procs:
        p.wait(30)
    out["stop_s"] = round(time.perf_counter() - t, 3)
    for i in range(len(sizes)):
        try:
            os.unlink(f"/dev/shm/gs-probe-{os.getpid()}-{i}")
        except FileNotFoundError:
            pass
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
