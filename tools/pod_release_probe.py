#!/usr/bin/env python3
"""Does a stopped pod process give its HBM back before it exits? Start one 128 GiB pod (fill
0.85), stop it, and read the device's VRAM use (SMI) right after its "done" event and after the
process has exited."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from aliyun_gpushare_device_plugin_amd.device.smi import SMI  # noqa: E402

SHIM = os.path.join(ROOT, "aliyun_gpushare_device_plugin_amd", "_native", "libgpushare_hipquota.so")


def vram_used(s):
    s.refresh()
    return s.device(0).vram_used


def main():
    out = {}
    with SMI("auto") as s:
        out["idle"] = vram_used(s)
        env = dict(os.environ, LD_PRELOAD=":".join(x for x in (SHIM, os.environ.get("LD_PRELOAD", "")) if x), PYTHONPATH=ROOT)
        p = subprocess.Popen([sys.executable, "-m", "aliyun_gpushare_device_plugin_amd.models.pod_worker"], env=env,
                             stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, bufsize=1)
        assert json.loads(p.stdout.readline())["event"] == "standby"
        q = s.device(0).vram_total * 128 // 288
        p.stdin.write(json.dumps({"cmd": "start", "env": {"GPUSHARE_QUOTA_BYTES": str(q)}, "fill": 0.85}) + "\n")
        out["ready"] = json.loads(p.stdout.readline())
        out["running"] = vram_used(s)
        hold_exit = os.environ.get("HOLD_EXIT", "0") == "1"
        if hold_exit:   # keep the process alive after "done": is the HBM back without an exit?
            p.stdin.write('{"cmd":"stop"}\n')
        else:
            p.stdin.write('{"cmd":"stop"}\n')
        out["done"] = json.loads(p.stdout.readline())
        t = time.perf_counter()
        out["after_done"] = vram_used(s)
        series = []
        exit_t = None
        while time.perf_counter() - t < 6.0:
            if exit_t is None and p.poll() is not None:
                exit_t = round(time.perf_counter() - t, 3)
            series.append((round(time.perf_counter() - t, 3), vram_used(s)))
            time.sleep(0.1)
        out["exit_s"] = exit_t
        out["series"] = series
        out["after_exit"] = vram_used(s)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
