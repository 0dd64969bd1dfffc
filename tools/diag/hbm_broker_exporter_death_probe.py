"""What a tenant sees when its HBM broker (the exporter of its granules) dies: SIGKILL the broker
while a tenant holds mapped granules, then have the tenant read, write and allocate, and exit.
Prints one JSON line (docs/HBM_TURNOVER.md, exporter death).

    python tools/diag/hbm_broker_exporter_death_probe.py
"""
from __future__ import annotations

import json
import os
from aliyun_gpushare_device_plugin_amd.utils.native import preload
import signal
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
GIB = 1 << 30

TENANT = r"""
import ctypes, json, sys, time
import torch
x = torch.empty(5 * (1 << 30), dtype=torch.uint8, device="cuda")
x.fill_(7)
torch.cuda.synchronize()
lib = ctypes.CDLL(None)
size, used = ctypes.c_uint64(), ctypes.c_uint64()
print(json.dumps({"phase": "held", "arena": lib.gpushare_shim_arena_stats(ctypes.byref(size), ctypes.byref(used)),
                  "arena_size": size.value}), flush=True)
sys.stdin.readline()                       # the broker is dead now
out = {"phase": "after"}
try:
    out["min_before"] = int(x.min().item()); out["max_before"] = int(x.max().item())
    x.add_(1)
    torch.cuda.synchronize()
    out["min_after"] = int(x.min().item()); out["max_after"] = int(x.max().item())
    y = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")   # the arena's rest
    y.fill_(3); torch.cuda.synchronize()
    out["alloc_after"] = "ok"
except Exception as e:
    out["error"] = f"{type(e).__name__}: {e}"[:500]
print(json.dumps(out), flush=True)
"""

FREE = "import torch, json; f, t = torch.cuda.mem_get_info(); print(json.dumps({'free': f, 'total': t}))"


def device_free() -> int:
    r = subprocess.run([sys.executable, "-c", FREE], capture_output=True, text=True, timeout=120)
    return json.loads(r.stdout.strip().splitlines()[-1])["free"]


def main() -> int:
    from aliyun_gpushare_device_plugin_amd.quota.hbmbroker import HBMBroker
    from aliyun_gpushare_device_plugin_amd.utils.native import ensure_built

    out: dict = {"free_before_gib": round(device_free() / GIB, 2)}
    d = tempfile.mkdtemp(prefix="gs-death-", dir="/tmp")
    b = HBMBroker.for_gpu(d, 0, device=0, gib=16, wait_s=20)
    out["broker"] = b.start()
    b.grant("x" * 32, 8 * GIB)
    env = dict(os.environ, LD_PRELOAD=preload(ensure_built("hipshim")), GPUSHARE_QUOTA_BYTES=str(12 * GIB),
               GPUSHARE_HBM_BROKER=b.socket_path, GPUSHARE_HBM_TOKEN="x" * 32)
    t = subprocess.Popen([sys.executable, "-c", TENANT], env=env, stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True)
    try:
        out["held"] = json.loads(t.stdout.readline())
        out["free_with_broker_gib"] = round(device_free() / GIB, 2)
        b.proc.send_signal(signal.SIGKILL)
        b.proc.wait(30)
        time.sleep(1.0)
        out["free_after_broker_death_gib"] = round(device_free() / GIB, 2)
        t.stdin.write("\n")
        t.stdin.flush()
        out["tenant"] = json.loads(t.stdout.readline() or "{}")
        t.stdin.close()
        out["tenant_rc"] = t.wait(60)
        out["tenant_stderr_tail"] = t.stderr.read()[-800:]
        time.sleep(1.0)
        out["free_after_tenant_exit_gib"] = round(device_free() / GIB, 2)
    finally:
        if t.poll() is None:
            t.kill()
        b.proc = None
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
