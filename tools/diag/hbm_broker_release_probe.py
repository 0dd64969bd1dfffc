"""Probe: after a pod frees everything and hands its broker arena back early
(gpushare_shim_arena_release), do its granules' dma-buf references drop at once, or only when
the process exits? Runs a tenant that allocates, runs one matmul, frees, releases, then sleeps 2 s
before exiting, while the broker's quarantine is sampled. Prints one JSON line."""
import json, os, sys, time
sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import test_hbm_broker as T
from aliyun_gpushare_device_plugin_amd.quota.hbmbroker import HBMBroker

from aliyun_gpushare_device_plugin_amd.utils.native import preload
TENANT = r"""
import ctypes, json, sys, time
import torch
x = torch.empty(3 << 30, dtype=torch.uint8, device="cuda")
a = torch.ones(1024, 1024, device="cuda", dtype=torch.bfloat16) * 2
a.sum().item()
del x, a
torch.cuda.synchronize()
torch.cuda.empty_cache()
lib = ctypes.CDLL(None)
live0 = torch.cuda.memory_allocated()
r1 = lib.gpushare_shim_arena_release()
if r1 == -1:
    try:
        torch._C._cuda_clearCublasWorkspaces()
    except Exception:
        pass
    torch.cuda.empty_cache()
    r2 = lib.gpushare_shim_arena_release()
else:
    r2 = None
print(json.dumps({"release_first": r1, "release_after_clearing_blas": r2, "torch_allocated": live0}), flush=True)
time.sleep(2.0)
"""
os.makedirs("/tmp/relprobe", exist_ok=True)
b = HBMBroker("/tmp/relprobe/hbm.sock", device=0, gib=8, wait_s=20)
b.start()
try:
    b.grant("y" * 32, 6 << 30)
    import subprocess
    from aliyun_gpushare_device_plugin_amd.utils.native import ensure_built
    env = dict(os.environ, LD_PRELOAD=preload(ensure_built("hipshim")), GPUSHARE_QUOTA_BYTES=str(8 << 30),
               GPUSHARE_HBM_BROKER=b.socket_path, GPUSHARE_HBM_TOKEN="y" * 32)
    p = subprocess.Popen([sys.executable, "-c", TENANT], env=env, stdout=subprocess.PIPE, text=True)
    first = json.loads(p.stdout.readline())
    t0 = time.time()
    trace = []
    while p.poll() is None or time.time() - t0 < 3.0:
        st = b.stat()
        trace.append((round(time.time() - t0, 3), st["releases"], st["quarantined"], st["free"], p.poll()))
        if time.time() - t0 > 4.0:
            break
        time.sleep(0.1)
    print(json.dumps({"tenant": first, "trace": trace}))
finally:
    b.stop()
