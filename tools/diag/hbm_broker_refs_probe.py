"""Probe: do a tenant's imports show in its granules' dma-buf reference counts, and when do they
drop after the tenant exits? (the HBM broker's quarantine relies on it; prints one JSON line)"""
import json, os, sys, time
sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import test_hbm_broker as T
from aliyun_gpushare_device_plugin_amd.quota.hbmbroker import HBMBroker
b = HBMBroker("/tmp/refsprobe/hbm.sock", device=0, gib=8, wait_s=20)
os.makedirs("/tmp/refsprobe", exist_ok=True)
b.start()
try:
    b.grant("z" * 32, 6 << 30)
    p = T._tenant(b, "z" * 32, "hold")
    first = json.loads(p.stdout.readline())
    during = b.stat()
    p.stdin.write("\n"); p.stdin.flush(); p.wait(60)
    t0 = time.time()
    trace = []
    while time.time() - t0 < 5:
        st = b.stat()
        trace.append((round(time.time() - t0, 3), st["quarantined"], st["free"]))
        if not st["quarantined"]:
            break
        time.sleep(0.05)
    print(json.dumps({"tenant": first, "base_refs": during["base_refs"],
                      "held_refs_over_base_while_imported": during["held_refs_max"],
                      "after_exit_trace": trace}))
finally:
    b.stop()
