#!/usr/bin/env python3
"""Where does the kubelet-side Allocate latency of the bench go? Churn 40 pods through the
bench's control plane (plugin process, fake apiserver process, fake kubelet in this process)
(a) with nothing else running, (b) while 4 pod processes run GEMM traffic on the GPU under
the shim, (c) as (b) plus 2 standby pod interpreters importing torch during the churn.
Prints kubelet-side and plugin-side p50 for each."""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def churn(cp, n=40):
    cp.plugin_latency(reset=True)
    cp.alloc_lat.clear()
    for _ in range(n):
        cp.churn()
    srv = cp.plugin_latency()
    return {"kubelet_p50_ms": bench.ms(bench.pct(cp.alloc_lat, 0.5)), "plugin_p50_ms": bench.ms(srv["p50"]) if srv else None}


def main():
    import torch

    torch.cuda.set_device(0)
    cp = bench.ControlPlane(1, "auto", "watch", "process", tempfile.mkdtemp(), with_shim=True)
    started = cp.fill()
    out = {"quiet": churn(cp)}
    fleet = bench.PodFleet(0, 4096, 8, 0.3, True, standby=4)
    for rec in started[0]:
        fleet.start(rec)
    time.sleep(3)
    out["with_traffic"] = churn(cp)
    for _ in range(2):
        fleet._spawn()             # two interpreters importing torch during the churn
    out["with_traffic_and_spawns"] = churn(cp, 20)
    fleet.close()
    cp.stop()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
