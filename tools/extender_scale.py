"""Scheduler-extender scale probe: filter + bind latency for a large pending queue.

Builds an Extender over N synthetic MI355X nodes (8 x 288 GiB each) with a stub apiserver
client (no network: what is measured is the extender's own placement work), optionally
pre-fills every GPU to a random level, queues Q mixed-size pods (8-128 GiB, as BASELINE
config 3), and schedules them one by one as kube-scheduler would, with new pods arriving while
the queue drains. Prints one JSON line: placed pods, per-call p50/p99/max and the total.

    python tools/extender_scale.py --nodes 512 --queue 14000 --busy
"""
from __future__ import annotations

import argparse
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from aliyun_gpushare_device_plugin_amd import const  # noqa: E402
from aliyun_gpushare_device_plugin_amd.extender import Extender  # noqa: E402

SIZES = (8, 16, 32, 56, 64, 96, 128)


def _node(i: int) -> dict:
    return {"metadata": {"name": f"n{i}", "labels": {"gpushare": "true"}, "annotations": {}},
            "status": {"capacity": {const.RESOURCE_NAME: str(8 * 288), const.RESOURCE_COUNT: "8"},
                       "allocatable": {const.RESOURCE_NAME: str(8 * 288), const.RESOURCE_COUNT: "8"}}}


def _pod(i: int, size: int) -> dict:
    return {"metadata": {"name": f"p{i}", "namespace": "default", "uid": f"u{i}", "annotations": {}},
            "spec": {"containers": [{"name": "c", "resources": {"limits": {const.RESOURCE_NAME: str(size)}}}]},
            "status": {"phase": "Pending"}}


class _Client:
    def __init__(self, n):
        self.n = n

    def list_nodes(self, label_selector=None):
        return [_node(i) for i in range(self.n)]

    def list_pods(self, *a, **k):
        return [], "1"

    def patch_pod(self, *a, **k):
        return None

    def bind_pod(self, *a, **k):
        return None


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--nodes", type=int, default=512)
    ap.add_argument("--queue", type=int, default=2000)
    ap.add_argument("--busy", action="store_true", help="pre-fill every GPU to a random level")
    ap.add_argument("--arrivals", type=int, default=5, help="new pods every 50 scheduled")
    ap.add_argument("--seed", type=int, default=2)
    a = ap.parse_args(argv)
    rnd = random.Random(a.seed)
    e = Extender(_Client(a.nodes))
    e.sync()
    if a.busy:
        for st in e.nodes.values():
            st.used = [rnd.choice([0, 32, 96, 160, 200, 240, 270]) for _ in range(8)]
    free = sum(sum(st.free()) for st in e.nodes.values())
    pods = [_pod(i, rnd.choice(SIZES)) for i in range(a.queue)]
    for p in pods:
        e.note_pending(p)
    lat, placed, seq = [], 0, a.queue
    t0 = time.perf_counter()
    for k, p in enumerate(pods):
        t = time.perf_counter()
        e.filter(p)
        placed += e.schedule(p) is not None
        lat.append(time.perf_counter() - t)
        if k and k % 50 == 0:
            for _ in range(a.arrivals):
                e.note_pending(_pod(seq, rnd.choice(SIZES)))
                seq += 1
    total = time.perf_counter() - t0
    lat.sort()
    demand = sum(int(p["spec"]["containers"][0]["resources"]["limits"][const.RESOURCE_NAME]) for p in pods)
    print(json.dumps({"nodes": a.nodes, "gpus": 8 * a.nodes, "queue": a.queue, "busy": a.busy,
                      "demand_over_free": round(demand / free, 3), "placed": placed,
                      "call_p50_ms": round(lat[len(lat) // 2] * 1e3, 3),
                      "call_p99_ms": round(lat[int(len(lat) * 0.99)] * 1e3, 3),
                      "call_max_ms": round(lat[-1] * 1e3, 3), "total_s": round(total, 2)}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
