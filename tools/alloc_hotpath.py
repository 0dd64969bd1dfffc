"""Plugin-side Allocate handler cost, in process (no gRPC): what ``plugin_allocate_p50_ms`` in
the bench line measures, isolated. Churn like the bench: a node holding 32 pods plus a few
hundred finished ones, each step deletes one pod and admits a same-size replacement whose fake
IDs are the freed ones (the kubelet recycles IDs), with the bench's plugin options
(write-behind patch, journal file, shim + per-container ledger dirs).

    python tools/alloc_hotpath.py [--steps 2000]
Prints one JSON line: p50/p90/p99 per phase (ms).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from aliyun_gpushare_device_plugin_amd import const  # noqa: E402
from aliyun_gpushare_device_plugin_amd.alloc.engine import Allocator, AllocatorOptions  # noqa: E402
from aliyun_gpushare_device_plugin_amd.api import v1beta1 as api  # noqa: E402
from aliyun_gpushare_device_plugin_amd.cluster import objects as O  # noqa: E402
from aliyun_gpushare_device_plugin_amd.cluster.podcache import WatchCache  # noqa: E402
from aliyun_gpushare_device_plugin_amd.device import smi as S  # noqa: E402
from aliyun_gpushare_device_plugin_amd.device.model import DeviceModel  # noqa: E402
from aliyun_gpushare_device_plugin_amd.quota import ShimConfig  # noqa: E402

PATTERNS = [[128, 64, 64, 32], [96, 96, 64, 32], [128, 96, 56, 8], [64, 64, 96, 64]]


class Cache(WatchCache):
    """The plugin's watch cache, fed events directly (no apiserver)."""

    def __init__(self):
        super().__init__(None, "n")
        self._synced.set()

    def put(self, p):
        self._apply({"type": "MODIFIED", "object": p})

    @property
    def by_uid(self):
        return self._pods


class Client:
    def __init__(self, cache):
        self.cache = cache

    def patch_pod(self, ns, name, patch, content_type=None):
        for p in self.cache.by_uid.values():
            if O.name(p) == name:
                q = dict(p, metadata=dict(p["metadata"], annotations=dict(p["metadata"]["annotations"])))
                for k, v in patch["metadata"]["annotations"].items():
                    q["metadata"]["annotations"][k] = v
                q["metadata"]["resourceVersion"] = str(int(p["metadata"]["resourceVersion"]) + 1)
                return q
        return None


def pod(name, size, gpu, t):
    return {"metadata": {"name": name, "namespace": "default", "uid": f"uid-{name}", "resourceVersion": "1",
                         "annotations": {const.ENV_RESOURCE_INDEX: str(gpu), const.ENV_RESOURCE_ASSUME_TIME: str(t),
                                         const.ENV_ASSIGNED_FLAG: "false"}},
            "spec": {"nodeName": "n", "containers": [{"name": "c", "resources": {"limits": {
                const.RESOURCE_NAME: str(size)}}}]},
            "status": {"phase": "Pending"}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--pace-ms", type=float, default=5.0, help="idle time between admissions (bench: ~250 ms)")
    a = ap.parse_args()
    work = tempfile.mkdtemp(prefix="gs-hot-")
    with S.SMI(f"fake:{a.gpus}x288G") as smi:
        model = DeviceModel(smi.devices(), const.GIB, "nearest")
    cache = Cache()
    al = Allocator(model, cache, Client(cache), "n", AllocatorOptions(
        shim=ShimConfig(work), async_patch=True, journal_path=os.path.join(work, "journal.jsonl"),
        ledger_dir=os.path.join(work, "ledgers")), None)
    free_ids = {g: [f"{model.gpu(g).uuid}-_-{j}" for j in range(288)] for g in range(a.gpus)}
    held: dict[str, list] = {}
    seq = iter(range(10 ** 9))
    resident = {g: [] for g in range(a.gpus)}

    def admit(size, g):
        name = f"p{next(seq)}"
        p = pod(name, size, g, time.time_ns())
        cache.put(p)
        ids, free_ids[g] = free_ids[g][:size], free_ids[g][size:]
        req = api.AllocateRequest(container_requests=[api.ContainerAllocateRequest(devices_ids=ids)])
        t0 = time.perf_counter()
        al.allocate(req)
        dt = time.perf_counter() - t0
        cur = cache.by_uid[O.uid(p)]
        cache.put(dict(cur, status={"phase": "Running"}, metadata=dict(cur["metadata"], resourceVersion=str(
            int(cur["metadata"]["resourceVersion"]) + 1))))
        held[O.uid(p)] = ids
        resident[g].append((O.uid(p), size))
        return dt

    for g in range(a.gpus):
        for s in PATTERNS[g % 4]:
            admit(s, g)
    al.flush_patches(10)
    time.sleep(1.0)                     # ledger-dir pool refilled, patcher idle
    al.metrics.allocate_latency.reset()
    lat = []
    for i in range(a.steps):
        g = i % a.gpus
        uid, size = resident[g].pop(0)
        p = cache.by_uid[uid]
        cache.put(dict(p, status={"phase": "Succeeded"}, metadata=dict(p["metadata"], resourceVersion=str(
            int(p["metadata"]["resourceVersion"]) + 1))))              # finished pods stay listed a while
        free_ids[g] = held.pop(uid) + free_ids[g]                     # the kubelet recycles freed IDs first
        lat.append(admit(size, g))
        if len(cache.by_uid) > 400:
            for u in [u for u, q in cache.by_uid.items() if O.is_terminated(q)][:50]:
                cache._apply({"type": "DELETED", "object": cache.by_uid[u]})
        time.sleep(a.pace_ms / 1e3)
    al.flush_patches(10)
    lat.sort()
    summ = {e["labels"].get("phase"): round(e["p50"] * 1e3, 4) for e in al.metrics.allocate_latency.summary()}
    print(json.dumps({"steps": a.steps, "p50_ms": round(lat[len(lat) // 2] * 1e3, 4),
                      "p90_ms": round(lat[int(len(lat) * 0.9)] * 1e3, 4), "p99_ms": round(lat[int(len(lat) * 0.99)] * 1e3, 4),
                      "phase_p50_ms": summ}))


if __name__ == "__main__":
    main()
