#!/usr/bin/env python3
"""Headline benchmark: bin-packed pods + HBM-GiB per node with Allocate latency, on 1/2/4/8 MI355X.

Metric (BASELINE.json): "bin-packed pods + HBM-GiB/node; Allocate p50 latency at 1/2/4/8 MI355X".

Scenario (one node with N = --gpus MI355X, one rank per GPU, rank 0 also hosts the control plane):
  * control plane = the real plugin (``gpushare-device-plugin`` in its own process, devices from
    librocm_smi/sysfs), a fake kube-apiserver process, the extender bin-packer and the fake kubelet
    (gRPC over UDS) — the same path pods take in production (sim/cluster.py);
  * warm-up fills every GPU with 4 pods of mixed size 8-128 GiB summing to 288 GiB (BASELINE
    config 3: 32 pods on 8 GPUs);
  * each timed step = one churn wave under real traffic: every resident pod launches a burst of
    bf16 MFMA GEMMs (hand-written gfx950 kernel, 4096^3, operands inside the pod's HBM share, one
    HIP stream per pod), and while the GPUs run, rank 0 retires the oldest pod on every GPU and
    admits a replacement of the same size through delete -> create -> extender bind -> kubelet
    Allocate -> Running. Per-GPU work is fixed (1 admission + 4 bursts), so scaling is weak.
``value`` = pod admissions per second for the whole node (higher is better). Also reported: Allocate
p50/p99 (kubelet-side gRPC round trip), pods and GiB bin-packed per node, advertised GiB per node and
the aggregate GEMM TFLOP/s delivered to the pods.

python bench.py --gpus N --steps K --warmup W   (N>1: launched by torch.distributed.run)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "bin-packed pods + HBM-GiB/node; Allocate p50 latency at 1/2/4/8 MI355X"
# Per-GPU pod sizes (GiB), each pattern sums to one MI355X (288 GiB); GPU g uses pattern g % 4.
PATTERNS = [[128, 64, 64, 32], [96, 96, 64, 32], [128, 96, 56, 8], [64, 64, 96, 64]]


def parse():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--burst", type=int, default=40, help="GEMMs per resident pod per step")
    ap.add_argument("--gemm", type=int, default=4096, help="GEMM M=N=K")
    ap.add_argument("--burst-mode", default="loop", choices=("loop", "fused"),
                    help="a pod's burst as one launch per GEMM, or one dispatch of all of them (same FLOPs)")
    ap.add_argument("--no-gpu", action="store_true", help="control plane only (CPU)")
    ap.add_argument("--smi-backend", default=None, help="default: auto on GPU, fake:Nx288G on CPU")
    ap.add_argument("--pod-source", default="watch", choices=("watch", "list", "kubelet"))
    ap.add_argument("--plugin-mode", default="process", choices=("process", "thread"))
    ap.add_argument("--json-out", default=None)
    return ap.parse_args()


def pct(xs, q):
    if not xs:
        return None
    s = sorted(xs)
    return s[min(len(s) - 1, max(0, int(round(q * (len(s) - 1)))))]


class ControlPlane:
    """Rank 0's view of the node: fake cluster + the real plugin process."""

    def __init__(self, n_gpus: int, smi_spec: str, pod_source: str, plugin_mode: str):
        from aliyun_gpushare_device_plugin_amd.sim.cluster import SimCluster

        self.n = n_gpus
        import socket

        with socket.socket() as s:              # a free port for the plugin's metrics endpoint
            s.bind(("127.0.0.1", 0))
            self.metrics_port = s.getsockname()[1]
        extra = ["--metrics-addr", f"127.0.0.1:{self.metrics_port}"] if plugin_mode == "process" else []
        self.cluster = SimCluster([("mi355x-node", smi_spec)], plugin_mode=plugin_mode, pod_source=pod_source,
                                  apiserver="process", gpu_indices=list(range(n_gpus)), health_poll_s=5.0,
                                  extra_plugin_args=extra)
        self.cluster.start()
        from aliyun_gpushare_device_plugin_amd import const
        from aliyun_gpushare_device_plugin_amd.cluster import objects as O

        node = self.cluster.client.get_node("mi355x-node")
        self.gpu_count = O.node_allocatable(node, const.RESOURCE_COUNT)
        self.units_per_gpu = O.node_allocatable(node, const.RESOURCE_NAME) // max(1, self.gpu_count)
        if self.gpu_count != n_gpus:
            raise RuntimeError(f"plugin advertises {self.gpu_count} GPUs, expected {n_gpus}")
        self.resident: dict[int, list] = {g: [] for g in range(n_gpus)}   # gpu -> [(pod, size)] oldest first
        import concurrent.futures as cf

        import threading

        self.pool = cf.ThreadPoolExecutor(max_workers=max(1, n_gpus), thread_name_prefix="churn")
        self._sched_lock = threading.Lock()
        self._kubelet = threading.Condition()
        self.alloc_lat: list[float] = []
        self.admit_lat: list[float] = []
        self.failed = 0
        self.fail_reasons: list[str] = []
        self.cp_time = 0.0

    def admit(self, size: int):
        t0 = time.perf_counter()
        pod, where, adm = self.cluster.run_pod(size)
        if where is None or adm is None or adm.error:
            self.failed += 1
            if where is not None:
                self.cluster.delete_pod(pod)
            return None
        self.alloc_lat.extend(adm.latencies)
        self.admit_lat.append(time.perf_counter() - t0)
        gpu = int(dict(adm.responses[0].envs)["ALIYUN_COM_GPU_MEM_IDX"])
        self.resident[gpu].append((pod, size))
        return gpu

    def fill(self):
        """Pods arrive as per-GPU-sized groups (think one StatefulSet per 288 GiB of demand), in
        pattern order. The extender's online best-fit places each group exactly onto one GPU, so
        the node packs 100 %; the same 32 pods in globally size-sorted order strand 56 GiB under
        that policy (31 of 32 placed at N = 8: its tie-break stacks two 128 GiB pods per GPU)."""
        for g in range(self.n):
            for s in PATTERNS[g % len(PATTERNS)]:
                self.admit(s)

    def churn(self):
        """Retire the oldest pod on every GPU and admit a same-size replacement.

        One pipeline per GPU, as in a real cluster where each replacement is independent:
        delete (controller) -> create -> scheduling cycle (extender decide, stamps the assume
        time) -> binding cycle (annotations + bind) -> kubelet admission. Only the scheduling
        cycle and the kubelet are serial: the kubelet's pod worker sees pods in bind order, so
        admissions are taken in assume-time order (a ticket per decision) and the plugin's
        earliest-assumed match is the pod actually being admitted. Every replacement has an
        exact-fit slot (its predecessor's), so best-fit keeps the node packed.
        """
        import itertools

        olds = [(g, self.resident[g].pop(0)) for g in range(self.n) if self.resident[g]]
        ext = self.cluster.extender
        tickets = itertools.count()
        turn = {"next": 0}

        def chain(it):
            _, (old, size) = it
            self.cluster.delete_pod(old)
            pod = self.cluster.create_pod(size)
            with self._sched_lock:                      # the scheduler's one-pod-at-a-time cycle
                where = ext.decide(pod)
                ticket, assume_ns = next(tickets), time.time_ns()
            try:
                bpod = ext.commit(pod, where, assume_ns) if where else None
                with self._kubelet:
                    while turn["next"] != ticket:
                        self._kubelet.wait()
                if bpod is None:
                    return None, size, None, 0.0
                t0 = time.perf_counter()
                adm = self.cluster.admit(bpod, async_status=True)
                return bpod, size, adm, time.perf_counter() - t0
            finally:
                with self._kubelet:
                    while turn["next"] != ticket:
                        self._kubelet.wait()
                    turn["next"] += 1
                    self._kubelet.notify_all()

        for bpod, size, adm, dt in self.pool.map(chain, olds):
            if adm is None or adm.error:
                self.failed += 1
                self.fail_reasons.append(f"{size}GiB: " + ("unschedulable" if bpod is None else f"admit: {adm and adm.error}"))
                if bpod is not None:
                    self.cluster.delete_pod(bpod)
                continue
            gpu = int(dict(adm.responses[0].envs)["ALIYUN_COM_GPU_MEM_IDX"])
            if gpu < 0:                                 # soft failure: no candidate matched
                self.failed += 1
                self.fail_reasons.append(f"{size}GiB: plugin found no candidate")
                self.cluster.delete_pod(bpod)
                continue
            self.alloc_lat.extend(adm.latencies)
            self.admit_lat.append(dt)
            self.resident[gpu].append((bpod, size))

    def plugin_latency(self, reset: bool = False) -> dict | None:
        """The plugin's own (server-side) Allocate latency quantiles from its metrics endpoint."""
        import urllib.request

        try:
            url = f"http://127.0.0.1:{self.metrics_port}/debug/latency" + ("?reset=1" if reset else "")
            with urllib.request.urlopen(url, timeout=5) as r:
                d = json.loads(r.read())
        except Exception:  # noqa: BLE001 - thread mode or endpoint unavailable
            return None
        for e in d.get("gpushare_allocate_latency_seconds", []):
            if e["labels"].get("phase") == "total":
                return e
        return None

    def placement(self) -> dict:
        from aliyun_gpushare_device_plugin_amd.cluster import objects as O

        return {g: [(O.uid(p), s) for p, s in pods] for g, pods in self.resident.items()}

    def stop(self):
        self.pool.shutdown(wait=True)
        self.cluster.stop()


def main():
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    n = a.gpus
    if world not in (1, n):
        raise SystemExit(f"WORLD_SIZE={world} but --gpus {n}")

    import torch
    import torch.distributed as dist

    use_gpu = torch.cuda.is_available() and not a.no_gpu
    if use_gpu:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local) if use_gpu else None
    if world > 1:
        dist.init_process_group("nccl" if use_gpu else "gloo", device_id=dev if use_gpu else None)

    def bcast(obj):
        if world == 1:
            return obj
        box = [obj]
        dist.broadcast_object_list(box, src=0)
        return box[0]

    def barrier():
        if world > 1:
            dist.barrier()
        if use_gpu:
            torch.cuda.synchronize()

    smi = a.smi_backend or ("auto" if use_gpu else f"fake:{n}x288G")
    cp = None
    info = None
    if rank == 0:
        if use_gpu and smi == "auto":
            from aliyun_gpushare_device_plugin_amd.device.smi import SMI
            with SMI("auto") as s:
                if s.count() < n:          # fewer visible GPUs than ranks: model the node
                    smi = f"fake:{n}x{s.device(0).vram_total}B"
        cp = ControlPlane(n, smi, a.pod_source, a.plugin_mode)
        info = {"units_per_gpu": cp.units_per_gpu, "gpu_count": cp.gpu_count}
    info = bcast(info)
    units = info["units_per_gpu"]

    players: dict[str, object] = {}
    gemm_flops = 0.0

    arena = None

    def sync_players(place):
        """Make this rank's players match the pods resident on its GPU."""
        if not use_gpu:
            return
        from aliyun_gpushare_device_plugin_amd.models.gemm_player import GemmPlayer, HBMArena

        nonlocal arena
        if arena is None:
            arena = HBMArena(dev, units)          # the GPU's shareable HBM, mapped once
        mine = dict(place.get(local, []))
        for uid in [u for u in players if u not in mine]:
            players.pop(uid).release()
            arena.free(uid)
        total = torch.cuda.get_device_properties(dev).total_memory
        for uid, size in mine.items():
            if uid not in players:
                players[uid] = GemmPlayer(total * size // units, dev, a.gemm, a.gemm, a.gemm,
                                          seed=hash(uid) & 0xffff, pool=arena.alloc(uid, size),
                                          fused_burst=a.burst_mode == "fused")

    def step(timed: bool):
        nonlocal gemm_flops
        for p in players.values():                  # traffic first: GPUs busy during admissions
            p.run(a.burst)
        if timed:
            gemm_flops += 2.0 * a.gemm ** 3 * a.burst * len(players)
        place = None
        if rank == 0:
            tc = time.perf_counter()
            cp.churn()
            if timed:
                cp.cp_time += time.perf_counter() - tc
            place = cp.placement()
        place = bcast(place)
        sync_players(place)
        for p in players.values():
            p.synchronize()

    # ---- warm-up: fill the node, then W untimed churn waves ----
    place = None
    if rank == 0:
        cp.fill()
        place = cp.placement()
    place = bcast(place)
    sync_players(place)
    for _ in range(a.warmup):
        step(False)
    if rank == 0:
        cp.alloc_lat.clear()
        cp.admit_lat.clear()
        cp.failed = 0
        cp.fail_reasons.clear()
        cp.plugin_latency(reset=True)

    barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(True)
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed, gemm_flops], dtype=torch.float64, device=dev if use_gpu else "cpu")
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        elapsed, gemm_flops = float(mx[0]), float(t[1])

    if rank == 0:
        srv = cp.plugin_latency()
        pods_node = sum(len(v) for v in cp.resident.values())
        gib_node = sum(s for v in cp.resident.values() for _, s in v)
        admissions = a.steps * n - cp.failed
        value = admissions / elapsed
        res = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "pod admissions/s",
            "n_gpus": n,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic pod specs (mixed 8-128 GiB), random-init bf16 GEMM operands",
            "config": {"model": "gpushare-device-plugin + MFMA GEMM pods (BASELINE config 3 churn)",
                       "global_batch": 4 * n, "seq_len": None, "parallelism": f"node{n}",
                       "pods_per_gpu": 4, "burst_gemms": a.burst, "burst_mode": a.burst_mode, "gemm_mnk": a.gemm,
                       "pod_source": a.pod_source, "smi_backend": smi},
            "allocate_p50_ms": round(pct(cp.alloc_lat, 0.5) * 1e3, 3) if cp.alloc_lat else None,
            "allocate_p99_ms": round(pct(cp.alloc_lat, 0.99) * 1e3, 3) if cp.alloc_lat else None,
            "admission_p50_ms": round(pct(cp.admit_lat, 0.5) * 1e3, 3) if cp.admit_lat else None,
            "plugin_allocate_p50_ms": round(srv["p50"] * 1e3, 3) if srv else None,
            "plugin_allocate_p99_ms": round(srv["p99"] * 1e3, 3) if srv else None,
            "control_plane_ms_per_step": round(cp.cp_time / a.steps * 1e3, 3),
            "pods_per_node": pods_node,
            "hbm_gib_per_node": gib_node,
            "advertised_gib_per_node": units * n,
            "packing_efficiency": round(gib_node / (units * n), 4) if units else None,
            "failed_admissions": cp.failed,
            "failure_reasons": cp.fail_reasons[:5],
            "gemm_tflops_node": round(gemm_flops / elapsed / 1e12, 1) if use_gpu else None,
        }
        line = json.dumps(res)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    for p in list(players.values()):
        p.release()
    if rank == 0:
        cp.stop()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
