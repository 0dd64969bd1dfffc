#!/usr/bin/env python3
"""Headline benchmark: bin-packed pods + HBM-GiB per node with Allocate latency, on 1/2/4/8 MI355X.

Metric (BASELINE.json): "bin-packed pods + HBM-GiB/node; Allocate p50 latency at 1/2/4/8 MI355X".

Scenario (one node with N = --gpus MI355X, one rank per GPU, rank 0 also hosts the control plane):
  * control plane = the real plugin (``gpushare-device-plugin`` in its own process, devices from
    librocm_smi/sysfs, quota shim injection, ledger dir, journal), a fake kube-apiserver, the
    extender bin-packer and the fake kubelet (gRPC over UDS) — the path pods take in production
    (sim/cluster.py);
  * every admitted pod becomes its own OS process (models/pod_worker.py), started with the
    Allocate response's env (quota, ledger, ROCR_VISIBLE_DEVICES) and the quota shim in
    LD_PRELOAD, exactly as the container runtime would start it; it holds 85 % of its quota
    (resident model state) and runs bf16 MFMA GEMM traffic (hand-written gfx950 kernel) until
    retired;
  * warm-up fills every GPU with 4 pods of mixed size 8-128 GiB summing to 288 GiB (BASELINE
    config 3: 32 pods on 8 GPUs) and runs W untimed churn waves;
  * each timed step = one churn cycle on every GPU while the other pods keep it busy: the
    oldest pod's process is stopped (the step waits until amdgpu, which wipes freed VRAM before
    returning it, reports room for a same-size pod), the pod
    is deleted, a same-size replacement is created, bin-packed by the extender, admitted by the
    kubelet through the plugin's Allocate, and its process starts under the shim and runs its
    first GEMM ("pod ready"). The interpreter of the replacement is pre-started (standby: torch
    imported, GPU untouched — an image already pulled; forked from one interpreter that imported
    torch once, so the pool does not take CPU from starting pods); HIP init, quota, HBM allocation and the
    first GEMM are inside the timed step. By default pods take their HBM from the GPU's HBM
    broker (native/hbmbroker, docs/HBM_TURNOVER.md): VMM granules lent per pod and scrubbed
    between pods, so an admission does not wait for amdgpu's wipe of the retired pod's HBM
    (--no-hbm-broker: fresh driver allocations, the wipe-bound path). Each GPU cycles independently (rank 0 serves the
    admissions, serialised like one kubelet); per-GPU work is fixed (1 admission per step), so
    scaling is weak.
``value`` = pods admitted-to-ready per second for the whole node (higher is better). Also in the
line: Allocate p50/p99 (kubelet-side gRPC round trip) and the plugin's server-side p50/p99; pod
ready p50; pods and GiB bin-packed per node; the aggregate GEMM TFLOP/s the pod processes
delivered during the timed window; quota denials; and a control-plane A/B at injected apiserver
RTTs of 1 and 5 ms: this build's default (watch cache + write-behind patch) against the
reference's cost model (LIST per Allocate + synchronous PATCH, ``allocate.go:63-152``).

python bench.py --gpus N --steps K --warmup W   (N>1: launched by torch.distributed.run)
"""
from __future__ import annotations

import argparse
import json
import os
import queue
import subprocess
import tempfile
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "bin-packed pods + HBM-GiB/node; Allocate p50 latency at 1/2/4/8 MI355X"
MAIN_NODE, REF_NODE = "mi355x-node", "ref-node"
# Per-GPU pod sizes (GiB), each pattern sums to one MI355X (288 GiB); GPU g uses pattern g % 4.
PATTERNS = [[128, 64, 64, 32], [96, 96, 64, 32], [128, 96, 56, 8], [64, 64, 96, 64]]
OVERSUB_SIZES = [8, 16, 32, 56, 64, 96, 128]     # GiB, the oversubscribed fill's size menu
NATIVE = os.path.join(ROOT, "aliyun_gpushare_device_plugin_amd", "_native")


def parse():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--burst", type=int, default=8, help="GEMMs between a pod process's control checks")
    ap.add_argument("--gemm", type=int, default=4096, help="GEMM M=N=K")
    ap.add_argument("--fill", type=float, default=0.85, help="fraction of its quota a pod process holds")
    ap.add_argument("--standby", type=int, default=9,
                    help="pre-started pod processes per GPU (images pulled, processes created, torch imported). "
                         "A fresh interpreter takes ~1.5 s of CPU (--no-pod-zygote), so the pool must cover the "
                         "admission rate: at ~3.5 pods/s per GPU a pool of 6 ran dry, up to 445 ms of waiting in a "
                         "step; 9 did not (profiles/r5/bench_n1_standby_ab/). Forked standbys take milliseconds")
    ap.add_argument("--no-pod-zygote", action="store_true",
                    help="start each standby as a fresh interpreter (~1.5 s of CPU each) instead of forking it "
                         "from one that imported torch once")
    ap.add_argument("--no-gpu", action="store_true", help="control plane only (CPU)")
    ap.add_argument("--smi-backend", default=None, help="default: auto on GPU, fake:Nx288G on CPU")
    ap.add_argument("--pod-source", default="watch", choices=("watch", "list", "kubelet"))
    ap.add_argument("--plugin-mode", default="process", choices=("process", "thread"))
    ap.add_argument("--compare-rtts", default="0,1,5", help="apiserver RTTs (ms) of the control-plane A/B ('' = off)")
    ap.add_argument("--compare-pods", type=int, default=24, help="admissions per A/B configuration")
    ap.add_argument("--no-ref-churn", action="store_true",
                    help="skip the reference-model node churned in lock-step with the real one")
    ap.add_argument("--fill-orders", default="grouped,random,size_desc,size_asc,burst_random,burst_size_asc,"
                                             "oversub,burst_oversub",
                    help="bin-pack stress: arrival orders of the node's mixed pods through the extender; burst_* = "
                         "all pods queued first, placed jointly ('' = off)")
    ap.add_argument("--room-slack-gib", type=float, default=2.0,
                    help="free HBM beyond a pod's state required before it allocates")
    ap.add_argument("--hbm-broker", action=argparse.BooleanOptionalAction, default=True,
                    help="pods take their HBM from a per-GPU broker (native/hbmbroker) instead of fresh driver "
                         "allocations: no wait for amdgpu's wipe of a retired pod's HBM (--no-hbm-broker: the "
                         "driver path; if the broker cannot start, the run falls back to it and says why)")
    ap.add_argument("--hbm-broker-reserve-gib", type=float, default=12.0,
                    help="HBM the broker leaves to the driver (runtimes' own allocations); the plugin grants each "
                         "pod 94 %% of its quota in whole GiB, 269-270 GiB for a GPU's 4 pods")
    ap.add_argument("--driver-path-steps", type=int, default=5,
                    help="after the timed run (1 GPU, broker on): this many churn steps of the driver path "
                         "(--no-hbm-broker) in a child run, reported as driver_path (0 = off)")
    ap.add_argument("--tenant-stop", default="cooperative", choices=("cooperative", "sigterm", "exit"),
                    help="how a retired pod's process ends: cooperative = it frees its HBM and hands its arena "
                         "back (gpushare_shim_arena_release) before it exits; sigterm = the kubelet's stop, SIGTERM "
                         "with the default action and nothing else; exit = its program ends (a normal exit, no "
                         "release call)")
    ap.add_argument("--comparator-steps", type=int, default=8,
                    help="after the timed run (1 GPU, broker on): this many churn steps each of an unmodified tenant "
                         "(--tenant-stop sigterm), of a normal exit (--tenant-stop exit) and of fresh standby "
                         "interpreters (--no-pod-zygote), in child runs, reported in the line (0 = off)")
    ap.add_argument("--stub-runtime", default=None,
                    help="CPU rehearsal of the broker path: a directory with the stub HIP runtime "
                         "(libamdhip64.so.7, tests/native/fake_hip.c), shim_driver and a gpushare-hbm-broker linked "
                         "against it; every rank runs a stub broker and its pods are stub processes under the real "
                         "quota shim that take their arenas from it")
    ap.add_argument("--comgr-cache", action=argparse.BooleanOptionalAction, default=True,
                    help="the DaemonSet's comgr cache (quota/comgr_cache.py): filled before the plugin starts, as its "
                         "init container does, and mounted read-only into every pod (--comgr-cache-dir)")
    ap.add_argument("--comgr-cache-dir", default=None, help="an already filled cache to use (the comparators' runs)")
    ap.add_argument("--reserved-cpus", type=int, default=0,
                    help="CPUs reserved for the device plugin, as a node reserves CPUs for its daemons (the kubelet's "
                         "reservedSystemCPUs): its watch threads and the native server's connection threads run there, "
                         "pod processes on the others; the simulated kubelet / apiserver are not pinned (0 = no "
                         "reservation, the default: on the test boxes, where a CPU quota and not a cpuset bounds the "
                         "job, 2 pinned CPUs cut the Allocates that wait for the watch to 1-2 of 20 but added one "
                         "0.9-5.8 ms transport stall per run, profiles/r6/allocate_tail.md)")
    ap.add_argument("--json-out", default=None)
    return ap.parse_args()


def pct(xs, q):
    if not xs:
        return None
    s = sorted(xs)
    return s[min(len(s) - 1, max(0, int(round(q * (len(s) - 1)))))]


def ms(x):
    return None if x is None else round(x * 1e3, 3)


def container_env(resp) -> dict:
    """The env a container runtime would give the pod's process: the Allocate response's envs
    with container paths (shim mount, ledger dir mount) mapped back to the host paths the
    response's mounts name."""
    env = dict(resp.envs)
    mounts = sorted(((m.container_path, m.host_path) for m in resp.mounts), key=lambda m: -len(m[0]))
    for k, v in list(env.items()):
        for cpath, hpath in mounts:
            if v == cpath or v.startswith(cpath.rstrip("/") + "/"):
                env[k] = hpath + v[len(cpath.rstrip("/")):]
                break
    return env


def free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def plugin_latency(port: int, reset: bool = False) -> dict | None:
    """The plugin's own (server-side) Allocate latency quantiles from its metrics endpoint."""
    import urllib.request

    try:
        url = f"http://127.0.0.1:{port}/debug/latency" + ("?reset=1" if reset else "")
        with urllib.request.urlopen(url, timeout=5) as r:
            d = json.loads(r.read())
    except Exception:  # noqa: BLE001 - thread mode or endpoint unavailable
        return None
    phases = {e["labels"].get("phase"): e for e in d.get("gpushare_allocate_latency_seconds", [])}
    tot = phases.get("total")
    if tot is not None:
        tot = dict(tot, phases={k: v.get("p50") for k, v in phases.items()})
        # apiserver round trips the handler itself made, per Allocate (measured, not assumed)
        rq = (d.get("gpushare_allocate_apiserver_requests") or [{}])[0]
        tot["requests"] = {"p50": rq.get("p50"), "p99": rq.get("p99"), "count": rq.get("count")}
    pub = {e["labels"].get("path"): e for e in d.get("gpushare_native_table_publish_seconds", [])}
    if tot is not None and pub:
        # the native table: how long the watch-thread hook (one pod) and a full rebuild take
        tot["table_publish"] = {k: {"p50_ms": round(v["p50"] * 1e3, 3), "count": v["count"]} for k, v in pub.items()}
    return tot


def native_stats(port: int) -> dict | None:
    """The native server's counters (plugin metrics endpoint)."""
    import urllib.request

    try:
        with urllib.request.urlopen(f"http://127.0.0.1:{port}/debug/latency", timeout=5) as r:
            return json.loads(r.read()).get("native_server")
    except Exception:  # noqa: BLE001
        return None


def native_share(before: dict | None, after: dict | None) -> dict | None:
    """Allocates the native server answered from the prepared table vs handed to the engine,
    between two readings of its counters, and why it declined."""
    b, a = before or {}, after or {}
    if not a:
        return None
    fast = a.get("fast", 0) - b.get("fast", 0)
    eng = a.get("forwarded_allocate", 0) - b.get("forwarded_allocate", 0)
    why = {k: v - (b.get("declined") or {}).get(k, 0) for k, v in (a.get("declined") or {}).items()}
    return {"native": fast, "engine": eng, "declined": {k: v for k, v in why.items() if v},
            "waited_for_table": a.get("waited", 0) - b.get("waited", 0),
            "waited_for_watch": a.get("watch_waits", 0) - b.get("watch_waits", 0),
            "table_wait_mean_ms": round((a.get("wait_ns", 0) - b.get("wait_ns", 0)) / 1e6
                                        / max(1, a.get("waited", 0) - b.get("waited", 0)), 3),
            # inside a native answer (mean over the answers): taking the server lock, the journal
            # record, and request-complete -> reply (all of the server's own time)
            "native_answer_mean_us": {k: round((a.get(f"{k}_ns", 0) - b.get(f"{k}_ns", 0)) / 1e3 / max(1, fast), 1)
                                      for k in ("lock", "journal", "answer")},
            "table_hook_skipped": {k: v - (b.get("table_hook_skipped") or {}).get(k, 0)
                                   for k, v in (a.get("table_hook_skipped") or {}).items()},
            # engine-state changes that retired the prepared table (each makes the next Allocates
            # wait for a rebuild), by cause
            "gen_bumps": {k: v - (b.get("gen_bumps") or {}).get(k, 0)
                          for k, v in (a.get("gen_bumps") or {}).items()
                          if k != "last_fixes" and v - (b.get("gen_bumps") or {}).get(k, 0)},
            # the placement fixes behind them (the plugin's last 16, newest last)
            "placement_fixes": [f for f in (a.get("gen_bumps") or {}).get("last_fixes", [])
                                if f not in (b.get("gen_bumps") or {}).get("last_fixes", [])],
            # the plugin's cyclic-GC collections in the window, by generation, and their time
            # (plugin/manager.py time_gc; max_us is over the plugin's life)
            "plugin_gc": _gc_delta(b.get("gc"), a.get("gc"))}


def _gc_delta(b: dict | None, a: dict | None) -> dict | None:
    if not a:
        return None
    b = b or {"collections": [0, 0, 0], "ns": [0, 0, 0]}
    return {"collections": [x - y for x, y in zip(a["collections"], b["collections"])],
            "us": [round((x - y) / 1e3, 1) for x, y in zip(a["ns"], b["ns"])],
            "max_us": round(a.get("max_ns", 0) / 1e3, 1)}


def pod_timeline(port: int, commits: dict) -> dict | None:
    """Where each timed pod's Allocate fell in its pod's timeline (ms relative to the Allocate's
    arrival at the plugin; CLOCK_MONOTONIC, shared by the node's processes): the extender's
    commit (annotate+label PATCH, then bind), the plugin's pre-bind watch delivering the placed
    pod and its table entry going live, the pod watch delivering the bind. The pods that waited
    for the plugin's watch are listed whole, with the step that was still missing."""
    import urllib.request

    try:
        with urllib.request.urlopen(f"http://127.0.0.1:{port}/debug/latency", timeout=5) as r:
            trace = json.loads(r.read()).get("pod_trace") or []
    except Exception:  # noqa: BLE001
        return None
    rows = []
    for t in trace:
        c = commits.get(t["uid"])
        if c is None:
            continue
        row = dict(t)
        tin = t.get("alloc_in_abs")                    # (the plugin's rows are relative already)
        if tin is not None:
            row["commit_start"] = round((c[0] - tin) / 1e6, 3)
            row["commit_done"] = round((c[1] - tin) / 1e6, 3)
        rows.append(row)
    if not rows:
        return None

    def med(k):
        xs = sorted(r[k] for r in rows if isinstance(r.get(k), (int, float)))
        return xs[len(xs) // 2] if xs else None

    # the pre-bind path's steps: wall time and this thread's CPU time (wall - CPU = waiting for
    # the interpreter lock or a CPU), medians in us
    steps = {}
    seq = ("pre_seen", "prep_ledger", "prep_hbm", "pre_prep", "pre_pub")
    for a_, b_ in zip(seq, seq[1:]):
        wall = sorted((r[b_] - r[a_]) * 1e3 for r in rows if isinstance(r.get(a_), (int, float)) and isinstance(r.get(b_), (int, float)))
        cpu = sorted((r[b_ + "_cpu_ns"] - r[a_ + "_cpu_ns"]) / 1e3 for r in rows
                     if r.get(a_ + "_cpu_ns") is not None and r.get(b_ + "_cpu_ns") is not None)
        if wall:
            steps[f"{a_}->{b_}"] = {"wall_us": round(wall[len(wall) // 2], 1),
                                    "cpu_us": round(cpu[len(cpu) // 2], 1) if cpu else None}
    waited = [r for r in rows if r.get("watch_wait_ns")]
    table_waited = [r for r in rows if r.get("table_wait_ns") and not r.get("watch_wait_ns")]
    causes: dict = {}
    for r in waited:
        if r.get("pre_pub") is not None and r["pre_pub"] <= 0:
            why = "prebind_entry_live"                 # (a size or order mismatch, not the watch)
        elif r.get("pre_seen") is None or r["pre_seen"] > 0:
            why = "prebind_event_after_allocate"       # the plugin had not read the placed pod yet
        elif r.get("pre_pub") is None:
            why = "prebind_not_published:" + ",".join(k[4:] for k in r if k.startswith("pre_") and k not in ("pre_seen", "pre_prep"))
        else:
            why = "prebind_publish_after_allocate"     # read, still preparing / publishing
        causes[why] = causes.get(why, 0) + 1
    keys = ("commit_start", "commit_done", "pre_read", "pre_seen", "prep_ledger", "prep_hbm", "pre_prep", "pre_pub",
            "bind_seen", "bind_pub", "tab")
    def whole(r):        # every mark of the pod (a pre_<reason> names why its pre-bind entry was not published)
        extra = tuple(k for k in r if k.startswith("pre_") and k not in keys and not k.endswith("_cpu_ns"))
        return {k: r.get(k) for k in keys + extra + ("watch_wait_ns", "table_wait_ns", "path") if r.get(k) is not None}

    return {"pods": len(rows), "watch_waited": len(waited), "causes": causes, "prebind_steps": steps,
            "median_ms": {k: med(k) for k in keys},
            "waited": [whole(r) for r in waited],
            # Allocates that found the pod but waited for its table entry (an answer being re-prepared)
            "table_waited": [whole(r) for r in table_waited]}


def transport_floor() -> float | None:
    """Kubelet-side round trip of an Allocate whose handler returns a prepared answer at once."""
    try:
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "grpc_server_probe.py"), "--models", "sync",
                            "--busy-threads", "0", "--calls", "200", "--gap-ms", "5"],
                           capture_output=True, text=True, timeout=120)
        return json.loads(r.stdout.strip().splitlines()[-1])["sync"]["p50_ms"]
    except Exception:  # noqa: BLE001 - a calibration, never fatal
        return None


def breakdown(splits) -> dict | None:
    """p50 of each leg of the kubelet-side Allocate round trip (ms): kubelet -> handler entry
    (gRPC client, transport, server dispatch), the handler, handler exit -> kubelet (reply
    serialisation, transport, client wake-up) — from the handler's own timestamps."""
    if not splits:
        return None
    return {k: ms(pct([x[i] for x in splits], 0.5))
            for i, k in enumerate(("kubelet_to_handler", "handler", "handler_to_kubelet"))}


def round_trips(srv) -> dict | None:
    """The plugin's own count of apiserver requests on its Allocate path (p50 / p99)."""
    rq = (srv or {}).get("requests") or {}
    return None if rq.get("p50") is None else {"p50": rq["p50"], "p99": rq["p99"]}


class ControlPlane:
    """Rank 0's view of the node: fake cluster + the real plugin process."""

    def __init__(self, n_gpus: int, smi_spec: str, pod_source: str, plugin_mode: str, workdir: str,
                 with_shim: bool, ref_spec: str | None = None, hbm_dir: str | None = None,
                 comgr_dir: str | None = None, daemon_cpus: dict | None = None):
        from aliyun_gpushare_device_plugin_amd.sim.cluster import SimCluster

        self.n = n_gpus
        self.metrics_port = free_port()         # the plugin's metrics endpoint
        self.ledger_dir = os.path.join(workdir, "ledgers")
        os.makedirs(self.ledger_dir, exist_ok=True)
        extra = ["--metrics-addr", f"127.0.0.1:{self.metrics_port}"] if plugin_mode == "process" else []
        extra += ["--ledger-dir", self.ledger_dir, "--journal-path", os.path.join(workdir, "alloc-journal.jsonl")]
        if with_shim:
            extra += ["--rocr-visible-devices"]
        if hbm_dir:
            # the plugin grants every pod its broker granules while it prepares the pod's answer
            extra += ["--hbm-broker-dir", hbm_dir]
        if comgr_dir:
            extra += ["--comgr-cache-dir", comgr_dir]       # the init container's cache, read-only in pods
        nodes = [(MAIN_NODE, smi_spec)]
        overrides = {}
        # the reference's cost model (LIST per Allocate + synchronous PATCH, allocate.go:63-152)
        # on a second, modelled node of the same shape, churned in lock-step with the real one so
        # both plugins are measured under the same pod load (control plane only: no processes)
        self.ref_port = None
        if ref_spec and plugin_mode == "process":
            self.ref_port = free_port()
            nodes.append((REF_NODE, ref_spec))
            overrides[REF_NODE] = {"pod_source": "list", "extra_args": [
                "--sync-patch", "--metrics-addr", f"127.0.0.1:{self.ref_port}", "--pod-resources-socket", "none"]}
        self.cluster = SimCluster(nodes, plugin_mode=plugin_mode, pod_source=pod_source,
                                  apiserver="process", kubelet="process", gpu_indices=list(range(n_gpus)), health_poll_s=5.0,
                                  extra_plugin_args=extra, shim_host_dir=NATIVE if with_shim else None,
                                  node_overrides=overrides, daemon_cpus=daemon_cpus)
        self.cluster.start()
        from aliyun_gpushare_device_plugin_amd import const
        from aliyun_gpushare_device_plugin_amd.cluster import objects as O

        node = self.cluster.client.get_node(MAIN_NODE)
        self.gpu_count = O.node_allocatable(node, const.RESOURCE_COUNT)
        self.units_per_gpu = O.node_allocatable(node, const.RESOURCE_NAME) // max(1, self.gpu_count)
        if self.gpu_count != n_gpus:
            raise RuntimeError(f"plugin advertises {self.gpu_count} GPUs, expected {n_gpus}")
        self.resident: dict[int, list] = {g: [] for g in range(n_gpus)}   # gpu -> [(pod, size)] oldest first
        import concurrent.futures as cf

        self.pool = cf.ThreadPoolExecutor(max_workers=max(1, n_gpus), thread_name_prefix="churn")
        self._sched_lock = threading.Lock()
        self._kubelet = threading.Condition()
        self.alloc_lat: list[float] = []
        self.alloc_lat_by_gpu: dict[int, list] = {g: [] for g in range(n_gpus)}
        self.ref_resident: dict[int, list] = {g: [] for g in range(n_gpus)}
        self.ref_lat: list[float] = []
        self.ref_splits: list = []
        self.splits: list = []
        self.steps_done = 0                     # alternates which node is admitted first
        self.mirror_s: list = []                # the reference-model node's step inside each churn step
        self.ref_failed = 0
        self.admit_lat: list[float] = []
        self.failed = 0
        self.fail_reasons: list[str] = []
        self.cp_time = 0.0
        self.commit_ns: dict[str, tuple] = {}    # uid -> CLOCK_MONOTONIC ns around the extender's commit

    def _record(self, pod, size, adm) -> tuple[int, dict] | None:
        from aliyun_gpushare_device_plugin_amd.cluster import objects as O

        gpu = int(dict(adm.responses[0].envs)["ALIYUN_COM_GPU_MEM_IDX"])
        if gpu < 0:
            return None
        self.resident[gpu].append((pod, size))
        return gpu, {"uid": O.uid(pod), "size": size, "env": container_env(adm.responses[0])}

    def fill(self) -> dict:
        """Pods arrive as per-GPU-sized groups (think one StatefulSet per 288 GiB of demand), in
        pattern order. The extender's online best-fit places each group exactly onto one GPU, so
        the node packs 100 %; the same 32 pods in globally size-sorted order strand 56 GiB under
        that policy (31 of 32 placed at N = 8: its tie-break stacks two 128 GiB pods per GPU)."""
        started: dict[int, list] = {g: [] for g in range(self.n)}
        for g in range(self.n):
            for s in PATTERNS[g % len(PATTERNS)]:
                pod, where, adm = self.cluster.run_pod(s, node_names=[MAIN_NODE])
                if where is None or adm is None or adm.error:
                    self.failed += 1
                    continue
                rec = self._record(pod, s, adm)
                if rec:
                    started[rec[0]].append(rec[1])
                if self.ref_port:
                    rpod, rwhere, radm = self.cluster.run_pod(s, node_names=[REF_NODE])
                    if rwhere is not None and radm is not None and not radm.error:
                        rg = int(dict(radm.responses[0].envs)["ALIYUN_COM_GPU_MEM_IDX"])
                        if rg >= 0:
                            self.ref_resident[rg].append((rpod, s))
        return started

    def _mirror(self, gpu: int, size: int) -> None:
        """The same churn step on the reference-model node: retire its oldest ``size`` pod
        (preferring GPU ``gpu``) and admit a same-size replacement through its plugin."""
        t0 = time.perf_counter()
        try:
            self._mirror_step(gpu, size)
        finally:
            self.mirror_s.append(time.perf_counter() - t0)

    def _mirror_step(self, gpu: int, size: int) -> None:
        cands = [(g, i) for g in [gpu] + [x for x in range(self.n) if x != gpu]
                 for i, (_, sz) in enumerate(self.ref_resident[g]) if sz == size]
        if not cands:
            return
        g, i = cands[0]
        old, _ = self.ref_resident[g].pop(i)
        self.cluster.delete_pod(old)
        pod = self.cluster.create_pod(size)
        where = self.cluster.extender.decide(pod, [REF_NODE])
        bpod = self.cluster.extender.commit(pod, where, time.time_ns()) if where else None
        if bpod is None:
            self.ref_failed += 1
            return
        adm = self.cluster.admit(bpod, async_status=True)
        rg = int(dict(adm.responses[0].envs)["ALIYUN_COM_GPU_MEM_IDX"]) if adm.error is None and adm.responses else -1
        if rg < 0:
            self.ref_failed += 1
            self.cluster.delete_pod(bpod)
            return
        self.ref_lat.extend(adm.latencies)
        self.ref_splits.extend(adm.splits)
        self.ref_resident[rg].append((bpod, size))

    def churn_one(self, gpu: int, uid: str | None = None) -> tuple[int, dict] | None:
        """Retire pod ``uid`` (default: the oldest) of ``gpu`` and admit a same-size replacement
        through delete (controller) -> create -> extender decide + bind (assume time stamped at
        the decision) -> kubelet admission (Allocate over gRPC). Serialised by the caller, as the
        scheduler's cycle and the kubelet's admissions are. The replacement lands where the
        extender's best fit puts it — the freed exact-fit hole on ``gpu``, or an equal hole
        another GPU freed at the same time. Returns (landed gpu, pod record) or None."""
        from aliyun_gpushare_device_plugin_amd.cluster import objects as O

        pods = self.resident[gpu]
        k = next((i for i, (p, _) in enumerate(pods) if uid is None or O.uid(p) == uid), None)
        if k is None:
            return None
        old, size = pods.pop(k)
        # the same churn step on the reference-model node, first on every other step: neither
        # node always admits right after a retired pod's teardown started
        self.steps_done += 1
        mirror_first = self.ref_port and self.steps_done % 2 == 0
        if mirror_first:
            self._mirror(gpu, size)
        tc = time.perf_counter()
        self.cluster.delete_pod(old)
        pod = self.cluster.create_pod(size)
        where = self.cluster.extender.decide(pod, [MAIN_NODE])
        c0 = time.monotonic_ns()
        bpod = self.cluster.extender.commit(pod, where, time.time_ns()) if where else None
        if bpod is not None:
            self.commit_ns[O.uid(bpod)] = (c0, time.monotonic_ns())   # annotate+label PATCH, then bind
        if bpod is None:
            self.failed += 1
            self.fail_reasons.append(f"{size}GiB: unschedulable")
            self.cp_time += time.perf_counter() - tc
            return None
        t0 = time.perf_counter()
        adm = self.cluster.admit(bpod, async_status=True)
        dt = time.perf_counter() - t0
        rec = self._record(bpod, size, adm) if adm.error is None else None
        self.cp_time += time.perf_counter() - tc
        if rec is None:
            self.failed += 1
            self.fail_reasons.append(f"{size}GiB: " + (f"admit: {adm.error}" if adm.error else "plugin found no candidate"))
            self.cluster.delete_pod(bpod)
            return None
        self.alloc_lat.extend(adm.latencies)
        self.alloc_lat_by_gpu[rec[0]].extend(adm.latencies)
        self.splits.extend(adm.splits)
        self.admit_lat.append(dt)
        if self.ref_port and not mirror_first:
            self._mirror(gpu, size)          # alternating admissions, same pod load
        return rec

    def plugin_latency(self, reset: bool = False) -> dict | None:
        return plugin_latency(self.metrics_port, reset)

    def stop(self):
        self.pool.shutdown(wait=True)
        self.cluster.stop()


def mode_comparison(rtts_ms: list[float], n_pods: int) -> dict:
    """Control-plane A/B at injected apiserver RTTs: this build's default (watch cache +
    write-behind ASSIGNED patch) vs the reference's cost model (LIST of the node's Pending pods
    per Allocate + synchronous PATCH before answering, ``allocate.go:63-152``). Kubelet-side
    Allocate latency over ``n_pods`` sequential admissions of 8 GiB pods per configuration."""
    from aliyun_gpushare_device_plugin_amd.sim.cluster import SimCluster

    out = {}
    runs = [(rtt, label, src, extra, "native") for rtt in rtts_ms
            for label, src, extra in (("default", "watch", []), ("reference", "list", ["--sync-patch"]))]
    if 0.0 in rtts_ms:
        # calibration: the same quiet A/B measured by a Python grpcio kubelet client (the client
        # of rounds 1-3; the real kubelet's is compiled grpc-go)
        runs += [(0.0, label + "+grpcio_client", src, extra, "python")
                 for label, src, extra in (("default", "watch", []), ("reference", "list", ["--sync-patch"]))]
    for rtt, label, src, extra, client in runs:
        lat, fails, splits = [], 0, []
        port = free_port()
        os.environ["GS_SIM_KUBELET_CLIENT"] = client          # inherited by the kubelet process
        with SimCluster([("cmp", "fake:1x288G")], plugin_mode="process", pod_source=src,
                        apiserver="process", kubelet="process", apiserver_latency_s=rtt / 1e3,
                        extra_plugin_args=extra + ["--metrics-addr", f"127.0.0.1:{port}"]) as c:
            req = []                                 # one apiserver round trip, as the plugin sees it
            for _ in range(10):
                t = time.perf_counter()
                c.client.get_node("cmp")
                req.append(time.perf_counter() - t)
            for _ in range(n_pods):
                pod, where, adm = c.run_pod(8)
                if adm is None or adm.error or int(dict(adm.responses[0].envs)["ALIYUN_COM_GPU_MEM_IDX"]) < 0:
                    fails += 1
                else:
                    lat += adm.latencies
                    splits += adm.splits
                c.delete_pod(pod)
            srv = plugin_latency(port) or {}
        os.environ.pop("GS_SIM_KUBELET_CLIENT", None)
        key = f"{label}@{rtt:g}ms"
        # apiserver round trips on the Allocate path: LIST + PATCH (reference), none (default:
        # watch-cache lookup, PATCH written behind); request_ms = one round trip through the
        # fake apiserver at this RTT (RTT + the fake's own ~1.5 ms per-request cost)
        # plugin_* = the plugin's own handler time (its metrics endpoint): the rest of the
        # kubelet-side number is gRPC transport and the harness's processes sharing the CPUs
        out[key] = {"allocate_p50_ms": ms(pct(lat, 0.5)), "allocate_p99_ms": ms(pct(lat, 0.99)),
                    "plugin_allocate_p50_ms": ms(srv.get("p50")), "plugin_allocate_p99_ms": ms(srv.get("p99")),
                    "allocate_breakdown_p50_ms": breakdown(splits),
                    "apiserver_round_trips_on_path": round_trips(srv), "request_ms": ms(pct(req, 0.5)),
                    "pod_source": src, "patch": "sync" if extra else "write-behind", "failed": fails}
    return out


def fill_orders(orders: list[str], n_gpus: int, units: int, seed: int = 0) -> dict:
    """Bin-pack stress (BASELINE config 3, control plane only): the node's 4·N mixed pods
    (``PATTERNS``, 8-128 GiB, summing to exactly the node's HBM) arrive in a given order
    through the extender's online best fit and the plugin's Allocate. ``grouped`` = per-GPU
    groups (the churn's fill: packs by construction); ``random`` = one seeded shuffle;
    ``size_desc`` / ``size_asc`` = sorted — each pod scheduled as it arrives (online best fit);
    ``burst_<order>`` = the same arrival order, but all pods are queued before the scheduler
    runs, so the extender places the queue jointly (``extender/packing.py``). Reports pods and GiB
    placed, the node's HBM left stranded when a pod could not be placed, and failed placements."""
    import random

    from aliyun_gpushare_device_plugin_amd.sim.cluster import SimCluster

    import random as _random

    sizes = [s for g in range(n_gpus) for s in PATTERNS[g % len(PATTERNS)]]
    cap = units * n_gpus
    # oversubscribed mix: seeded sizes that do not sum to an exact fit, drawn until the demand
    # is 125 % of the node's HBM (the demo's bin-pack workload at MI355X scale)
    rng = _random.Random(seed + 1)
    over: list[int] = []
    while sum(over) < 1.25 * cap:
        over.append(rng.choice(OVERSUB_SIZES))
    out = {}
    for order in orders:
        burst = order.startswith("burst_")
        base = order[len("burst_"):] if burst else order
        seq = list(over if base == "oversub" else sizes)
        if base == "oversub":
            pass                                      # arrival order = the seeded draw order
        elif base == "random":
            random.Random(seed).shuffle(seq)
        elif base == "size_desc":
            seq.sort(reverse=True)
        elif base == "size_asc":
            seq.sort()
        elif base != "grouped":
            raise ValueError(f"fill order {order!r}")
        placed, failed, admit_fail = [], 0, 0
        with SimCluster([("fill", f"fake:{n_gpus}x288G")], plugin_mode="thread", apiserver="thread",
                        kubelet="thread") as c:
            queued = [c.create_pod(sz) for sz in seq] if burst else []
            for k, sz in enumerate(seq):
                if burst:
                    pod = queued[k]
                    where = c.schedule(pod)
                    adm = c.admit(pod) if where else None
                else:
                    pod, where, adm = c.run_pod(sz)
                if where is None:
                    failed += 1
                elif adm is None or adm.error or int(dict(adm.responses[0].envs)["ALIYUN_COM_GPU_MEM_IDX"]) < 0:
                    admit_fail += 1
                else:
                    placed.append(sz)
        gib = sum(placed)
        out[order] = {"pods_placed": len(placed), "pods_total": len(seq), "gib_placed": gib,
                      "packing_efficiency": round(gib / cap, 4) if units else None,
                      "stranded_gib": cap - gib if failed or admit_fail else 0,
                      "failed_placements": failed, "failed_admissions": admit_fail}
        if base == "oversub":
            out[order]["demand_gib"] = sum(seq)
    return out


class AdmissionService:
    """Rank 0's admission endpoint for the per-GPU churn pipelines: ``churn(gpu, uid)`` retires a
    pod and admits its replacement, then returns the next pod that landed on ``gpu`` (each
    retirement opens one exact-fit hole and each admission fills one, so every waiting GPU gets
    a pod). Ranks > 0 reach it over a loopback TCP socket (one JSON line per request)."""

    def __init__(self, cp: ControlPlane):
        self.cp = cp
        self.lock = threading.Lock()                        # one admission at a time, like the kubelet
        self.mail = {g: queue.Queue() for g in range(cp.n)}
        self.server = None

    def churn(self, gpu: int, uid: str | None) -> dict | None:
        with self.lock:
            landed = self.cp.churn_one(gpu, uid)
        if landed is None:
            return None
        self.mail[landed[0]].put(landed[1])
        return self.mail[gpu].get(timeout=300)

    def serve(self) -> int:
        import socketserver

        svc = self

        class H(socketserver.StreamRequestHandler):
            def handle(self):
                for ln in self.rfile:
                    req = json.loads(ln)
                    rec = svc.churn(req["gpu"], req.get("uid"))
                    self.wfile.write((json.dumps({"rec": rec}) + "\n").encode())
                    self.wfile.flush()

        class Srv(socketserver.ThreadingTCPServer):
            daemon_threads = True
            allow_reuse_address = True

        self.server = Srv(("127.0.0.1", 0), H)
        threading.Thread(target=self.server.serve_forever, daemon=True).start()
        return self.server.server_address[1]

    def stop(self):
        if self.server is not None:
            self.server.shutdown()
            self.server.server_close()


class AdmissionClient:
    def __init__(self, port: int):
        import socket

        self.sock = socket.create_connection(("127.0.0.1", port))
        self.f = self.sock.makefile("rw")

    def churn(self, gpu: int, uid: str | None) -> dict | None:
        self.f.write(json.dumps({"gpu": gpu, "uid": uid}) + "\n")
        self.f.flush()
        return json.loads(self.f.readline())["rec"]

    def close(self):
        self.sock.close()


class _Forked:
    """A pod process the zygote forked: the part of ``subprocess.Popen`` the fleet uses. It is
    the zygote's child, so it is watched through a pidfd; its exit status is not known here."""

    def __init__(self, pid: int, stdin, stdout):
        self.pid, self.stdin, self.stdout = pid, stdin, stdout
        self.returncode = None
        try:
            self._pidfd = os.pidfd_open(pid)
        except ProcessLookupError:
            self._pidfd, self.returncode = None, 0

    def _exited(self, timeout) -> bool:
        import select

        if self._pidfd is None:
            return True
        r, _, _ = select.select([self._pidfd], [], [], timeout)
        if r:
            os.close(self._pidfd)
            self._pidfd, self.returncode = None, 0
        return bool(r)

    def poll(self):
        self._exited(0)
        return self.returncode

    def wait(self, timeout=None):
        if not self._exited(timeout):
            raise subprocess.TimeoutExpired(f"pod {self.pid}", timeout)
        return self.returncode

    def kill(self):
        try:
            os.kill(self.pid, 9)
        except ProcessLookupError:
            pass

    def terminate(self):
        try:
            os.kill(self.pid, 15)
        except ProcessLookupError:
            pass


class _Zygote:
    """One interpreter that imported torch and forks the standby pod processes
    (``pod_worker.zygote``): keeping the pool full costs a fork per pod, not a torch import
    (~1.5 s of CPU) taken from the pods that are starting at the same time."""

    def __init__(self, env: dict):
        import socket

        self._sock, theirs = socket.socketpair(socket.AF_UNIX, socket.SOCK_STREAM)
        self._proc = subprocess.Popen([sys.executable, "-m", "aliyun_gpushare_device_plugin_amd.models.pod_worker",
                                       "--zygote", str(theirs.fileno())], env=env, pass_fds=(theirs.fileno(),),
                                      stdin=subprocess.DEVNULL, stdout=subprocess.DEVNULL)
        theirs.close()
        self._sock.settimeout(120)      # a fork answers in milliseconds; the first waits for the torch import
        self._rd = self._sock.makefile("r")
        self._lock = threading.Lock()

    def fork(self) -> _Forked:
        import socket

        c_in, p_in = os.pipe()          # the pod reads its commands from c_in
        p_out, c_out = os.pipe()        # and writes its events to c_out
        line = ""
        try:
            with self._lock:
                socket.send_fds(self._sock, [b"F"], [c_in, c_out])
                line = self._rd.readline()
        finally:
            os.close(c_in)
            os.close(c_out)
            if not line:                # no child: nothing will read or write the other ends
                os.close(p_in)
                os.close(p_out)
        if not line:
            raise RuntimeError(f"the pod zygote exited (status {self._proc.poll()})")
        return _Forked(int(line), os.fdopen(p_in, "w", buffering=1), os.fdopen(p_out, "r"))

    def close(self):
        try:
            self._rd.close()                # the socket's fd closes with its last file object
            self._sock.close()
            self._proc.wait(30)
        except Exception:  # noqa: BLE001
            self._proc.kill()
            self._proc.wait(10)


class PodFleet:
    pod_cpus = ""          # GS_POD_CPUS for every pod process (cpu_split)

    """The pod processes of this rank's GPU, plus one standby process (interpreter up, torch
    imported, GPU untouched) that becomes the next admitted pod."""

    def __init__(self, local: int, gemm: int, burst: int, fill: float, visible_by_uuid: bool, standby: int = 2,
                 slack: int = 2 << 30, ordinal: int | None = None, broker=None, zygote: bool = True,
                 stop_mode: str = "cooperative"):
        self.local, self.gemm, self.burst, self.fill, self.slack = local, gemm, burst, fill, slack
        self.stop_mode = stop_mode            # how a retired pod's process ends (--tenant-stop)
        self._zygote = _Zygote(self._pod_env()) if zygote else None
        self.broker = broker                  # HBMBroker: pods' HBM comes from it (no driver wipe on the path)
        self.ordinal = local if ordinal is None else ordinal     # this GPU's HIP ordinal (bind_device)
        self.visible_by_uuid = visible_by_uuid
        self.pods: dict[str, dict] = {}       # uid -> {"proc", "q", "size", "ready"}
        self.standby: list[dict] = []         # pre-started interpreters, oldest first
        self.ready_ms: list[float] = []
        self.slowest: dict = {}
        self.retired_gemms = 0
        self.denied = 0
        self.held_bytes = 0
        self.released_residue = 0             # shim-ledger bytes a stopped pod still held after freeing
        self.release_ms: list[float] = []     # stop -> the GPU physically has room for the replacement
        self.release_by_size: dict[int, list] = {}
        self.release_bytes_s: list[tuple] = [] # (retired pod's bytes, stop -> room back seconds)
        self.retired_bytes = 0                 # HBM the retired pods held (turned over by amdgpu)
        self._stopped_at = None                # (time, size, held bytes) of the last retirement, until its room came back
        self.phase_ms: dict[str, list] = {"stop": [], "init": [], "room": [], "alloc": [], "hold": []}
        self.trace: list | None = [] if os.environ.get("GS_BENCH_POD_TRACE") else None
        self._vram_used, self._vram_total = self._vram_reader()
        if broker is not None:
            self._vram_used = None            # the broker's TAKE waits for the granules, not for the driver
        for _ in range(max(1, standby)):
            self._spawn()

    def _vram_reader(self):
        """(reader of amdgpu's used-VRAM count for this rank's GPU, its total VRAM) from sysfs, or
        (None, 0)."""
        try:
            from aliyun_gpushare_device_plugin_amd.device.smi import SMI

            with SMI("auto") as s:
                minor = s.device(self.local).render_minor if s.count() > self.local else -1
        except Exception:  # noqa: BLE001
            return None, 0
        base = f"/sys/class/drm/renderD{minor}/device/mem_info_vram_"
        if minor < 0 or not os.path.exists(base + "used"):
            return None, 0
        with open(base + "total") as f:
            total = int(f.read())

        def read():
            with open(base + "used") as f:
                return int(f.read())
        return read, total

    @staticmethod
    def _pod_env() -> dict:
        # the shim first; whatever this process already preloads (a profiler, the host's own
        # libraries) stays preloaded in the pods too
        # (and the comgr action cache, as answers preload it: inert unless the answer's env turns
        # it on, i.e. the plugin mounts a comgr cache)
        cc = os.path.join(NATIVE, "libgpushare_comgrcache.so")
        pre = ":".join(x for x in (os.path.join(NATIVE, "libgpushare_hipquota.so"), cc if os.path.exists(cc) else "",
                                   os.environ.get("LD_PRELOAD", "")) if x)
        env = dict(os.environ, LD_PRELOAD=pre,
                   PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""), GS_POD_NICE="5")
        if PodFleet.pod_cpus:
            env["GS_POD_CPUS"] = PodFleet.pod_cpus       # not the CPUs reserved for the node's daemons
        for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
                  "TORCHELASTIC_RUN_ID", "GROUP_RANK", "ROLE_RANK"):
            env.pop(k, None)
        return env

    def _spawn(self):
        if self._zygote is not None:
            p = self._zygote.fork()
        else:
            p = subprocess.Popen([sys.executable, "-m", "aliyun_gpushare_device_plugin_amd.models.pod_worker"],
                                 env=self._pod_env(), stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True,
                                 bufsize=1)
        q: "queue.Queue" = queue.Queue()

        def pump():
            for ln in p.stdout:
                if ln.startswith("{"):
                    q.put(json.loads(ln))
            q.put({"event": "eof"})

        threading.Thread(target=pump, daemon=True).start()
        self.standby.append({"proc": p, "q": q})

    @staticmethod
    def _wait(w, event, timeout=120.0):
        while True:
            ev = w["q"].get(timeout=timeout)
            if ev.get("event") == event:
                return ev
            if ev.get("event") == "eof":
                raise RuntimeError(f"pod process {w['proc'].pid} exited while waiting for {event!r}")

    def start(self, rec: dict) -> float:
        """Hand the oldest standby its pod's env; return the ready latency (seconds). The pod's
        runtime comes up while the GPU may still be wiping a retired pod's HBM (as a container
        starts right after its admission); its state is allocated once the GPU has room."""
        if not self.standby:                            # (the pool refills in the background)
            self._spawn()
        w = self.standby.pop(0)
        # replenish the pool off this pod's path (forking this large process costs tens of ms)
        t_sp = time.perf_counter()
        th = threading.Thread(target=self._spawn, daemon=True)
        th.start()
        self._spawners = [t for t in getattr(self, "_spawners", []) if t.is_alive()] + [th]
        self.phase_ms.setdefault("standby_spawn", []).append(time.perf_counter() - t_sp)
        t_sb = time.perf_counter()
        self._wait(w, "standby")
        self.phase_ms.setdefault("standby_wait", []).append(time.perf_counter() - t_sb)
        env = dict(rec["env"])
        env.pop("LD_PRELOAD", None)                     # preloaded since exec (same host path)
        if not self.visible_by_uuid:                    # modelled node (fake SMI): this rank's GPU
            env.pop("ROCR_VISIBLE_DEVICES", None)
            env["HIP_VISIBLE_DEVICES"] = str(self.ordinal)
        # a fresh container's own, empty cache home: comgr keeps what a process compiles under
        # $XDG_CACHE_HOME by default, which pods of one image never share (their blit kernels come
        # from the node's read-only comgr cache when the plugin mounts one, --comgr-cache-dir)
        env["XDG_CACHE_HOME"] = tempfile.mkdtemp(prefix="gs-pod-home-", dir="/tmp")
        from aliyun_gpushare_device_plugin_amd import const

        # with an HBM broker the plugin granted the pod its granules while it prepared the answer:
        # the env carries the broker socket (host path, container_env) and the pod's token
        t0 = time.perf_counter()
        w["proc"].stdin.write(json.dumps({"cmd": "start", "env": env, "gemm": self.gemm, "burst": self.burst,
                                          "fill": self.fill, "two_phase": True}) + "\n")
        inited = self._wait(w, "inited")
        t1 = time.perf_counter()
        take = inited.get("take_ms") or {}
        for k, name in (("cuda_init_ms", "init_cuda_init"), ("runtime_ms", "init_first_alloc")):
            if k in inited:       # torch.cuda.init(); the first allocation (the TAKE inside it)
                self.phase_ms.setdefault(name, []).append(inited[k] / 1e3)
        for k in ("connect", "wait", "map"):          # the broker TAKE inside init (shim timing)
            if k in take:
                self.phase_ms.setdefault(f"init_take_{k}", []).append(take[k] / 1e3)
        self._wait_room(int(env.get(const.ENV_SHIM_QUOTA_BYTES, 0)) * self.fill + 3 * self.gemm ** 2 * 2)
        t2 = time.perf_counter()
        free2 = self._vram_total - self._vram_used() if self._vram_used is not None else None
        if self._stopped_at is not None:                # retired pod's HBM back (room for this one)
            dt_rel = time.perf_counter() - self._stopped_at[0]
            self.release_ms.append(dt_rel)
            self.release_by_size.setdefault(self._stopped_at[1], []).append(dt_rel)
            if self._stopped_at[2] > 0:
                self.release_bytes_s.append((self._stopped_at[2], dt_rel))
            self._stopped_at = None
        w["proc"].stdin.write('{"cmd":"alloc"}\n')
        ev = self._wait(w, "ready")
        t3 = time.perf_counter()
        dt = t3 - t0
        for k, v in (("init", t1 - t0), ("room", t2 - t1), ("alloc", t3 - t2), ("hold", ev.get("hold_ms", 0) / 1e3)):
            self.phase_ms[k].append(v)
        stream = ev.get("stream") or {}
        for k in ("wait_ms", "map_ms"):               # a streaming TAKE: owed granules, inside "alloc"
            if k in stream:
                self.phase_ms.setdefault(f"alloc_more_{k[:-3]}", []).append(stream[k] / 1e3)
        for k in ("first_reserve_ms", "first_access_ms", "first_import_ms", "first_map_ms", "answer_ms"):
            if k in stream:        # parts of init_take_map (first_*) and of init_take_wait (answer)
                self.phase_ms.setdefault(f"init_take_{k[:-3]}", []).append(stream[k] / 1e3)
        if "first" in stream:      # a count, stored /1e3 so the line's ms conversion prints it as is
            self.phase_ms.setdefault("init_take_first_batch_granules", []).append(stream["first"] / 1e3)
        if self.trace is not None:
            self.trace.append({"size": rec["size"], "init": t1 - t0, "room": t2 - t1, "alloc": t3 - t2,
                               "hold_chunk_ms": ev.get("hold_chunk_ms"),
                               "free_at_alloc": free2})
        w.update(size=rec["size"], ready=ev)
        self.pods[rec["uid"]] = w
        self.held_bytes += ev.get("held", 0)
        self.ready_ms.append(dt)
        if dt > self.slowest.get("ready", 0) / 1e3:     # the slowest pod of the run, phase by phase
            self.slowest = {"ready": dt * 1e3, "size_gib": rec["size"], "init": (t1 - t0) * 1e3,
                            "cuda_init": inited.get("cuda_init_ms"), "first_alloc": inited.get("runtime_ms"),
                            "take": {k: take[k] for k in ("connect", "wait", "map") if k in take},
                            "room": (t2 - t1) * 1e3, "alloc": (t3 - t2) * 1e3}
        return dt

    def _wait_room(self, nbytes: float, limit_s: float = 30.0) -> None:
        """Before a pod allocates its state: the GPU must physically have room for what it will
        hold. In the churn that is the retired pod's HBM coming back; at the fill, e.g. right after
        a previous run on the same GPU, amdgpu may still be wiping (~33 GB/s, seconds for a full GPU)."""
        if self._vram_used is None or nbytes <= 0:
            return
        deadline = time.perf_counter() + limit_s
        while self._vram_total - self._vram_used() < nbytes + self.slack and time.perf_counter() < deadline:
            time.sleep(0.01)

    def stop(self, uid: str, wait_release: bool = False):
        """Retire a pod: it frees everything through KFD before it answers. amdgpu returns the
        VRAM asynchronously (it wipes it first, ~26 ms per GiB); the replacement's start waits for
        physical room (``start``), so the wipe overlaps the admission and the new pod's runtime
        start-up. ``wait_release`` waits for that room here instead."""
        w = self.pods.pop(uid, None)
        if w is None:
            return
        if self.stop_mode != "cooperative":
            return self._stop_uncooperative(w)
        t0 = time.perf_counter()
        w["proc"].stdin.write('{"cmd":"stop"}\n')
        ev = self._wait(w, "done")                      # freed through KFD at this point
        self.phase_ms["stop"].append(time.perf_counter() - t0)
        for k, v in (ev.get("stop_ms") or {}).items():  # inside the pod: burst in flight, free, arena
            self.phase_ms.setdefault(f"stop_{k}", []).append(v / 1e3)
        for k, v in (ev.get("release_ms") or {}).items():   # inside the shim's arena release
            self.phase_ms.setdefault(f"stop_release_{k}", []).append(v / 1e3)
        threading.Thread(target=w["proc"].wait, daemon=True).start()   # reap the exit off the path
        self._stopped_at = (t0, w["size"], w["ready"].get("held", 0))
        self.retired_bytes += w["ready"].get("held", 0)
        if self._vram_used is not None and wait_release:
            self._wait_room(w["ready"].get("held", 0), limit_s=20.0)
        self.released_residue = max(self.released_residue, ev.get("used_after_release") or 0)
        self.retired_gemms += ev["gemms"]
        self.held_bytes -= w["ready"].get("held", 0)
        self.denied += ((ev.get("shim") or {}).get("denied") or 0)

    def _stop_uncooperative(self, w) -> None:
        """A retired pod stopped as the kubelet stops a container (``sigterm``: SIGTERM, the default
        action, no release call) or whose program just ends (``exit``: a normal exit without
        freeing or releasing anything). The step's stop lasts until the process is gone; its HBM
        comes back as the broker sees its granules' last references go."""
        w["proc"].stdin.write('{"cmd":"stats"}\n')
        gemms = self._wait(w, "stats")["gemms"]         # the work it did, asked between bursts
        t0 = time.perf_counter()
        if self.stop_mode == "sigterm":
            w["proc"].terminate()
        else:
            w["proc"].stdin.write('{"cmd":"exit"}\n')
        w["proc"].wait(60)
        self.phase_ms["stop"].append(time.perf_counter() - t0)
        self._stopped_at = (t0, w["size"], w["ready"].get("held", 0))
        self.retired_bytes += w["ready"].get("held", 0)
        self.retired_gemms += gemms
        self.held_bytes -= w["ready"].get("held", 0)

    def oldest(self) -> str | None:
        return next(iter(self.pods), None)

    def gemms(self) -> int:
        """Cumulative GEMMs of every pod this fleet ran (live pods asked between bursts)."""
        live = list(self.pods.values())
        for w in live:
            w["proc"].stdin.write('{"cmd":"stats"}\n')
        return self.retired_gemms + sum(self._wait(w, "stats")["gemms"] for w in live)

    def close(self):
        for uid in list(self.pods):
            self.stop(uid)
        for t in getattr(self, "_spawners", []):
            t.join(60)                                  # every standby started is in the pool
        for w in self.standby:
            try:
                w["proc"].stdin.close()
                w["proc"].wait(30)
            except Exception:  # noqa: BLE001
                w["proc"].kill()
        if self._zygote is not None:
            self._zygote.close()


class StubFleet:
    """CPU rehearsal of the broker path (``--stub-runtime``): each admitted pod is a process of
    the stub HIP runtime (``tests/native/shim_driver``) under the real quota shim, with the
    Allocate answer's env. It takes its arena from this rank's stub broker at its first
    allocation, holds ``fill`` of its quota, reports, and waits; stopping it ends the process
    (its broker connection closes and the granules go back). No GEMMs: the rehearsal is about
    every rank's broker serving every pod, not about throughput."""

    def __init__(self, stub_dir: str, fill: float):
        self.stub_dir, self.fill = stub_dir, fill
        self.pods: dict[str, dict] = {}
        self.ready_ms: list[float] = []
        self.arenas = 0                       # pods whose allocations came from the broker arena
        self.denied = self.held_bytes = self.released_residue = self.retired_bytes = 0
        self.release_ms: list[float] = []
        self.release_by_size: dict[int, list] = {}
        self.release_bytes_s: list[tuple] = []
        self.phase_ms: dict[str, list] = {"stop": [], "init": [], "room": [], "alloc": [], "hold": []}
        self.trace = None

    def start(self, rec: dict) -> float:
        from aliyun_gpushare_device_plugin_amd import const

        env = dict(os.environ, **rec["env"])
        env.update(LD_PRELOAD=":".join(x for x in (os.path.join(NATIVE, "libgpushare_hipquota.so"),
                                                   os.environ.get("LD_PRELOAD", "")) if x), LD_LIBRARY_PATH=self.stub_dir,
                   FAKE_HIP_TOTAL_GIB="288", GPUSHARE_HBM_WAIT_S="30")
        quota = int(env.get(const.ENV_SHIM_QUOTA_BYTES, 0))
        t0 = time.perf_counter()
        p = subprocess.Popen([os.path.join(self.stub_dir, "shim_driver"), "alloc", str(int(quota * self.fill)),
                              "arena", "wait"], env=env, stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
        alloc = arena = None
        for ln in p.stdout:
            if ln.startswith("{"):
                ev = json.loads(ln)
                if ev["op"] == "alloc":
                    alloc = ev
                elif ev["op"] == "arena":
                    arena = ev
                    break
        dt = time.perf_counter() - t0
        if alloc is None or arena is None:
            raise RuntimeError(f"stub pod {rec['uid']} exited before it reported (rc {p.poll()})")
        self.denied += alloc["err"] != 0
        self.arenas += arena["on"] == 1
        held = int(quota * self.fill) if alloc["err"] == 0 else 0
        self.held_bytes += held
        self.pods[rec["uid"]] = {"proc": p, "size": rec["size"], "held": held, "arena": arena}
        self.ready_ms.append(dt)
        self.phase_ms["alloc"].append(dt)
        return dt

    def stop(self, uid: str):
        w = self.pods.pop(uid, None)
        if w is None:
            return
        t0 = time.perf_counter()
        w["proc"].stdin.close()
        w["proc"].wait(30)
        self.phase_ms["stop"].append(time.perf_counter() - t0)
        self.held_bytes -= w["held"]
        self.retired_bytes += w["held"]

    def oldest(self) -> str | None:
        return next(iter(self.pods), None)

    def gemms(self) -> int:
        return 0

    def close(self):
        for uid in list(self.pods):
            self.stop(uid)


def cpu_split(n_reserved: int) -> tuple[dict | None, str]:
    """The node's CPU split (``--reserved-cpus``): daemons' CPUs by role (SimCluster
    ``daemon_cpus``) and the pods' CPUs (GS_POD_CPUS), from this process's allowed set."""
    allowed = sorted(os.sched_getaffinity(0))
    if n_reserved <= 0 or len(allowed) < n_reserved + 4:
        return None, ""
    res = allowed[-n_reserved:]
    return ({f"plugin:{MAIN_NODE}": ",".join(map(str, res))},
            ",".join(map(str, allowed[:-n_reserved])))


def child_run(a, steps: int, *flags: str, tenant_stop: str | None = None, zygote: bool | None = None) -> dict:
    """A short child run of this churn on 1 GPU with one thing changed (``flags``, the tenant's
    stop, fresh standby interpreters); its headline. The comparators of the line: each measured on
    the same box right after the main run handed every byte back."""
    import tempfile

    out = os.path.join(tempfile.mkdtemp(prefix="gs-child-", dir="/tmp"), "line.json")
    stop = tenant_stop or a.tenant_stop
    cmd = [sys.executable, os.path.abspath(__file__), "--gpus", "1", "--steps", str(steps), "--warmup", "1",
           "--compare-rtts", "", "--fill-orders", "", "--no-ref-churn", "--driver-path-steps", "0",
           "--comparator-steps", "0", "--gemm", str(a.gemm), "--fill", str(a.fill), "--standby", str(a.standby),
           "--tenant-stop", stop, "--json-out", out, "--reserved-cpus", str(a.reserved_cpus)]
    if a.comgr_cache and a.comgr_cache_dir:
        cmd += ["--comgr-cache-dir", a.comgr_cache_dir]     # the same sealed cache (flags may turn it off)
    cmd += list(flags)
    if (a.no_pod_zygote if zygote is None else not zygote):
        cmd.append("--no-pod-zygote")
    t0 = time.perf_counter()
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=420)
        with open(out) as f:
            d = json.loads(f.read())
    except Exception as e:  # noqa: BLE001 - a comparator, never fatal to the headline
        return {"error": f"{type(e).__name__}: {e}"[:300]}
    broker = d.get("hbm_broker") or {}
    return {"value": d["value"], "unit": d["unit"], "steps": d["steps"], "ms_per_step": d["ms_per_step"],
            "pod_ready_p50_ms": d.get("pod_ready_p50_ms"), "pod_ready_p99_ms": d.get("pod_ready_p99_ms"),
            "pod_phase_p50_ms": d.get("pod_phase_p50_ms"), "pod_phase_max_ms": d.get("pod_phase_max_ms"),
            "pod_slowest_ms": d.get("pod_slowest_ms"), "allocate_p50_ms": d.get("allocate_p50_ms"),
            "failed_admissions": d.get("failed_admissions"), "quota_denials": d.get("quota_denials"),
            "tenant_stop": d.get("config", {}).get("tenant_stop"),
            "standby_forked_from_zygote": d.get("config", {}).get("standby_forked_from_zygote"),
            "broker_quarantine_ms_max": broker.get("quarantine_ms_max"), "broker_ends": broker.get("ends"),
            "rc": r.returncode, "wall_s": round(time.perf_counter() - t0, 1)}


def driver_path_run(a) -> dict:
    """The driver path (``--no-hbm-broker``: every pod allocates fresh from amdgpu, which wipes a
    retired pod's HBM first) with this run's pod shapes."""
    return child_run(a, a.driver_path_steps, "--no-hbm-broker")


def relaunch(n: int) -> int:
    """``bench.py --gpus N`` started without a launcher (no ``WORLD_SIZE``): run the same command
    as N ranks under ``torch.distributed.run`` in a child process and return its exit code. Called
    before anything touches the GPU (no torch import yet), so the parent never holds a device."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    sys.stderr.write(f"bench: --gpus {n} without a launcher: running {n} ranks under torch.distributed.run\n")
    sys.stderr.flush()
    return subprocess.call(cmd, env=dict(os.environ, MASTER_ADDR="127.0.0.1"))


def bind_device(smi_index: int) -> tuple[int, dict]:
    """The HIP ordinal of the plugin's GPU ``smi_index`` (the plugin enumerates SMI devices and
    this rank churns that GPU), matched by PCI address — HIP and SMI orders are not promised to
    agree. Returns (ordinal, binding record); exits when no visible HIP device has that address."""
    import torch

    from aliyun_gpushare_device_plugin_amd.device.smi import SMI

    with SMI("auto") as s:
        if s.count() <= smi_index:
            raise SystemExit(f"bench: rank for plugin GPU {smi_index} but SMI sees {s.count()} GPU(s)")
        g = s.device(smi_index)
    dom, bus, rest = g.bdf.split(":")
    want = (int(dom, 16), int(bus, 16), int(rest.split(".")[0], 16))
    for i in range(torch.cuda.device_count()):
        p = torch.cuda.get_device_properties(i)
        if (p.pci_domain_id, p.pci_bus_id, p.pci_device_id) == want:
            return i, {"smi_index": smi_index, "uuid": g.uuid, "bdf": g.bdf, "hip_ordinal": i}
    raise SystemExit(f"bench: no HIP device at {g.bdf} (plugin GPU {smi_index}, {g.uuid})")


def main():
    a = parse()
    # the plugin's per-pod timeline carries each pre-bind step's thread CPU time (pod_timeline)
    os.environ.setdefault("GPUSHARE_TRACE_CPU", "1")
    n = a.gpus
    if "WORLD_SIZE" not in os.environ and n > 1:
        sys.exit(relaunch(n))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != n:
        raise SystemExit(f"WORLD_SIZE={world} but --gpus {n}: one rank per GPU")

    import tempfile

    import torch
    import torch.distributed as dist

    use_gpu = torch.cuda.is_available() and not a.no_gpu
    stub = os.path.abspath(a.stub_runtime) if a.stub_runtime and not use_gpu else None
    binding = None
    ordinal = local
    if use_gpu:
        ordinal, binding = bind_device(local)
        torch.cuda.set_device(ordinal)
    dev = torch.device("cuda", ordinal) if use_gpu else None
    if world > 1:
        dist.init_process_group("nccl" if use_gpu else "gloo", device_id=dev if use_gpu else None)

    def bcast(obj):
        if world == 1:
            return obj
        box = [obj]
        dist.broadcast_object_list(box, src=0)
        return box[0]

    def gather(obj):
        if world == 1:
            return [obj]
        out = [None] * world
        dist.all_gather_object(out, obj)
        return out

    def barrier():
        if world > 1:
            dist.barrier()
        if use_gpu:
            torch.cuda.synchronize()

    smi = a.smi_backend or ("auto" if use_gpu else f"fake:{n}x288G")
    cp = None
    info = None
    daemon_cpus, pod_cpus = cpu_split(a.reserved_cpus) if use_gpu else (None, "")
    PodFleet.pod_cpus = pod_cpus
    comgr_info = {"prefilled": True} if a.comgr_cache_dir else None
    workdir = tempfile.mkdtemp(prefix="gs-bench-", dir="/tmp")
    if rank == 0:
        ref_spec = smi if smi.startswith("fake:") else None
        if use_gpu and smi == "auto":
            from aliyun_gpushare_device_plugin_amd.device.smi import SMI
            with SMI("auto") as s:
                # every rank bound its plugin GPU above (bind_device), so the node has >= n GPUs
                ref_spec = f"fake:{n}x{s.device(0).vram_total}B"
        hbm_dir = tempfile.mkdtemp(prefix="gs-hbm-", dir="/tmp") if (use_gpu or stub) and a.hbm_broker else None
        if use_gpu and a.comgr_cache and not a.comgr_cache_dir:
            # what the DaemonSet's comgr-cache init container does before the plugin starts
            from aliyun_gpushare_device_plugin_amd.quota import comgr_cache

            cdir = tempfile.mkdtemp(prefix="gs-comgr-", dir="/tmp")
            t_c = time.perf_counter()
            w = comgr_cache.warm(cdir, ("system", "torch"), device=ordinal)
            comgr_cache.seal(cdir)
            a.comgr_cache_dir = cdir
            comgr_info = {"files": w["files"], "bytes": w["bytes"], "action_entries": w.get("action_entries"),
                          "fill_s": round(time.perf_counter() - t_c, 2),
                          "runtimes": {k: bool(v.get("ok")) for k, v in w["runtimes"].items()}}
        cp = ControlPlane(n, smi, a.pod_source, a.plugin_mode, workdir, with_shim=use_gpu or bool(stub),
                          ref_spec=None if a.no_ref_churn else ref_spec, hbm_dir=hbm_dir,
                          comgr_dir=a.comgr_cache_dir if use_gpu and a.comgr_cache else None,
                          daemon_cpus=daemon_cpus)
        info = {"units_per_gpu": cp.units_per_gpu, "gpu_count": cp.gpu_count, "hbm_dir": hbm_dir}
    info = bcast(info)
    units = info["units_per_gpu"]
    broker = None
    broker_error = None
    if (use_gpu or stub) and info.get("hbm_dir"):
        from aliyun_gpushare_device_plugin_amd.quota.hbmbroker import HBMBroker

        # the broker of the plugin's GPU <local> (this rank's device, bound by PCI address), in
        # the node layout the plugin's --hbm-broker-dir names
        kw = {}
        if stub:
            kw = dict(exe=os.path.join(stub, "gpushare-hbm-broker"),
                      env=dict(os.environ, FAKE_HIP_TOTAL_GIB="288", LD_LIBRARY_PATH=stub))
        broker = HBMBroker.for_gpu(info["hbm_dir"], local, device=ordinal, reserve_gib=a.hbm_broker_reserve_gib, **kw)
        try:
            broker.start()
        except Exception as e:  # noqa: BLE001 - reported in the line; the churn runs on the driver path
            broker_error = f"{type(e).__name__}: {e}"[:500]
            sys.stderr.write(f"bench: hbm broker unavailable, pods allocate from the driver: {broker_error}\n")
            broker = None
    # every rank's broker listens before rank 0 fills the node: the plugin grants each pod while it
    # prepares its answer (a grant that finds no broker is re-sent on the granter's next poll, and
    # the pod's shim waits for its broker, but the fill should not depend on that)
    barrier()
    # pod processes see their GPU through the Allocate response's ROCR_VISIBLE_DEVICES (UUID)
    if use_gpu:
        fleet = PodFleet(local, a.gemm, a.burst, a.fill, not smi.startswith("fake:"), a.standby,
                         slack=int(a.room_slack_gib * (1 << 30)), ordinal=ordinal, broker=broker,
                         zygote=not a.no_pod_zygote, stop_mode=a.tenant_stop)
    else:
        fleet = StubFleet(stub, a.fill) if stub else None
    topo_report = cp_topo = None
    topo_failed = False
    problems: list = []

    def launch(started: dict) -> float:
        """Start this rank's newly admitted pods; returns the slowest ready latency."""
        worst = 0.0
        if fleet is not None:
            for rec in started.get(local, []):
                worst = max(worst, fleet.start(rec))
        return worst

    # Per-GPU churn pipelines: every rank cycles its own GPU (stop the oldest pod -> its HBM is
    # back -> ask rank 0's admission service for the replacement -> start it) without waiting for
    # the other GPUs; rank 0 serialises the admissions themselves, as one kubelet does.
    svc = client = None
    port = None
    if rank == 0:
        svc = AdmissionService(cp)
        port = svc.serve() if world > 1 else None
    port = bcast(port)
    if rank != 0:
        client = AdmissionClient(port)

    done = {"churned": 0, "started": 0}          # this rank's GPU, timed region only (reset below)

    idle = os.environ.get("GS_BENCH_IDLE_RANK")   # test hook: this rank's pipeline does nothing

    step_parts: dict[str, list] = {"stop": [], "admission": [], "start": [], "total": []}

    def cycle():
        if idle is not None and int(idle) == rank:
            return
        uid = None
        t0 = time.perf_counter()
        if fleet is not None:
            uid = fleet.oldest()
            if uid is not None:
                fleet.stop(uid)                  # the replacement's start waits for the HBM
        t1 = time.perf_counter()
        rec = svc.churn(local, uid) if rank == 0 else client.churn(local, uid)
        t2 = time.perf_counter()
        if rec is not None:
            done["churned"] += 1
            if fleet is not None:
                fleet.start(rec)
                done["started"] += 1
        t3 = time.perf_counter()
        for k, v in (("stop", t1 - t0), ("admission", t2 - t1), ("start", t3 - t2), ("total", t3 - t0)):
            step_parts[k].append(v)

    # ---- warm-up: fill the node, start its pods, then W untimed churn cycles per GPU ----
    started = bcast(cp.fill() if rank == 0 else None)
    launch(started)
    barrier()
    for _ in range(a.warmup):
        cycle()
    barrier()
    if rank == 0:
        cp.alloc_lat.clear()
        for v in cp.alloc_lat_by_gpu.values():
            v.clear()
        cp.admit_lat.clear()
        cp.ref_lat.clear()
        cp.ref_splits.clear()
        cp.splits.clear()
        cp.ref_failed = 0
        cp.mirror_s.clear()
        cp.cp_time = 0.0
        cp.failed = 0
        cp.fail_reasons.clear()
        cp.native_before = native_stats(cp.metrics_port)
        cp.commit_ns.clear()
        cp.plugin_latency(reset=True)
        if cp.ref_port:
            plugin_latency(cp.ref_port, reset=True)
    if fleet is not None:
        fleet.ready_ms.clear()
        if hasattr(fleet, "slowest"):
            fleet.slowest = {}
        fleet.release_ms.clear()
        fleet.release_by_size.clear()
        fleet.release_bytes_s.clear()
        fleet.retired_bytes = 0
        for v in fleet.phase_ms.values():
            v.clear()

    done.update(churned=0, started=0)
    for v in step_parts.values():
        v.clear()
    barrier()
    g0 = fleet.gemms() if fleet is not None else 0
    t0 = time.perf_counter()
    for _ in range(a.steps):
        cycle()
    barrier()
    elapsed = time.perf_counter() - t0
    g1 = fleet.gemms() if fleet is not None else 0
    gemm_flops = 2.0 * a.gemm ** 3 * (g1 - g0)
    if world > 1:
        t = torch.tensor([elapsed, gemm_flops], dtype=torch.float64, device=dev if use_gpu else "cpu")
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        elapsed, gemm_flops = float(mx[0]), float(t[1])
    parts_all: dict = {}
    for d_ in gather(step_parts):
        for k, v in d_.items():
            parts_all.setdefault(k, []).extend(v)
    ready = gather(fleet.ready_ms if fleet is not None else [])
    ready_all = [x for r in ready for x in r]
    slowest = max(gather(getattr(fleet, "slowest", {}) if fleet is not None else {}), key=lambda w: w.get("ready", 0))
    held = gather(fleet.held_bytes if fleet is not None else 0)
    denied = gather(fleet.denied if fleet is not None else 0)
    residue = gather(fleet.released_residue if fleet is not None else 0)
    release = gather(fleet.release_ms if fleet is not None else [])
    release_all = [x for r in release for x in r]
    retired = gather(fleet.retired_bytes if fleet is not None else 0)
    rel = [x for r in gather(fleet.release_bytes_s if fleet is not None else []) for x in r]
    per_rank = gather(dict(done, rank=rank, gpu=local, binding=binding,
                           pods_live=len(fleet.pods) if fleet is not None else None,
                           arenas=getattr(fleet, "arenas", None),
                           broker=broker.stat() if broker is not None else None,
                           broker_error=broker_error))
    by_size: dict = {}
    phases: dict = {}
    for d in gather(fleet.phase_ms if fleet is not None else {}):
        for k, v in d.items():
            phases.setdefault(k, []).extend(v)
    for d in gather(fleet.release_by_size if fleet is not None else {}):
        for k, v in d.items():
            by_size.setdefault(k, []).extend(v)

    if world > 1:
        from aliyun_gpushare_device_plugin_amd.cluster import nodestatus
        from aliyun_gpushare_device_plugin_amd.parallel import topology as T

        topo = healthy = None
        if rank == 0:
            node = cp.cluster.client.get_node(MAIN_NODE)
            topo = cp_topo = nodestatus.read_topology(node)
            hmap = json.loads((node.get("metadata", {}).get("annotations") or {}).get(
                "gpushare.amd.com/gpu-health", "{}") or "{}")
            healthy = [bool((hmap.get(str(i)) or {}).get("healthy", True)) for i in range(n)]
        topo_report = T.bench_report(rank, world, use_gpu, topo, dev)
        if rank == 0:
            ok, why = T.verdict(topo, n, healthy)
            topo_report["verdict"] = "pass" if ok else "fail"
            topo_report["reasons"] = why
            topo_failed = not ok

    if rank == 0:
        from aliyun_gpushare_device_plugin_amd.plugin import native_server
        from aliyun_gpushare_device_plugin_amd.sim.h2client import NativeUnaryClient

        srv = cp.plugin_latency()
        ref_srv = plugin_latency(cp.ref_port) if cp.ref_port else None
        pods_node = sum(len(v) for v in cp.resident.values())
        gib_node = sum(s for v in cp.resident.values() for _, s in v)
        # real admissions of the timed region (every churn_one that admitted a replacement),
        # never steps x n: a GPU whose pipeline did not run contributes nothing
        admissions = len(cp.admit_lat)
        value = admissions / elapsed
        problems = []
        for r in per_rank:
            if r["churned"] == 0:
                problems.append(f"GPU {r['gpu']} (rank {r['rank']}): no admissions in the timed region")
            if (use_gpu or stub) and (r["started"] == 0 or not r["pods_live"]):
                problems.append(f"GPU {r['gpu']} (rank {r['rank']}): no pod processes started")
        if n > 1 and (topo_report is None or "verdict" not in topo_report):
            problems.append("no topology verdict for a multi-GPU node")
        under_churn = {"default": {
            "allocate_p50_ms": ms(pct(cp.alloc_lat, 0.5)), "allocate_p99_ms": ms(pct(cp.alloc_lat, 0.99)),
            "plugin_allocate_p50_ms": ms(srv["p50"]) if srv else None,
            "plugin_allocate_p99_ms": ms(srv["p99"]) if srv else None,
            "allocate_breakdown_p50_ms": breakdown(cp.splits),
            "answered_by": native_share(getattr(cp, "native_before", None), native_stats(cp.metrics_port)),
            "pod_timeline": pod_timeline(cp.metrics_port, cp.commit_ns),
            "native_table_publish": (srv or {}).get("table_publish"),
            "admissions": len(cp.alloc_lat), "pod_source": a.pod_source, "patch": "write-behind",
            "apiserver_round_trips_on_path": round_trips(srv)}}
        if cp.ref_port:
            under_churn["reference"] = {
                "allocate_p50_ms": ms(pct(cp.ref_lat, 0.5)), "allocate_p99_ms": ms(pct(cp.ref_lat, 0.99)),
                "plugin_allocate_p50_ms": ms(ref_srv["p50"]) if ref_srv else None,
                "plugin_allocate_p99_ms": ms(ref_srv["p99"]) if ref_srv else None,
                "plugin_allocate_phase_p50_ms": {k: ms(v) for k, v in ref_srv["phases"].items() if v is not None}
                if ref_srv else None,
                "allocate_breakdown_p50_ms": breakdown(cp.ref_splits),
                "admissions": len(cp.ref_lat), "failed": cp.ref_failed, "pod_source": "list", "patch": "sync",
                "apiserver_round_trips_on_path": round_trips(ref_srv)}
        svc.stop()
        cp.stop()
        modes = mode_comparison([float(x) for x in a.compare_rtts.split(",") if x], a.compare_pods) \
            if a.compare_rtts else {}
        fills = fill_orders([x for x in a.fill_orders.split(",") if x], n, units) if a.fill_orders else {}
        floor = transport_floor() if a.compare_rtts else None
        res = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "pods admitted-to-ready/s",
            "n_gpus": n,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic pod specs (mixed 8-128 GiB), random-init bf16 GEMM operands; one OS process per pod "
                    "under the quota shim",
            "config": {"model": "gpushare-device-plugin + MFMA GEMM pods (BASELINE config 3 churn)",
                       "global_batch": 4 * n, "seq_len": None, "parallelism": f"node{n}",
                       "pods_per_gpu": 4, "gemm_mnk": a.gemm, "pod_fill": a.fill, "pod_source": a.pod_source,
                       "smi_backend": smi, "pod_processes": use_gpu, "hbm_broker": broker is not None,
                       "standby_interpreters_per_gpu": a.standby,
                       "standby_forked_from_zygote": not a.no_pod_zygote,
                       "tenant_stop": a.tenant_stop,
                       "comgr_cache": comgr_info if a.comgr_cache and use_gpu else False,
                       "reserved_cpus": {"daemons": daemon_cpus, "pods": pod_cpus} if daemon_cpus else None,
                       # the plugin's gRPC server and the simulated kubelet's Allocate client
                       "grpc_server": "native" if native_server.available() else "python",
                       "kubelet_client": "native" if NativeUnaryClient.wanted() else "grpcio"},
            "allocate_p50_ms": ms(pct(cp.alloc_lat, 0.5)),
            "allocate_p99_ms": ms(pct(cp.alloc_lat, 0.99)),
            "allocate_breakdown_p50_ms": breakdown(cp.splits),
            # the slowest Allocate of the run, leg by leg: where its tail comes from
            "allocate_slowest_ms": (lambda w: {"total": ms(sum(w)), **{k: ms(w[i]) for i, k in enumerate(
                ("kubelet_to_handler", "handler", "handler_to_kubelet"))}})(max(cp.splits, key=sum)) if cp.splits else None,
            "plugin_allocate_p50_ms": ms(srv["p50"]) if srv else None,
            "plugin_allocate_p99_ms": ms(srv["p99"]) if srv else None,
            "plugin_allocate_phase_p50_ms": {k: ms(v) for k, v in srv["phases"].items() if v is not None}
            if srv else None,
            "admission_p50_ms": ms(pct(cp.admit_lat, 0.5)),
            "pod_ready_p50_ms": ms(pct(ready_all, 0.5)),
            "pod_ready_p99_ms": ms(pct(ready_all, 0.99)),
            "pod_room_wait_p50_ms": ms(pct(release_all, 0.5)),
            "pod_room_wait_p50_ms_by_gib": {str(k): ms(pct(v, 0.5)) for k, v in sorted(by_size.items())},
            # one churn cycle on a GPU: stop (old pod frees) -> admission -> new pod's runtime up
            # (init) -> physical room for its state (room) -> state allocated + first GEMM (alloc)
            "pod_phase_p50_ms": {k: ms(pct(v, 0.5)) for k, v in phases.items()},
            "pod_phase_max_ms": {k: ms(max(v)) for k, v in phases.items() if v},
            "pod_slowest_ms": {k: round(v, 3) if isinstance(v, float) else v for k, v in slowest.items()} or None,
            "control_plane_ms_per_admission": round(cp.cp_time / max(1, admissions) * 1e3, 3),
            # the reference-model node's own churn step runs inside each timed step (the
            # allocate_under_churn comparison): its share of ms_per_step
            "reference_mirror_ms_per_step": round(sum(cp.mirror_s) / max(1, len(cp.mirror_s)) * 1e3, 3) if cp.mirror_s else None,
            # a timed step, part by part (mean over steps and GPUs): the retired pod's stop, the
            # admission (rank 0's control plane, the reference mirror inside), the replacement's
            # start (standby hand-over + ready)
            "step_parts_mean_ms": {k: round(sum(v) / len(v) * 1e3, 3) for k, v in parts_all.items() if v},
            "allocate_p50_ms_by_gpu": {str(g): ms(pct(v, 0.5)) for g, v in cp.alloc_lat_by_gpu.items()},
            # both plugins during the same timed churn (alternating admissions, same pod load)
            "allocate_under_churn": under_churn,
            # the same A/B on a quiet cluster at injected apiserver RTTs
            "allocate_by_mode": modes,
            # what the two transport legs cost with a handler that does nothing: a Python gRPC
            # client (the fake kubelet; the real one is Go) calling a grpcio server like the
            # plugin's, every 5 ms, nothing else running (tools/grpc_server_probe.py)
            "allocate_transport_floor_p50_ms": floor,
            "fill_orders": fills,
            "pods_per_node": pods_node,
            "hbm_gib_per_node": gib_node,
            "advertised_gib_per_node": units * n,
            "packing_efficiency": round(gib_node / (units * n), 4) if units else None,
            # the same node under 125 % demand of seeded mixed sizes (no exact fit): HBM placed /
            # HBM advertised, online (one pod at a time) and burst (queue placed jointly)
            "oversub_packing_efficiency": {k: (fills.get(o) or {}).get("packing_efficiency")
                                           for k, o in (("online", "oversub"), ("burst", "burst_oversub"))},
            "hbm_held_by_pods_gib": round(sum(held) / (1 << 30), 1) if use_gpu else None,
            "quota_denials": sum(denied),
            "pod_hbm_residue_after_free_mib": round(max(residue) / (1 << 20), 1) if use_gpu else None,
            "admissions": admissions,
            "admissions_by_gpu": {str(r["gpu"]): r["churned"] for r in per_rank},
            "pods_started_by_gpu": {str(r["gpu"]): r["started"] for r in per_rank} if use_gpu else None,
            "failed_admissions": cp.failed,
            "failure_reasons": cp.fail_reasons[:5],
            "gemm_tflops_node": round(gemm_flops / elapsed / 1e12, 1) if use_gpu else None,
            # the churn's physical bound: every cycle turns a retired pod's HBM over, and amdgpu wipes
            # freed VRAM before it returns it. Turnover per GPU near the wipe rate = the step is at
            # that bound, not in the plugin (control_plane_ms_per_admission is the plugin's share).
            "hbm_turnover_GBps_per_gpu": round(sum(retired) / n / elapsed / 1e9, 1) if use_gpu else None,
            # bytes-weighted over the retirements: sum(bytes held) / sum(stop -> GPU has room again)
            "amdgpu_release_GBps": round(sum(b for b, _ in rel) / sum(t for _, t in rel) / 1e9, 1) if rel else None,
        }
        # pods' HBM from the per-GPU brokers (--hbm-broker): each GPU's broker counters
        brokers = {str(r["gpu"]): r["broker"] for r in per_rank}
        res["hbm_broker"] = brokers.get(str(local))
        res["hbm_broker_by_gpu"] = brokers if len(brokers) > 1 else None
        if stub:
            # the CPU rehearsal: stub pods whose allocations came from their GPU's broker arena
            res["stub_pods_with_arena_by_gpu"] = {str(r["gpu"]): r["arenas"] for r in per_rank}
        errs = {str(r["gpu"]): r["broker_error"] for r in per_rank if r.get("broker_error")}
        if errs:
            res["hbm_broker_error"] = errs
        if topo_report is not None:
            res["topology"] = topo_report
            if use_gpu:
                # each rank's device, bound by PCI address, against the plugin's matrix row
                binds = {str(r["gpu"]): r["binding"] for r in per_rank}
                topo_report["device_binding"] = binds
                rows = {str(k): g for k, g in enumerate((cp_topo or {}).get("gpus") or [])}
                for k, b in binds.items():
                    row = rows.get(k)
                    if b is None or row is None or row.get("bdf") != b["bdf"]:
                        problems.append(f"rank of GPU {k} bound {b} but the plugin's topology row is {row}")
        if problems:
            res["run_problems"] = problems
    if fleet is not None:
        if fleet.trace is not None:              # per-pod cycle phases (GS_BENCH_POD_TRACE=<path>)
            with open(f"{os.environ['GS_BENCH_POD_TRACE']}.{rank}", "w") as f:
                f.writelines(json.dumps(r) + "\n" for r in fleet.trace)
        fleet.close()
    if broker is not None:
        broker.stop()
    if client is not None:
        client.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    import shutil

    shutil.rmtree(workdir, ignore_errors=True)
    if rank == 0:
        if world == 1 and use_gpu and broker is not None and a.driver_path_steps > 0:
            # the same churn without the broker, after this run has handed every GPU byte back: what
            # the broker buys, measured on the same box in the same line
            res["driver_path"] = driver_path_run(a)
        if world == 1 and use_gpu and broker is not None and a.comparator_steps > 0:
            # tenants that do nothing for the broker (the kubelet's SIGTERM, a
            # program that just ends), and the harness's forked standbys against fresh interpreters
            for key, stop in (("cooperative_tenant", "cooperative"), ("unmodified_tenant", "sigterm"),
                              ("normal_exit_tenant", "exit")):
                if stop != a.tenant_stop:
                    res[key] = child_run(a, a.comparator_steps, tenant_stop=stop)
            res["no_pod_zygote"] = child_run(a, a.comparator_steps, zygote=False)
            if a.comgr_cache:
                # the same churn with every pod compiling its blit kernels itself
                res["no_comgr_cache"] = child_run(a, a.comparator_steps, "--no-comgr-cache")
        line = json.dumps(res)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    if topo_failed:
        # a broken topology export must not pass as a successful multi-GPU run
        sys.stderr.write("bench: topology verdict FAIL: " + "; ".join(topo_report["reasons"]) + "\n")
        sys.exit(3)
    if problems:
        # a GPU that did no work must not pass as an N-GPU measurement
        sys.stderr.write("bench: run FAILED: " + "; ".join(problems) + "\n")
        sys.exit(4)


if __name__ == "__main__":
    main()
