#!/usr/bin/env python3
"""BASELINE config 4: two Llama-3-8B bf16 pods co-located on one MI355X under the HIP quota shim.

1. The real plugin (real SMI) admits two pods of --pod-gib GiB each through the extender and the
   kubelet; their Allocate responses carry the env contract, /dev/kfd + render node, and the
   quota shim (mount + LD_PRELOAD).
2. Each pod runs as its own process with exactly that environment (the shim's container path is
   mapped back through the response's mount) and runs Llama-3-8B prefill.
3. Phase "solo": pod A alone. Phase "colocated": A and B together (synchronized start).
Reports tokens/s solo vs co-located (interference), per-iteration latency p50/p99, the quota each
pod saw, and whether an over-quota allocation was refused. Output: one JSON line (and --out).

``--hbm-broker`` (the shipped default: the DaemonSet's hbm-brokers container) starts the GPU's
HBM broker as the DS does (``--reserve-gib 12 --start-empty``, sized by the plugin) and runs the
plugin with ``--hbm-broker-dir``: each pod's memory comes from its granted granules; the line
then carries the broker's counters and each pod's shim counters (quota denials, arena use).

``--isolation cu`` admits the pods with the plugin's ``--compute-isolation=cu`` (each pod requests
``--slots-a`` / ``--slots-b`` CU slots, i.e. 8 CUs per slot, one per XCD); ``both`` runs the
experiment under time-slicing and under CU slots back to back. ``--batch-b`` makes B a heavier
neighbour than A (A = latency-sensitive tenant).
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pod_env(resp) -> dict:
    env = dict(os.environ)
    envs = dict(resp.envs)
    for m in resp.mounts:                     # container path -> host path (no container here)
        for k, v in list(envs.items()):
            if v.startswith(m.container_path):
                envs[k] = m.host_path + v[len(m.container_path):]
    env.update(envs)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    return env


def run_pods(specs, seconds, args, sync=True):
    """Start one process per pod; release them together once all report ``ready``."""
    import queue
    import threading

    start = os.path.join(tempfile.mkdtemp(prefix="coloc-"), "go")
    procs, q = [], queue.Queue()
    lines = {i: [] for i in range(len(specs))}
    errs = {i: [] for i in range(len(specs))}
    for i, (name, env, extra) in enumerate(specs):
        cmd = [sys.executable, "-m", "aliyun_gpushare_device_plugin_amd.models.llama_pod", "--name", name,
               "--seconds", str(seconds), "--batch", str(args.batch), "--seq", str(args.seq),
               "--layers", str(args.layers)] + extra + (["--start-file", start] if sync else [])
        if args.profile_dir and len(specs) > 1 and name == "llama-a":
            # (diagnosis) the colocated pod A's kernels, under rocprofv3
            cmd = ["rocprofv3", "--kernel-trace", "--stats", "-d", os.path.abspath(args.profile_dir), "-o", name,
                   "--"] + cmd
        p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        procs.append(p)

        def pump(i=i, p=p):
            for line in p.stdout:
                if line.startswith("{"):
                    d = json.loads(line)
                    lines[i].append(d)
                    q.put((i, d))
                    print(f"[{specs[i][0]}] {line.strip()[:200]}", file=sys.stderr, flush=True)   # progress for long runs
            q.put((i, None))

        def drain(i=i, p=p):
            for line in p.stderr:
                errs[i].append(line)

        threading.Thread(target=pump, daemon=True).start()
        threading.Thread(target=drain, daemon=True).start()
    ready, ended = set(), set()
    deadline = time.time() + 900
    while len(ready) < len(procs):
        i, d = q.get(timeout=max(1.0, deadline - time.time()))
        if d is None:
            ended.add(i)
            if i not in ready:
                procs[i].wait()
                raise RuntimeError(f"pod {i} exited early: {''.join(errs[i])[-3000:]}")
        elif d["event"] == "ready":
            ready.add(i)
    open(start, "w").close()
    for i, p in enumerate(procs):
        p.wait(timeout=seconds + 600)
        if p.returncode != 0:
            raise RuntimeError(f"pod {i} failed: {''.join(errs[i])[-3000:]}")
    while len(ended) < len(procs):
        i, d = q.get(timeout=30)
        if d is None:
            ended.add(i)
    return [lines[i] for i in range(len(procs))]


def start_broker(hbm_dir: str):
    """GPU 0's broker, started as the DaemonSet starts it (empty; the plugin sizes it)."""
    from aliyun_gpushare_device_plugin_amd.quota.hbmbroker import HBMBroker

    b = HBMBroker.for_gpu(hbm_dir, 0, device=0, reserve_gib=12, extra_args=["--start-empty"])
    b.start()
    return b


def wait_sized(broker, timeout: float = 120.0) -> dict:
    """Until the plugin's granter has sized the broker and it holds its target (the fill)."""
    end = time.time() + timeout
    st = broker.stat()
    while time.time() < end and not (st.get("target") and st["granules"] >= st["target"] and not st.get("scrubbing")):
        time.sleep(0.2)
        st = broker.stat()
    return st


def admit_pair(args, isolation: str, hbm_dir: str | None = None, broker=None):
    """Admit pods A and B through the real plugin; returns their pod environments + Allocate ms."""
    from aliyun_gpushare_device_plugin_amd import const
    from aliyun_gpushare_device_plugin_amd.sim.cluster import SimCluster
    from aliyun_gpushare_device_plugin_amd.utils.native import ensure_built

    shim_dir = os.path.dirname(ensure_built("hipshim"))
    ann = [None, None]
    if isolation == "cu":
        ann = [{const.POD_ANNOTATION_CU_SLOTS_REQUEST: str(args.slots_a)},
               {const.POD_ANNOTATION_CU_SLOTS_REQUEST: str(args.slots_b)}]
    extra = ["--hbm-broker-dir", hbm_dir] if hbm_dir else []
    with SimCluster([("mi355x", args.smi_backend)], shim_host_dir=shim_dir, compute_isolation=isolation,
                    extra_plugin_args=extra) as c:
        if broker is not None:
            wait_sized(broker)
        pa, wa, adm_a = c.run_pod(args.pod_gib, name="llama-a", annotations=ann[0])
        pb, wb, adm_b = c.run_pod(args.pod_gib, name="llama-b", annotations=ann[1])
        assert adm_a.error is None and adm_b.error is None and wa[1] == wb[1]
        return (pod_env(adm_a.responses[0]), pod_env(adm_b.responses[0]),
                [x * 1e3 for x in adm_a.latencies + adm_b.latencies])


def run_mode(args, isolation: str, hbm_dir: str | None = None, broker=None) -> dict:
    env_a, env_b, alloc_ms = admit_pair(args, isolation, hbm_dir, broker)
    for name, env in (("a", env_a), ("b", env_b)):
        if name not in args.arena_pods:               # (experiments) this pod allocates from the driver
            env.pop("GPUSHARE_HBM_TOKEN", None)
            env.pop("GPUSHARE_HBM_BROKER", None)
        if args.kernarg != "answer":                  # (experiments) override the answer's setting
            env["HIP_FORCE_DEV_KERNARG"] = "1" if args.kernarg == "device" else "0"
    if args.split_brokers and broker is not None and env_b.get("GPUSHARE_HBM_TOKEN"):
        # (experiment) pod B's granules from a second broker process on the same GPU
        from aliyun_gpushare_device_plugin_amd.quota.hbmbroker import HBMBroker

        broker.size(150)                              # room for the second one (the plugin is gone)
        d2 = tempfile.mkdtemp(prefix="gs-hbm2-", dir="/tmp")
        b2 = HBMBroker.for_gpu(d2, 0, device=0, gib=args.pod_gib)
        b2.start()
        q = args.pod_gib << 30
        b2.grant(env_b["GPUSHARE_HBM_TOKEN"], int(q * 0.94) >> 30 << 30, q)
        env_b["GPUSHARE_HBM_BROKER"] = b2.socket_path
        run_mode.second = b2
    extra_b = ["--batch", str(args.batch_b)] if args.batch_b else []
    extra_a = (["--mode", args.mode_a] + (["--seq", str(args.seq_a)] if args.seq_a else [])
               + (["--eager"] if args.decode_eager else [])
               + (["--stream-priority", args.priority_a] if args.mode_a == "decode" else []))
    solo = run_pods([("llama-a", env_a, ["--probe-quota"] + extra_a)], args.seconds, args)[0]
    both = run_pods([("llama-a", env_a, extra_a), ("llama-b", env_b, extra_b)], args.seconds, args)
    solo_b = run_pods([("llama-b", env_b, extra_b)], args.seconds, args)[0] if args.batch_b else None

    def done(ls):
        return [x for x in ls if x["event"] == "done"][0]

    def start(ls):
        return [x for x in ls if x["event"] == "start"][0]

    s = done(solo)
    ca, cb = done(both[0]), done(both[1])
    sb = done(solo_b) if solo_b else s
    probe = [x for x in solo if x["event"] == "quota_probe"]
    shims = [s.get("shim"), ca.get("shim"), cb.get("shim")]

    def denials(run, done_ev):
        """Allocations the shim refused during one run, the deliberate over-quota probe aside
        (a pod's ledger counts across its runs)."""
        d1 = int((done_ev.get("shim") or {}).get("denied") or 0)
        d0 = int(start(run).get("shim_denied") or 0)
        probe_d = sum(int(x.get("probe_denied") or 0) for x in run if x["event"] == "quota_probe")
        return d1 - d0 - probe_d

    runs = [("solo_a", solo, s), ("colocated_a", both[0], ca), ("colocated_b", both[1], cb)]
    if solo_b:
        runs.append(("solo_b", solo_b, sb))
    return {
        "hbm_broker": bool(env_a.get("GPUSHARE_HBM_BROKER") or env_b.get("GPUSHARE_HBM_BROKER")),
        "arena_pods": args.arena_pods if args.hbm_broker else "none",
        "hbm_token": [bool(env_a.get("GPUSHARE_HBM_TOKEN")), bool(env_b.get("GPUSHARE_HBM_TOKEN"))],
        # every pod run's shim counters: its ledger, its broker arena
        "shim": {"solo_a": shims[0], "colocated_a": shims[1], "colocated_b": shims[2]},
        "quota_denials": {k: denials(r, d) for k, r, d in runs},
        "isolation": isolation,
        "cu_slots": [env_a.get("GPUSHARE_CU_SLOTS"), env_b.get("GPUSHARE_CU_SLOTS")],
        "hsa_cu_mask": [env_a.get("HSA_CU_MASK"), env_b.get("HSA_CU_MASK")],
        "cus_seen": [ca["cus"], cb["cus"]],
        "allocate_ms": [round(x, 3) for x in alloc_ms],
        "quota_bytes_seen": start(solo)["quota_total"],
        "over_quota_alloc": probe[0]["over_quota_alloc"] if probe else None,
        "solo_tokens_per_s": round(s["tokens_per_s"], 1), "solo_tflops": round(s["tflops"], 1),
        "solo_b_tokens_per_s": round(sb["tokens_per_s"], 1),
        "solo_lat_ms": [s["lat_p50_ms"], s["lat_p99_ms"]],
        "colocated_tokens_per_s": [round(ca["tokens_per_s"], 1), round(cb["tokens_per_s"], 1)],
        "colocated_sum_tokens_per_s": round(ca["tokens_per_s"] + cb["tokens_per_s"], 1),
        "colocated_lat_ms_a": [ca["lat_p50_ms"], ca["lat_p99_ms"], ca["lat_max_ms"]],
        "colocated_lat_ms_b": [cb["lat_p50_ms"], cb["lat_p99_ms"], cb["lat_max_ms"]],
        # pod A's throughput with B running, relative to A alone under the same policy
        "a_retained": round(ca["tokens_per_s"] / s["tokens_per_s"], 3),
        "b_retained": round(cb["tokens_per_s"] / sb["tokens_per_s"], 3),
        "interference": round((ca["tokens_per_s"] + cb["tokens_per_s"]) / 2 / s["tokens_per_s"], 3),
        "aggregate_speedup_vs_solo": round((ca["tokens_per_s"] + cb["tokens_per_s"]) / s["tokens_per_s"], 3),
        "peak_mem_bytes": [ca["peak_mem"], cb["peak_mem"]],
        # how long KFD kept each colocated pod's queues evicted during the timed run
        "evicted_ms": {"solo_a": s.get("evicted_ms"), "colocated_a": ca.get("evicted_ms"), "colocated_b": cb.get("evicted_ms")},
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pod-gib", type=int, default=64)
    ap.add_argument("--seconds", type=float, default=20)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--batch-b", type=int, default=0, help="pod B's batch (0 = same as A); B then also runs solo")
    ap.add_argument("--seq", type=int, default=2048)
    ap.add_argument("--mode-a", default="prefill", choices=("prefill", "decode"),
                    help="decode: pod A is a serving pod (KV-cache decode, hipGraph per step)")
    ap.add_argument("--seq-a", type=int, default=0, help="pod A's prompt length (0 = --seq)")
    ap.add_argument("--decode-eager", action="store_true", help="pod A decodes without a hipGraph")
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--smi-backend", default="auto")
    ap.add_argument("--isolation", default="none", choices=("none", "cu", "both"),
                    help="plugin --compute-isolation for the pods; both = run the experiment under each")
    ap.add_argument("--slots-a", type=int, default=16, help="CU slots pod A requests (cu isolation)")
    ap.add_argument("--slots-b", type=int, default=16)
    ap.add_argument("--hbm-broker", action=argparse.BooleanOptionalAction, default=True,
                    help="pods' HBM from the GPU's broker (the DaemonSet default)")
    ap.add_argument("--arena-pods", default="ab",
                    help="with --hbm-broker: which pods take their arena (experiments: a, b, ab, none)")
    ap.add_argument("--split-brokers", action="store_true",
                    help="(experiment) pod B takes its granules from a second broker process")
    ap.add_argument("--priority-a", default="normal", choices=("normal", "high"),
                    help="decode pod A's stream priority (its steps, eager or graph replay)")
    ap.add_argument("--kernarg", default="answer", choices=("answer", "device", "host"),
                    help="(diagnosis) kernel arguments in device or host memory for both pods, "
                         "instead of what the Allocate answer sets")
    ap.add_argument("--profile-dir", default=None, help="(diagnosis) run the colocated pod A under rocprofv3")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    hbm_dir = broker = None
    if args.hbm_broker:
        hbm_dir = tempfile.mkdtemp(prefix="gs-hbm-", dir="/tmp")
        broker = start_broker(hbm_dir)

    modes = ["none", "cu"] if args.isolation == "both" else [args.isolation]
    res = {"config": "2 x Llama-3-8B bf16 pods on one MI355X (BASELINE config 4)", "mode_a": args.mode_a, "decode_eager": args.decode_eager,
           "pod_gib": args.pod_gib, "batch": args.batch, "batch_b": args.batch_b or args.batch, "seq": args.seq,
           "layers": args.layers}
    try:
        for m in modes:
            r = run_mode(args, m, hbm_dir, broker)
            if broker is not None:
                st = broker.stat()
                r["broker"] = {k: st.get(k) for k in ("granules", "granules_max", "target", "free", "held", "takes",
                                                      "releases", "timeouts", "extended", "quarantine_ms_max")}
            print(json.dumps(r), flush=True)
            res[m] = r
    finally:
        if broker is not None:
            broker.stop()
    if len(modes) == 1:
        res.update(res.pop(modes[0]))
    line = json.dumps(res)
    print(line)
    if args.mode_a != "prefill":
        res["note"] = "pod A tokens/s = generated tokens (batch per decode step); aggregate ratios mix units"
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
