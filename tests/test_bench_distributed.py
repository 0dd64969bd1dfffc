"""bench.py contract on CPU: single process and a 2-rank torchrun (gloo) launch."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REQUIRED = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config"}


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def parse(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_bench_single_process_cpu():
    r = subprocess.run([sys.executable, "bench.py", "--no-gpu", "--steps", "4", "--warmup", "1"], cwd=ROOT,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    d = parse(r.stdout)
    assert REQUIRED <= set(d) and d["n_gpus"] == 1 and d["steps"] == 4 and d["scaling"] == "weak"
    assert d["metric"] == json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
    assert d["pods_per_node"] == 4 and d["hbm_gib_per_node"] == 288 and d["failed_admissions"] == 0
    assert d["allocate_p50_ms"] is not None and d["value"] > 0


def test_bench_torchrun_two_ranks_gloo():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", "2",
                        "--no-gpu", "--steps", "4", "--warmup", "1"],
                       cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    d = parse(r.stdout)           # only rank 0 prints
    assert d["n_gpus"] == 2 and d["pods_per_node"] == 8 and d["advertised_gib_per_node"] == 576
    assert d["config"]["parallelism"] == "node2"
    # N>1: the topology the plugin exported and an all-reduce on the TP pair best_group picks
    topo = d["topology"]
    assert topo["tp_pair"] == [0, 1] and topo["pair_link"] == "xgmi" and topo["pair_hops"] == 1
    assert topo["verdict"] == "pass" and topo["reasons"] == []
    # both plugins measured under the same churn, in the same line
    uc = d["allocate_under_churn"]
    assert uc["default"]["admissions"] == uc["reference"]["admissions"] == 8
    # measured by the plugins themselves: LIST + PATCH for the reference model, none by default
    assert uc["reference"]["apiserver_round_trips_on_path"]["p50"] == 2
    # (a LIST only when the plugin's pod watch lagged the kubelet's past watch_grace_s: rare)
    assert uc["default"]["apiserver_round_trips_on_path"]["p50"] == 0
    assert uc["default"]["apiserver_round_trips_on_path"]["p99"] <= 1
    assert set(uc["default"]["allocate_breakdown_p50_ms"]) == {"kubelet_to_handler", "handler", "handler_to_kubelet"}
    assert set(d["allocate_p50_ms_by_gpu"]) == {"0", "1"}
    assert topo["tp_pair_allreduce"]["busbw_GBps"] > 0 and topo["backend"] == "gloo"
    # the control-plane A/B is in the same line: default vs the reference's cost model
    ab = d["allocate_by_mode"]
    assert ab["reference@5ms"]["apiserver_round_trips_on_path"]["p50"] == 2
    assert ab["default@5ms"]["allocate_p50_ms"] < ab["reference@5ms"]["allocate_p50_ms"]


def test_bench_torchrun_four_ranks_gloo():
    """N=4: ranks outside the TP pair take the non-member path of its group, and admissions from
    four churn pipelines interleave through rank 0's admission service (the shape of the
    driver's 8-GPU run)."""
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
                        "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", "4",
                        "--no-gpu", "--steps", "3", "--warmup", "1", "--compare-rtts", ""],
                       cwd=ROOT, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, MASTER_ADDR="127.0.0.1"))
    assert r.returncode == 0, r.stderr[-3000:]
    d = parse(r.stdout)
    assert d["n_gpus"] == 4 and d["pods_per_node"] == 16 and d["hbm_gib_per_node"] == 4 * 288
    assert d["failed_admissions"] == 0 and d["value"] > 0
    assert len(d["topology"]["tp_pair"]) == 2 and d["topology"]["pair_hops"] == 1


def test_tp_pair_demo_gloo():
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "-m",
                        "aliyun_gpushare_device_plugin_amd.parallel.tp_demo", "--iters", "2"],
                       cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = parse(r.stdout)
    assert d["world"] == 2 and d["tp_block_rel_err"] < 1e-3 and d["backend"] == "gloo"


def test_bench_fails_loudly_on_a_broken_topology(tmp_path):
    """Round-2 review item 7: with N>1 a topology export that is not one-hop xGMI on a healthy
    node (here: a fake 2-GPU node whose pair is PCIe) fails the run (exit 3) while still
    printing its measurement line with the verdict."""
    spec = tmp_path / "pcie.json"
    spec.write_text(json.dumps({"devices": [{"vram_total": 288 << 30}, {"vram_total": 288 << 30}], "xgmi": "none"}))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", "2",
                        "--no-gpu", "--steps", "2", "--warmup", "0", "--smi-backend", f"fake:{spec}",
                        "--compare-rtts", "", "--fill-orders", ""],
                       cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode != 0
    d = parse(r.stdout)
    assert d["topology"]["verdict"] == "fail" and "pcie" in d["topology"]["reasons"][0]
    assert "topology verdict FAIL" in r.stderr


def test_topology_verdict_rules():
    from aliyun_gpushare_device_plugin_amd.parallel import topology as T

    full = {"link_type": [["self", "xgmi"], ["xgmi", "self"]], "hops": [[0, 1], [1, 0]]}
    assert T.verdict(full, 2) == (True, [])
    assert not T.verdict(None, 2)[0]
    assert "expected 4x4" in T.verdict(full, 4)[1][0]
    pcie = {"link_type": [["self", "pcie"], ["pcie", "self"]], "hops": [[0, 3], [3, 0]]}
    assert not T.verdict(pcie, 2)[0]
    assert T.verdict(pcie, 2, healthy=[True, False]) == (True, [])     # a sick GPU excuses its links


def test_bench_plain_multi_gpu_runs_every_gpu():
    """Round-3 review item 1: ``bench.py --gpus 4`` without a launcher re-launches itself as 4
    ranks (before touching any GPU), so every GPU churns: 4 x steps real admissions, a p50 per
    GPU and a topology verdict — not one pipeline divided by 4x the admissions."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "4", "--no-gpu", "--steps", "4", "--warmup", "1",
                        "--compare-rtts", "", "--fill-orders", ""],
                       cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "torch.distributed.run" in r.stderr
    d = parse(r.stdout)
    assert d["n_gpus"] == 4 and d["admissions"] == 16
    assert d["admissions_by_gpu"] == {"0": 4, "1": 4, "2": 4, "3": 4}
    assert all(d["allocate_p50_ms_by_gpu"][str(g)] is not None for g in range(4))
    assert d["topology"]["verdict"] == "pass" and "run_problems" not in d
    assert abs(d["value"] - d["admissions"] / (d["ms_per_step"] * d["steps"] / 1e3)) < 0.05 * d["value"]


def test_bench_fails_when_a_gpu_does_no_work():
    """A rank whose pipeline never churns makes the run fail (exit 4) and is named in the line;
    the value counts only the admissions that happened."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["GS_BENCH_IDLE_RANK"] = "1"
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--no-gpu", "--steps", "3", "--warmup", "0",
                        "--compare-rtts", "", "--fill-orders", "", "--no-ref-churn"],
                       cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode != 0
    d = parse(r.stdout)
    assert d["admissions"] == 3 and d["admissions_by_gpu"] == {"0": 3, "1": 0}
    assert any("GPU 1" in p for p in d["run_problems"]) and "run FAILED" in r.stderr


def test_pod_zygote_forks_standby_pods_that_serve_their_own_pipes():
    """The bench's standby pods are forked from one interpreter that imported torch once: each
    child answers "standby" on its own pipe, with its own pid, and exits when its stdin closes.
    Closing the zygote ends it. (CPU: the child is told nothing more than to go away.)"""
    sys.path.insert(0, ROOT)
    import bench

    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    z = bench._Zygote(env)
    try:
        kids = [z.fork() for _ in range(3)]
        pids = set()
        for k in kids:
            ev = json.loads(k.stdout.readline())
            assert ev == {"event": "standby", "pid": k.pid}
            pids.add(k.pid)
        assert len(pids) == 3 and z._proc.pid not in pids
        assert all(k.poll() is None for k in kids)
        for k in kids:
            k.stdin.close()
            assert k.wait(30) == 0
            assert k.stdout.read() == ""
    finally:
        z.close()
    assert z._proc.returncode == 0


def test_a_dead_pod_zygote_fails_the_fork_loudly():
    """A zygote that died answers no fork: the bench gets an error at once, not a hang."""
    import pytest

    sys.path.insert(0, ROOT)
    import bench

    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    z = bench._Zygote(env)
    try:
        k = z.fork()
        assert json.loads(k.stdout.readline())["event"] == "standby"
        z._proc.kill()
        z._proc.wait(30)
        with pytest.raises((RuntimeError, OSError)):
            z.fork()
        k.stdin.close()
        assert k.wait(30) == 0                # its forked standby is a process of its own
    finally:
        z.close()
