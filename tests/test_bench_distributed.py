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
    assert topo["tp_pair_allreduce"]["busbw_GBps"] > 0 and topo["backend"] == "gloo"
    # the control-plane A/B is in the same line: default vs the reference's cost model
    ab = d["allocate_by_mode"]
    assert ab["reference@5ms"]["apiserver_round_trips_on_path"] == 2
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
