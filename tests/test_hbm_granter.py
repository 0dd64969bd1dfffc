"""The plugin's HBM granter (``quota/hbmbroker.py`` HBMGranter) with real broker processes on the
stub HIP runtime and real pod processes under the quota shim (``stub_runtime``): the broker path
must hold under any start order and any restart, as the reference's stateless plugin does after a
restart (``pkg/gpu/nvidia/gpumanager.go:63-108``).

* the plugin starts 5 s before the broker: every pod still takes its arena;
* the broker is killed and relaunched by ``gpushare-hbm-brokers`` while pods run: the granter sees
  the new boot id and re-grants, and a restarted container gets its arena back;
* the plugin is SIGKILLed and restarted: the replayed answer's token (node secret) is granted;
* a deleted pod's token is revoked and refused;
* an 8-rank gloo rehearsal of bench.py with a stub broker per rank: every broker serves its pods.
"""
from __future__ import annotations

import json
import os
import signal
import socket
import subprocess
import sys
import time
import uuid

import pytest
from aliyun_gpushare_device_plugin_amd.utils.native import preload

from aliyun_gpushare_device_plugin_amd.cli import hbmbroker as cli
from aliyun_gpushare_device_plugin_amd.quota import hbmbroker as hb

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GIB = 1 << 30
QUOTA = 4 * GIB                     # 94 % in whole granules: a 3-granule arena


def broker(stub, host, gpu=0, gib=12, policy="exit"):
    return hb.HBMBroker.for_gpu(str(host), gpu, gib=gib, exe=os.path.join(stub, "gpushare-hbm-broker"),
                                env=dict(os.environ, LD_LIBRARY_PATH=stub),
                                extra_args=["--ungranted-wait-s", "10", "--release-policy", policy])


def pod(stub, native_shim, host, token, args, gpu=0, wait_s=30, **extra_env):
    """A pod's container process: the stub runtime under the quota shim, its env as the plugin's
    answer gives it (host paths: no container here)."""
    env = dict(os.environ, LD_PRELOAD=preload(native_shim), LD_LIBRARY_PATH=stub, GPUSHARE_QUOTA_BYTES=str(QUOTA),
               GPUSHARE_LEDGER=f"/gs-test-{uuid.uuid4().hex[:12]}", GPUSHARE_HBM_BROKER=hb.pod_socket(str(host), gpu),
               GPUSHARE_HBM_TOKEN=token, GPUSHARE_HBM_WAIT_S=str(wait_s), **{k: str(v) for k, v in extra_env.items()})
    return subprocess.Popen([os.path.join(stub, "shim_driver"), *map(str, args)], env=env, stdin=subprocess.PIPE,
                            stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)


def lines_until(p, op, timeout=30.0):
    out = []
    end = time.monotonic() + timeout
    while time.monotonic() < end:
        ln = p.stdout.readline()
        if not ln:
            break
        if ln.startswith("{"):
            out.append(json.loads(ln))
            if out[-1]["op"] == op:
                return out
    raise AssertionError(f"no {op!r} from the pod: {out} / {p.stderr.read() if p.poll() is not None else ''}")


def wait_for(cond, timeout=15.0, what=""):
    end = time.monotonic() + timeout
    while time.monotonic() < end:
        v = cond()
        if v:
            return v
        time.sleep(0.05)
    raise AssertionError(f"timed out waiting for {what}")


def take(path, token):
    s = socket.socket(socket.AF_UNIX)
    s.settimeout(15)
    s.connect(path)
    s.sendall(f"TAKE {token}\n".encode())
    h = b""
    while not h.endswith(b"\n"):
        c = s.recv(1)
        if not c:
            break
        h += c
    return s, h.decode().strip()


def test_broker_state_is_exported_as_metrics(stub_runtime, native_shim, tmp_path):
    """The plugin's /metrics carries each broker's state from its last STAT:
    up, granules by state, takes / releases, and the granter's own grant counters."""
    from aliyun_gpushare_device_plugin_amd.utils.metrics import Registry

    host = tmp_path / "hbm"
    b = broker(stub_runtime, host)
    b.start()
    g = hb.HBMGranter(str(host), poll_s=0.1, startup_grace_s=0.0, live=lambda: {})
    try:
        assert g.reconcile_now()                                   # the broker is seen: answers carry tokens
        assert g.submit(0, g.token("m1", 0), QUOTA) and g.flush()
        p = pod(stub_runtime, native_shim, host, g.token("m1", 0), ["alloc", GIB, "arena", "freeall", "arenarelease"])
        assert p.wait(30) == 0
        assert g.reconcile_now()
        reg = Registry()
        reg.add_collector(g.exposition)
        text = reg.render()
        assert 'gpushare_hbm_broker_up{gpu="0"} 1' in text
        assert 'gpushare_hbm_broker_granules{gpu="0",state="granules"} 12' in text
        assert 'gpushare_hbm_broker_takes_total{gpu="0"} 1' in text
        assert 'gpushare_hbm_broker_releases_total{gpu="0"} 1' in text
        assert 'gpushare_hbm_granter_total{op="grants"} 1' in text
    finally:
        g.stop()
        b.stop()


def test_plugin_before_broker_every_pod_takes_its_arena(stub_runtime, native_shim, tmp_path):
    host = tmp_path / "hbm"
    g = hb.HBMGranter(str(host), poll_s=0.2, startup_grace_s=60.0, live=lambda: {})
    b = None
    pods = []
    try:
        toks = [g.token(f"uid-{k}", 0) for k in range(3)]
        assert all(g.submit(0, t, QUOTA) for t in toks)          # no broker yet: pending, the token rides
        pods = [pod(stub_runtime, native_shim, host, t, ["alloc", GIB, "arena", "stats"]) for t in toks]
        time.sleep(5.0)
        assert all(p.poll() is None for p in pods)               # their shims wait for the broker
        b = broker(stub_runtime, host)
        b.start()
        for p in pods:
            out = lines_until(p, "stats")
            alloc, arena, st = out[-3:]
            assert alloc["err"] == 0 and arena == {"op": "arena", "on": 1, "size": 3 * GIB, "used": GIB}, out
            assert st["used"] == 3 * GIB                          # the arena on the pod's ledger
            p.wait(10)
        st = b.stat()
        assert st["takes"] == 3 and st["timeouts"] == 0 and st["grants"] == 3
        assert g.stats()["failures"] == 0 or g.stats()["grants"] >= 3
    finally:
        for p in pods:
            if p.poll() is None:
                p.kill()
        g.stop()
        if b is not None:
            assert b.stop() == 0


def test_broker_restart_regrants_and_a_restarted_container_gets_its_arena(stub_runtime, native_shim, tmp_path,
                                                                          monkeypatch):
    host = tmp_path / "hbm"
    brokers = {0: broker(stub_runtime, host)}
    sup = cli.Supervisor(brokers, backoff_s=0.1)
    sup.start()
    g = None
    p1 = p2 = None
    try:
        tok = hb.HBMGranter(str(host), start=False).token("uid-r", 0)
        live = {tok: (0, QUOTA)}
        g = hb.HBMGranter(str(host), poll_s=0.1, startup_grace_s=0.0, revoke_grace_s=0.5, live=lambda: dict(live))
        assert g.reconcile_now() and brokers[0].list()["grants"] == {tok: 3}
        p1 = pod(stub_runtime, native_shim, host, tok, ["alloc", GIB, "arena", "wait"])
        assert lines_until(p1, "arena")[-1]["on"] == 1
        boot1 = brokers[0].stat()["boot"]
        brokers[0].proc.send_signal(signal.SIGKILL)               # the broker dies under a running pod
        brokers[0].proc.wait()
        sup.watch_once()                                          # the launcher starts it again
        assert sup.restarts == {0: 1}
        boot2 = brokers[0].stat()["boot"]
        assert boot2 != boot1
        wait_for(lambda: brokers[0].list()["grants"] == {tok: 3}, what="the re-grant")
        assert g.stats()["regrants"] == 1
        p1.kill()                                                 # the container restarts (same env)
        p1.wait()
        p2 = pod(stub_runtime, native_shim, host, tok, ["alloc", GIB, "arena"])
        assert lines_until(p2, "arena")[-1] == {"op": "arena", "on": 1, "size": 3 * GIB, "used": GIB}
        p2.wait(10)
        assert brokers[0].stat()["takes"] == 1
    finally:
        for p in (p1, p2):
            if p is not None and p.poll() is None:
                p.kill()
        if g is not None:
            g.stop()
        sup.stop()


GRANTER_PROC = """
import sys, time
sys.path.insert(0, {root!r})
from aliyun_gpushare_device_plugin_amd.quota import hbmbroker as hb
host, uid = sys.argv[1], sys.argv[2]
box = {{}}
g = hb.HBMGranter(host, poll_s=0.1, startup_grace_s=0.0, live=lambda: {{box["tok"]: (0, {quota})}})
box["tok"] = g.token(uid, 0)
print(box["tok"], flush=True)
time.sleep(600)
"""


def test_plugin_restart_grants_the_replayed_token(stub_runtime, native_shim, tmp_path):
    """The plugin process is SIGKILLed and a new one starts: its tokens come from the node secret,
    so the answer a replay hands out (the journal's bytes, token included) is granted by the new
    process — here on a broker that lost its grants meanwhile (it restarted too)."""
    host = tmp_path / "hbm"
    b = broker(stub_runtime, host)
    b.start()
    code = GRANTER_PROC.format(root=ROOT, quota=QUOTA)
    procs = []
    try:
        p1 = subprocess.Popen([sys.executable, "-c", code, str(host), "uid-replayed"], stdout=subprocess.PIPE, text=True)
        procs.append(p1)
        tok = p1.stdout.readline().strip()
        wait_for(lambda: b.list()["grants"].get(tok) == 3, what="the first instance's grant")
        p1.send_signal(signal.SIGKILL)
        p1.wait()
        assert b.stop() == 0
        b.start()                                                 # grants gone
        assert b.list()["grants"] == {}
        p2 = subprocess.Popen([sys.executable, "-c", code, str(host), "uid-replayed"], stdout=subprocess.PIPE, text=True)
        procs.append(p2)
        assert p2.stdout.readline().strip() == tok                # same node secret, same token
        wait_for(lambda: b.list()["grants"].get(tok) == 3, what="the new instance's grant")
        p = pod(stub_runtime, native_shim, host, tok, ["alloc", GIB, "arena"])
        assert lines_until(p, "arena")[-1]["on"] == 1
        p.wait(10)
        assert oct(os.stat(hb.secret_path(str(host))).st_mode & 0o777) == "0o600"
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        b.stop()


def test_deleted_pods_token_is_revoked_and_refused(stub_runtime, tmp_path):
    host = tmp_path / "hbm"
    b = broker(stub_runtime, host)
    b.start()
    g = None
    try:
        g0 = hb.HBMGranter(str(host), start=False)
        keep, gone = g0.token("uid-keep", 0), g0.token("uid-gone", 0)
        stale = "f" * 32                                     # granted by nobody this granter knows
        b.grant(stale, 2 * GIB)
        live = {keep: (0, QUOTA), gone: (0, QUOTA)}
        g = hb.HBMGranter(str(host), poll_s=0.1, startup_grace_s=0.0, revoke_grace_s=0.3, live=lambda: dict(live))
        wait_for(lambda: set(b.list()["grants"]) == {keep, gone}, what="grants, and the stale one revoked")
        del live[gone]                                        # the pod is deleted
        wait_for(lambda: set(b.list()["grants"]) == {keep}, what="the revocation")
        s, head = take(b.socket_path, gone)
        assert head == "ERR revoked"
        s.close()
        s, head = take(b.socket_path, keep)
        assert head.startswith("FDS 3 ")
        s.close()
        # (the count moves once the REVOKE's answer is back: after the broker already dropped it)
        wait_for(lambda: g.stats()["revokes"] == 2, what="both revocations counted")
        # a granter without a pod view revokes nothing
        g.stop()
        g = hb.HBMGranter(str(host), poll_s=0.1, startup_grace_s=0.0, revoke_grace_s=0.0, live=lambda: None)
        assert g.reconcile_now() and set(b.list()["grants"]) == {keep}
    finally:
        if g is not None:
            g.stop()
        b.stop()


def test_broker_down_for_good_answers_lose_the_token_and_get_it_back(stub_runtime, tmp_path):
    host = tmp_path / "hbm"
    calls = []
    g = hb.HBMGranter(str(host), poll_s=0.1, startup_grace_s=0.3, down_grace_s=0.5, live=lambda: {},
                      on_readiness=lambda: calls.append(time.monotonic()))
    b = None
    try:
        hb.prepare_dirs(str(host), [0])
        assert g.submit(0, g.token("u1", 0), QUOTA)          # within the start-up grace
        time.sleep(0.6)
        assert g.reconcile_now()
        assert not g.submit(0, g.token("u2", 0), QUOTA)      # never came: no token, driver at once
        assert calls                                         # the engine was told to re-prepare
        b = broker(stub_runtime, host)
        b.start()
        wait_for(lambda: g.submit(0, g.token("u3", 0), QUOTA), what="readiness")
        wait_for(lambda: len(calls) >= 2, what="the engine told again")   # (at the end of that pass)
        assert g.flush() and set(b.list()["grants"]) >= {g.token("u1", 0), g.token("u3", 0)}
    finally:
        g.stop()
        if b is not None:
            b.stop()


def test_bench_rehearsal_eight_ranks_with_stub_brokers(stub_runtime):
    """bench.py as the driver runs it at N=8 (torchrun, one rank per GPU), on CPU over gloo, with
    the broker path live: every rank starts its GPU's (stub) broker, the barrier holds the fill
    until all 8 listen, and every admitted pod takes its arena from its own GPU's broker."""
    port = socket.socket()
    port.bind(("127.0.0.1", 0))
    pnum = port.getsockname()[1]
    port.close()
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
                        "--master-addr", "127.0.0.1", "--master-port", str(pnum), "bench.py", "--gpus", "8",
                        "--no-gpu", "--steps", "2", "--warmup", "0", "--compare-rtts", "", "--fill-orders", "",
                        "--no-ref-churn", "--stub-runtime", stub_runtime],
                       cwd=ROOT, capture_output=True, text=True, timeout=600, env=dict(os.environ, MASTER_ADDR="127.0.0.1"))
    assert r.returncode == 0, r.stderr[-4000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["n_gpus"] == 8 and d["failed_admissions"] == 0 and "run_problems" not in d
    by = d["hbm_broker_by_gpu"]
    assert sorted(by) == [str(i) for i in range(8)]
    for gpu, st in by.items():
        assert st["takes"] > 0 and st["timeouts"] == 0, (gpu, st)
    # every pod started on every GPU (4 at the fill + the churn's replacements) had its arena
    assert d["stub_pods_with_arena_by_gpu"] == {str(i): 4 + d["admissions_by_gpu"][str(i)] for i in range(8)}
    assert d["quota_denials"] == 0
    # the line explains itself per GPU: each GPU's broker STAT (above) and its Allocate p50
    assert sorted(d["allocate_p50_ms_by_gpu"]) == [str(i) for i in range(8)]
