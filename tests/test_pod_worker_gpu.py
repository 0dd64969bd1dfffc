"""The bench's pod process on an MI355X (``models/pod_worker.py``): a standby, forked from the
zygote or started as a fresh interpreter, gets its pod's env and runs under the quota shim.
It reads the quota back, holds its share, runs GEMMs and frees everything when stopped."""
from __future__ import annotations

import json
import os
import sys
import uuid

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GIB = 1 << 30


def _events(proc, want):
    """The pod's next ``want`` event (the test's own timeout bounds the wait)."""
    while True:
        ln = proc.stdout.readline()
        assert ln, f"pod {proc.pid} exited before {want!r}"
        if ln.startswith("{"):
            ev = json.loads(ln)
            if ev.get("event") == want:
                return ev


@pytest.mark.parametrize("how", ["forked", "fresh"])
def test_a_standby_becomes_a_pod_under_the_shim(how):
    import subprocess

    sys.path.insert(0, ROOT)
    import bench

    env = bench.PodFleet._pod_env()
    name = f"/gs-test-{uuid.uuid4().hex[:12]}"
    z = None
    if how == "forked":
        z = bench._Zygote(env)
        p = z.fork()
    else:
        p = subprocess.Popen([sys.executable, "-m", "aliyun_gpushare_device_plugin_amd.models.pod_worker"], env=env,
                             stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, bufsize=1)
    try:
        assert _events(p, "standby")["pid"] == p.pid
        quota = 8 * GIB
        p.stdin.write(json.dumps({"cmd": "start", "env": {"GPUSHARE_QUOTA_BYTES": quota, "GPUSHARE_LEDGER": name},
                                  "gemm": 1024, "burst": 2, "fill": 0.5}) + "\n")
        ready = _events(p, "ready")
        assert ready["quota"] == quota                       # the shim's quota, read back by the pod
        assert ready["held"] >= quota // 2
        assert ready["shim"] is not None and ready["shim"]["denied"] == 0
        p.stdin.write('{"cmd":"stats"}\n')
        assert _events(p, "stats")["gemms"] >= 1
        p.stdin.write('{"cmd":"stop"}\n')
        done = _events(p, "done")
        assert done["gemms"] >= 1 and set(done["stop_ms"]) == {"burst_in_flight", "free", "arena_release"}
        assert done["used_after_release"] is not None and done["used_after_release"] < quota // 4
        assert p.wait(60) == 0
    finally:
        if p.poll() is None:
            p.kill()
        if z is not None:
            z.close()
        try:
            os.unlink("/dev/shm" + name)
        except FileNotFoundError:
            pass
