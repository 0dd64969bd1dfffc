"""The per-GPU HBM broker (native/hbmbroker) and the quota shim's broker arena, on MI355X.

A pod under the shim with ``GPUSHARE_HBM_BROKER``/``GPUSHARE_HBM_TOKEN`` takes its granted
granules at its first allocation and serves every ``hipMalloc`` from them. Checked here:
the next pod sees only zeros (the broker scrubbed), a pod waits for granules a retiring pod still
holds instead of failing, and a pod with an unknown token gets no arena.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import time

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
GIB = 1 << 30

TENANT = r"""
import ctypes, faulthandler, json, sys, time
faulthandler.enable()
import torch
mode = sys.argv[1]
t0 = time.perf_counter()
x = torch.empty(5 * (1 << 30), dtype=torch.uint8, device="cuda")      # inside the arena
t1 = time.perf_counter()
lib = ctypes.CDLL(None)
size, used = ctypes.c_uint64(), ctypes.c_uint64()
on = lib.gpushare_shim_arena_stats(ctypes.byref(size), ctypes.byref(used))
out = {"arena": on, "arena_size": size.value, "arena_used": used.value, "alloc_ms": (t1 - t0) * 1e3,
       "free_total": list(torch.cuda.mem_get_info())}
if mode == "check":
    out["nonzero"] = int(x.max().item())                               # a reduction: no full-size temporary
x.fill_(7)
torch.cuda.synchronize()
if mode == "hold":
    print(json.dumps(out), flush=True)
    sys.stdin.readline()                                               # hold until told to exit
else:
    print(json.dumps(out), flush=True)
"""


@pytest.fixture
def broker(tmp_path):
    from aliyun_gpushare_device_plugin_amd.quota.hbmbroker import HBMBroker

    b = HBMBroker(str(tmp_path / "hbm.sock"), device=0, gib=8, wait_s=20)
    b.start()
    yield b
    b.stop()


def _settled(broker, timeout=5.0) -> dict:
    """The broker's counters once no released granule is quarantined any more (a retired
    tenant's references drop when the kernel has torn its process down)."""
    deadline = time.time() + timeout
    st = broker.stat()
    while st["quarantined"] and time.time() < deadline:
        time.sleep(0.02)
        st = broker.stat()
    return st


def _tenant(broker, token, mode, **kw):
    from aliyun_gpushare_device_plugin_amd.utils.native import ensure_built

    env = dict(os.environ, LD_PRELOAD=ensure_built("hipshim"), GPUSHARE_QUOTA_BYTES=str(8 * GIB),
               GPUSHARE_HBM_BROKER=broker.socket_path, GPUSHARE_HBM_TOKEN=token, GPUSHARE_SHIM_LOG="1",
               PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    return subprocess.Popen([sys.executable, "-c", TENANT, mode], env=env, stdin=subprocess.PIPE,
                            stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, **kw)


def _result(p, timeout=120):
    out, err = p.communicate(timeout=timeout)
    assert p.returncode == 0, err[-3000:]
    return json.loads(out.strip().splitlines()[-1])


def test_the_next_pod_sees_only_zeros(broker):
    assert broker.grant("a" * 32, 6 * GIB) == 6
    a = _result(_tenant(broker, "a" * 32, "write"))
    assert a["arena"] == 1 and a["arena_size"] == 6 * GIB and a["arena_used"] >= 5 * GIB
    # what the pod sees as free is the arena's rest, under a total of its quota
    assert a["free_total"][1] == 8 * GIB and a["free_total"][0] <= GIB
    assert broker.grant("b" * 32, 6 * GIB) == 6
    b = _result(_tenant(broker, "b" * 32, "check"))
    assert b["arena"] == 1 and b["nonzero"] == 0
    st = _settled(broker)
    assert st["takes"] == 2 and st["releases"] == 2 and st["free"] == st["granules"]
    assert st["scrubbed_bytes"] >= 12 * GIB


def test_a_restarted_container_takes_its_grant_again(broker):
    """A grant belongs to the pod: after its process exits (a container restart keeps the env and
    the token), the next process with the same token gets its granules back, zeroed."""
    broker.grant("r" * 32, 6 * GIB)
    first = _result(_tenant(broker, "r" * 32, "write"))
    again = _result(_tenant(broker, "r" * 32, "check"), timeout=60)
    assert first["arena"] == 1 and again["arena"] == 1 and again["nonzero"] == 0
    st = broker.stat()
    assert st["takes"] == 2 and st["timeouts"] == 0


def test_a_pod_waits_for_granules_a_retiring_pod_holds(broker):
    broker.grant("c" * 32, 6 * GIB)
    holder = _tenant(broker, "c" * 32, "hold")
    first = json.loads(holder.stdout.readline())
    assert first["arena"] == 1
    broker.grant("d" * 32, 6 * GIB)                       # 6 + 6 > 8: must wait for the holder
    waiter = _tenant(broker, "d" * 32, "check")
    time.sleep(3.0)
    assert waiter.poll() is None and broker.stat()["waiting"] == 1
    holder.stdin.write("\n")
    holder.stdin.flush()
    holder.wait(60)
    r = _result(waiter)
    assert r["arena"] == 1 and r["nonzero"] == 0


def test_an_unknown_token_gets_no_arena(tmp_path):
    from aliyun_gpushare_device_plugin_amd.quota.hbmbroker import HBMBroker

    b = HBMBroker(str(tmp_path / "hbm.sock"), device=0, gib=4, wait_s=1)
    b.start()
    try:
        r = _result(_tenant(b, "never-granted", "write"))
        assert r["arena"] == 0                           # refused: the pod's allocations go to the driver
        assert b.stat()["timeouts"] == 1
    finally:
        b.stop()


def test_launcher_brings_up_the_broker_of_every_gpu_by_pci_address(tmp_path):
    """The node launcher (``gpushare-hbm-brokers``) on the box: one broker per GPU of the SMI
    enumeration, found by PCI address, answering on <dir>/hbm<index>.sock; a pod takes a grant
    from it."""
    from aliyun_gpushare_device_plugin_amd.cli import hbmbroker as cli
    from aliyun_gpushare_device_plugin_amd.device.smi import SMI

    with SMI("auto") as s:
        gpus = [s.device(i) for i in range(s.count())]
    d = tmp_path / "hbm"
    d.mkdir()
    brokers = {g.index: cli.HBMBroker(str(d / cli.socket_name(g.index)), pci_bus_id=g.bdf, gib=8)
               for g in gpus[:1]}
    sup = cli.Supervisor(brokers)
    try:
        sup.start()
        b = brokers[gpus[0].index]
        assert b.stat()["granules"] == 8
        b.grant("e" * 32, 6 * GIB)
        r = _result(_tenant(b, "e" * 32, "check"))
        assert r["arena"] == 1 and r["nonzero"] == 0
    finally:
        sup.stop()


def test_broker_under_asan(tmp_path, monkeypatch):
    """The broker built with ASan+UBSan (host code: it is compiled by g++, the scrub is a HIP
    runtime memset), through grants, takes, a waiting take and releases, against the real HIP
    runtime. Built beforehand: ``python native/build.py hbmbroker --sanitize asan``."""
    from aliyun_gpushare_device_plugin_amd.quota.hbmbroker import HBMBroker
    from aliyun_gpushare_device_plugin_amd.utils.native import NATIVE_DIR

    exe = os.path.join(NATIVE_DIR, "asan", "gpushare-hbm-broker")
    if not os.path.exists(exe):
        pytest.skip("ASan broker not built")
    monkeypatch.setenv("GPUSHARE_HBM_BROKER_EXE", exe)
    monkeypatch.setenv("ASAN_OPTIONS", "detect_leaks=0:halt_on_error=1")
    monkeypatch.setenv("UBSAN_OPTIONS", "halt_on_error=1:print_stacktrace=1")
    b = HBMBroker(str(tmp_path / "hbm.sock"), device=0, gib=8, wait_s=20)
    b.start()
    rc = None
    try:
        b.grant("s" * 32, 6 * GIB)
        holder = _tenant(b, "s" * 32, "hold")
        assert json.loads(holder.stdout.readline())["arena"] == 1
        b.grant("t" * 32, 6 * GIB)
        waiter = _tenant(b, "t" * 32, "check")
        time.sleep(1.0)
        holder.stdin.write("\n")
        holder.stdin.flush()
        holder.wait(60)
        r = _result(waiter)
        assert r["arena"] == 1 and r["nonzero"] == 0
        st = b.stat()
        assert st["takes"] == 2 and st["releases"] == 2
    finally:
        rc = b.stop()
    assert rc == 0, b.last_stderr[-3000:]
    assert "AddressSanitizer" not in b.last_stderr and "runtime error" not in b.last_stderr


def test_granules_a_tenant_still_refers_to_are_not_lent_again(broker):
    """A tenant that keeps its granules' dma-buf fds (or hands them to another process) after
    its connection ends must not share them with the next pod: the broker sees the references
    (the dma-buf's fdinfo count), keeps the granules out of the free list, and scrubs and lends
    them only once the last reference is gone."""
    import socket

    broker.grant("q" * 32, 2 * GIB)
    s = socket.socket(socket.AF_UNIX)
    s.settimeout(10)
    s.connect(broker.socket_path)
    s.sendall(b"TAKE " + b"q" * 32 + b"\n")
    head = b""
    while not head.endswith(b"\n"):
        head += s.recv(1)
    assert head.decode().startswith("FDS 2 ")
    _, fds, _, _ = socket.recv_fds(s, 1, 200)
    assert len(fds) == 2
    s.close()                                    # released, but the fds are still held here
    deadline = time.time() + 5
    while broker.stat()["releases"] < 1 and time.time() < deadline:
        time.sleep(0.05)
    st = broker.stat()
    assert st["quarantined"] == 2 and st["free"] == st["granules"] - 2
    for fd in fds:
        os.close(fd)
    deadline = time.time() + 5
    while broker.stat()["quarantined"] and time.time() < deadline:
        time.sleep(0.05)
    st = broker.stat()
    assert st["quarantined"] == 0 and st["free"] == st["granules"] and st["quarantined_total"] == 2
