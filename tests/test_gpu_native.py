"""Real-MI355X tests of the native device layer and the quota shim (run with ``-m gpu``)."""
import json
import os
import subprocess
import sys
import textwrap

import pytest
from aliyun_gpushare_device_plugin_amd.utils.native import preload

from aliyun_gpushare_device_plugin_amd import const
from aliyun_gpushare_device_plugin_amd.device import smi as S
from aliyun_gpushare_device_plugin_amd.device.model import DeviceModel

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("backend", ["auto", "rocm_smi", "sysfs"])
def test_enumerates_mi355x(backend):
    with S.SMI(backend) as smi:
        assert smi.count() >= 1
        g = smi.device(0)
        assert g.gfx == "gfx950" or backend == "rocm_smi"
        assert g.vram_total > 280 * (1 << 30)          # 288 GB class HBM3E
        assert g.uuid.startswith("GPU-") and len(g.uuid) == 20
        assert g.render_minor >= 128
        assert os.path.exists(f"/dev/dri/renderD{g.render_minor}")


@pytest.mark.parametrize("backend", ["rocm_smi", "amdsmi"])
def test_backends_agree(backend):
    """rocm_smi and amdsmi enumerate the same GPUs, in the same (HIP ordinal) order, with the same
    HBM bytes, BDF, render node and link types as the sysfs/KFD view."""
    with S.SMI(backend) as a, S.SMI("sysfs") as b:
        assert a.backend == backend
        da, db = a.devices(), b.devices()
        assert [d.uuid for d in da] == [d.uuid for d in db]
        assert [d.vram_total for d in da] == [d.vram_total for d in db]
        assert [(d.bdf, d.render_minor) for d in da] == [(d.bdf, d.render_minor) for d in db]
        n = len(da)
        assert [[a.link(i, j).type for j in range(n)] for i in range(n)] == \
               [[b.link(i, j).type for j in range(n)] for i in range(n)]
        a.events_start()
        st = a.health_status()
        # the health path is live on MI355X: event notification armed on every GPU and the HBM
        # (UMC) ECC counters read on every GPU at the last refresh
        assert st["events_api"] == 1 and st["events_armed"] == n, st
        assert st["ecc_api"] == 1 and st["ecc_reads_ok"] == n and st["ecc_reads_failed"] == 0, st
        ev = a.wait_event(50)                     # no fault on a healthy box: a timeout
        assert ev is None or ev.kind in (1, 2, 3, 4), ev


def test_advertised_units_mi355x():
    with S.SMI("auto") as smi:
        m_near = DeviceModel(smi.devices(), const.GIB, "nearest")
        m_floor = DeviceModel(smi.devices(), const.GIB, "floor")
    assert m_near.units_of(0) == 288        # nominal capacity
    assert m_floor.units_of(0) in (287, 288)
    ids = m_near.device_list()
    assert len(ids) == 288 * m_near.count()


def test_hip_agrees_with_smi():
    code = "import torch;print(torch.cuda.get_device_properties(0).total_memory)"
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    with S.SMI("auto") as smi:
        assert int(r.stdout.strip().splitlines()[-1]) == smi.device(0).vram_total


QUOTA_SCRIPT = textwrap.dedent("""
    import json, torch
    free, total = torch.cuda.mem_get_info()
    props = torch.cuda.get_device_properties(0).total_memory
    out = {"free": free, "total": total, "props": props}
    x = torch.empty(int(total * 0.8) // 2, dtype=torch.bfloat16, device="cuda")
    out["ok_alloc"] = True
    try:
        y = torch.empty(int(total * 0.5) // 2, dtype=torch.bfloat16, device="cuda")
        out["over_alloc"] = "allowed"
    except torch.OutOfMemoryError:
        out["over_alloc"] = "denied"
    del x
    torch.cuda.empty_cache()
    z = torch.empty(int(total * 0.9) // 2, dtype=torch.bfloat16, device="cuda")
    out["after_free"] = True
    print(json.dumps(out))
""")


def _run_under_shim(env_extra, script=QUOTA_SCRIPT):
    from aliyun_gpushare_device_plugin_amd.utils.native import ensure_built
    env = dict(os.environ)
    env.update({"LD_PRELOAD": ensure_built("hipshim"), "GPUSHARE_SHIM_LOG": "1"})
    env.update({k: str(v) for k, v in env_extra.items()})
    r = subprocess.run([sys.executable, "-c", script], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1]), r.stderr


def test_shim_quota_under_pytorch():
    out, err = _run_under_shim({const.ENV_RESOURCE_BY_CONTAINER: 64, const.ENV_RESOURCE_BY_DEV: 288})
    with S.SMI("auto") as smi:
        real = smi.device(0).vram_total
    quota = real * 64 // 288
    assert out["total"] == quota and out["props"] == quota
    assert out["free"] <= quota
    assert out["ok_alloc"] and out["over_alloc"] == "denied" and out["after_free"]
    assert "quota" in err


def test_shim_expandable_segments_vmm_path():
    out, _ = _run_under_shim({const.ENV_RESOURCE_BY_CONTAINER: 32, const.ENV_RESOURCE_BY_DEV: 288,
                              "PYTORCH_HIP_ALLOC_CONF": "expandable_segments:True"})
    assert out["over_alloc"] == "denied"


def test_granule_matches_hardware():
    """hipMalloc consumes HBM in 2 MiB fragments on MI355X: the shim's default granule."""
    code = textwrap.dedent("""
        import ctypes, json, torch
        torch.cuda.init()
        hip = ctypes.CDLL("libamdhip64.so.7")
        res = {}
        for sz in (1, 4096, 2 << 20, (2 << 20) + 1, (64 << 20) + 4096):
            f0, t = ctypes.c_size_t(), ctypes.c_size_t()
            hip.hipMemGetInfo(ctypes.byref(f0), ctypes.byref(t))
            p = ctypes.c_void_p()
            assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(sz)) == 0
            f1 = ctypes.c_size_t()
            hip.hipMemGetInfo(ctypes.byref(f1), ctypes.byref(t))
            res[sz] = f0.value - f1.value
            hip.hipFree(p)
        print(json.dumps(res))
    """)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    res = {int(k): v for k, v in json.loads(r.stdout.strip().splitlines()[-1]).items()}
    g = 2 << 20
    for sz, delta in res.items():
        assert delta == (sz + g - 1) // g * g, (sz, delta)


def _probe(args, **env):
    """native/probes/shim_probe.hip under the shim (LD_PRELOAD, like a container process)."""
    from aliyun_gpushare_device_plugin_amd.utils.native import ensure_built
    exe = os.path.join(os.path.dirname(ensure_built("hipshim")), "shim_probe")
    e = dict(os.environ, LD_PRELOAD=preload(ensure_built("hipshim")), GPUSHARE_SHIM_LOG="1")
    e.update({k: str(v) for k, v in env.items()})
    r = subprocess.run([exe, *map(str, args)], env=e, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    return [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")], r.stderr


GIB, MIB = 1 << 30, 1 << 20


def test_shim_kfd_charge_equals_device_consumption():
    """At the KFD boundary the charge is the HBM the runtime takes: equal to the device's own
    accounting for every allocation of a 2 MiB fragment or more (sub-fragment buffers share a
    fragment the ledger already holds, so their charge is never above the device's)."""
    out, err = _probe(["granule", "smalls", 100, 4096, "smalls", 20, 3 * MIB], GPUSHARE_QUOTA_BYTES=64 * GIB)
    assert "mode kfd" in err
    for row in out:
        if row.get("requested", row.get("size", 0)) >= 2 * MIB - 1:
            assert row["shim_charge"] == row["device_bytes"], row
        else:
            assert row["shim_charge"] <= row["device_bytes"] <= 2 * MIB, row


def test_shim_kfd_charges_pool_retention_and_scratch():
    """What the HIP-level hooks could not see (round-1 review): a stream-ordered pool's block
    stays charged until the pool trims, and a scratch-heavy kernel's private-segment buffer —
    allocated inside the runtime, no HIP allocation call — is charged."""
    out, _ = _probe(["pool", GIB, "scratch", 4], GPUSHARE_QUOTA_BYTES=64 * GIB)
    pool, scratch = out
    assert pool["rc"] == [0, 0, 0, 0]
    assert pool["after_alloc"] - pool["used_before"] >= GIB
    assert pool["after_trim"] <= pool["after_alloc"] - GIB
    assert scratch["rc"] == [0, 0]
    assert scratch["after_launch"] - scratch["used_before"] >= GIB         # ~2 GiB of scratch on 256 CUs
    assert scratch["device_delta"] > 0


def test_shim_kfd_denial_is_clean():
    """Over quota the KFD allocation fails with ENOMEM, as on a full GPU: hipMalloc returns
    hipErrorOutOfMemory and the process keeps working within its quota."""
    out, _ = _probe(["alloc", 256 * MIB, "alloc", GIB, "alloc", 256 * MIB], GPUSHARE_QUOTA_BYTES=768 * MIB)
    assert [o["rc"] for o in out] == [0, 2, 0]
    assert out[1]["denied"] >= 1 and out[2]["used"] <= 768 * MIB


def _gpus() -> int:
    with S.SMI("auto") as s:
        return s.count()


def test_xgmi_matrix_on_multi_gpu_node():
    """On an MI355X UBB every GPU pair is one xGMI hop; the exported matrix must say so
    (round-1 review: only fake fixtures had been seen). Needs >= 2 visible GPUs."""
    from aliyun_gpushare_device_plugin_amd.parallel import topology as T

    if _gpus() < 2:
        pytest.skip("needs >= 2 GPUs (runs on the 8-GPU node)")
    with S.SMI("auto") as s:
        topo = T.build_topology(s)
    n = len(topo["gpus"])
    for i in range(n):
        for j in range(n):
            if i != j:
                assert topo["link_type"][i][j] == "xgmi" and topo["hops"][i][j] == 1, (i, j, topo)
    assert T.best_group(topo, [288] * n, 2, 64) is not None


def test_rccl_tp_pair_allreduce():
    """The RCCL TP-pair demo on two GPUs (torch.distributed 'nccl' = RCCL over xGMI): numerics
    of the tensor-parallel block and a non-trivial bus bandwidth. Needs >= 2 visible GPUs."""
    if _gpus() < 2:
        pytest.skip("needs >= 2 GPUs (runs on the 8-GPU node)")
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), "-m",
                        "aliyun_gpushare_device_plugin_amd.parallel.tp_demo", "--iters", "10"],
                       cwd=root, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["backend"] == "nccl" and d["tp_block_rel_err"] < 5e-2 and d["busbw_GBps"] > 10


def test_rccl_single_rank_tp_block_on_mi355x():
    """The RCCL path on the 1-GPU box: the TP demo as one rank (torch.distributed 'nccl' = RCCL
    on ROCm; communicator init, the all-reduce kernels, the MFMA GEMM block) — the 2-GPU pair
    test above needs the 8-GPU node."""
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), "-m",
                        "aliyun_gpushare_device_plugin_amd.parallel.tp_demo", "--iters", "5"],
                       cwd=root, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["backend"] == "nccl" and d["world"] == 1 and d["tp_block_rel_err"] < 5e-2
    assert d["allreduce_bytes"] == 256 << 20 and d["allreduce_ms"] > 0


def test_hbm_used_gauge_matches_sysfs():
    """gpushare_hbm_used_bytes{gpu} (set from the health poll's SMI sample) tracks amdgpu's
    mem_info_vram_used while this process holds 8 GiB on GPU 0."""
    import time

    import torch

    from aliyun_gpushare_device_plugin_amd.device.health import HealthMonitor
    from aliyun_gpushare_device_plugin_amd.utils.metrics import PluginMetrics

    m = PluginMetrics()
    with S.SMI("auto") as smi:
        model = DeviceModel(smi.devices(), const.GIB, "nearest")
        card = f"/sys/bus/pci/devices/{smi.device(0).bdf}/mem_info_vram_used"
        mon = HealthMonitor(smi, model, 0.2, on_sample=lambda i, d: m.hbm_used.set(d.vram_used, gpu=str(i)))
        mon.start()
        try:
            held = torch.empty(8 << 30, dtype=torch.uint8, device="cuda:0")
            torch.cuda.synchronize()
            time.sleep(0.6)
            sysfs = int(open(card).read())
            got = m.hbm_used.value(gpu="0")
            assert sysfs >= 8 << 30 and got >= 8 << 30
            assert abs(got - sysfs) < (1 << 30), (got, sysfs)   # same counter, sampled ~0.2 s apart
            del held
        finally:
            mon.stop()


_GEM_CHILD = r'''
import ctypes, json, os, sys, time
minor, sizes = int(sys.argv[1]), [int(x) for x in sys.argv[2:]]
libc = ctypes.CDLL(None, use_errno=True)          # global lookup: the preloaded shim's ioctl
fd = os.open(f"/dev/dri/renderD{minor}", os.O_RDWR)
used_path = f"/sys/class/drm/renderD{minor}/device/mem_info_vram_used"
class Create(ctypes.Structure):
    _fields_ = [("bo_size", ctypes.c_uint64), ("alignment", ctypes.c_uint64), ("domains", ctypes.c_uint64),
                ("domain_flags", ctypes.c_uint64)]
class Close(ctypes.Structure):
    _fields_ = [("handle", ctypes.c_uint32), ("pad", ctypes.c_uint32)]
CREATE = (3 << 30) | (32 << 16) | (ord("d") << 8) | 0x40     # DRM_IOCTL_AMDGPU_GEM_CREATE
CLOSE = (1 << 30) | (8 << 16) | (ord("d") << 8) | 0x09       # DRM_IOCTL_GEM_CLOSE
libc.ioctl.argtypes = [ctypes.c_int, ctypes.c_ulong, ctypes.c_void_p]
stats = libc.gpushare_shim_stats
stats.argtypes = [ctypes.POINTER(ctypes.c_uint64)] * 4
def ledger():
    u, q, d, p = (ctypes.c_uint64() for _ in range(4))
    stats(ctypes.byref(u), ctypes.byref(q), ctypes.byref(d), ctypes.byref(p))
    return u.value, d.value
def dev():
    return int(open(used_path).read())
handles = []
for n in sizes:
    before, dev0 = ledger()[0], dev()
    a = Create(n, 4096, 0x4, 0)                               # AMDGPU_GEM_DOMAIN_VRAM
    r = libc.ioctl(fd, CREATE, ctypes.addressof(a))
    err = ctypes.get_errno() if r else 0
    time.sleep(0.05)
    after, denied = ledger()
    h = ctypes.cast(ctypes.pointer(a), ctypes.POINTER(ctypes.c_uint32))[0] if r == 0 else None
    if h is not None:
        handles.append(h)
    print(json.dumps({"size": n, "rc": r, "errno": err, "charge": after - before, "device_delta": dev() - dev0,
                      "denied": denied}), flush=True)
for h in handles:
    before = ledger()[0]
    c = Close(h, 0)
    libc.ioctl(fd, CLOSE, ctypes.addressof(c))
    print(json.dumps({"closed": h, "released": before - ledger()[0]}), flush=True)
os.close(fd)
'''


def test_shim_charges_render_node_gem_vram():
    """Round-2 review item 5: HBM allocated on the container's render node (amdgpu GEM_CREATE,
    VRAM domain; a raw ioctl through ctypes, no HIP) is charged to the container's quota: within
    quota the charge equals the device's VRAM delta, over quota it is refused with ENOMEM, and
    GEM_CLOSE releases it."""
    from aliyun_gpushare_device_plugin_amd.utils.native import lib_path

    with S.SMI("auto") as smi:
        minor = smi.device(0).render_minor
    env = dict(os.environ, LD_PRELOAD=preload(lib_path("hipshim")), GPUSHARE_QUOTA_BYTES=str(4 * GIB),
               GPUSHARE_SHIM_LOG="1")
    r = subprocess.run([sys.executable, "-c", _GEM_CHILD, str(minor), str(2 * GIB), str(3 * GIB), str(GIB)],
                       env=env, capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr[-2000:]
    rows = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    ok2, over, ok1 = rows[:3]
    assert ok2["rc"] == 0 and ok2["charge"] == 2 * GIB
    assert abs(ok2["device_delta"] - 2 * GIB) <= 64 * MIB, ok2         # the device saw the same 2 GiB
    assert over["rc"] != 0 and over["errno"] == 12 and over["denied"] >= 1 and over["charge"] == 0
    assert ok1["rc"] == 0 and ok1["charge"] == GIB
    assert [x["released"] for x in rows[3:]] == [2 * GIB, GIB]


_GEM_ESCAPES = r'''
import ctypes, json, os, sys, time
minor = int(sys.argv[1])
GIB = 1 << 30
libc = ctypes.CDLL(None, use_errno=True)
used_path = f"/sys/class/drm/renderD{minor}/device/mem_info_vram_used"
class Create(ctypes.Structure):
    _fields_ = [("bo_size", ctypes.c_uint64), ("alignment", ctypes.c_uint64), ("domains", ctypes.c_uint64),
                ("domain_flags", ctypes.c_uint64)]
class Close(ctypes.Structure):
    _fields_ = [("handle", ctypes.c_uint32), ("pad", ctypes.c_uint32)]
class Prime(ctypes.Structure):
    _fields_ = [("handle", ctypes.c_uint32), ("flags", ctypes.c_uint32), ("fd", ctypes.c_int32)]
CREATE = (3 << 30) | (32 << 16) | (ord("d") << 8) | 0x40
CLOSE = (1 << 30) | (8 << 16) | (ord("d") << 8) | 0x09
PRIME = (3 << 30) | (12 << 16) | (ord("d") << 8) | 0x2d
libc.ioctl.argtypes = [ctypes.c_int, ctypes.c_ulong, ctypes.c_void_p]
libc.close.argtypes = [ctypes.c_int]
stats = libc.gpushare_shim_stats
stats.argtypes = [ctypes.POINTER(ctypes.c_uint64)] * 4
def ledger():
    u, q, d, p = (ctypes.c_uint64() for _ in range(4))
    stats(ctypes.byref(u), ctypes.byref(q), ctypes.byref(d), ctypes.byref(p))
    return u.value
def dev():
    time.sleep(0.3)                       # amdgpu returns freed VRAM asynchronously
    return int(open(used_path).read())
def create(fd, n):
    a = Create(n, 4096, 0x4, 0)
    r = libc.ioctl(fd, CREATE, ctypes.addressof(a))
    return (ctypes.cast(ctypes.pointer(a), ctypes.POINTER(ctypes.c_uint32))[0] if r == 0 else None), \
        (ctypes.get_errno() if r else 0)
def out(**k):
    print(json.dumps(k), flush=True)
def fresh():
    return os.open(f"/dev/dri/renderD{minor}", os.O_RDWR)
# 1) dup + close: the DRM file lives on through the dup, so does the charge
base = dev()
a = fresh()
h, e = create(a, GIB)
b = os.dup(a)
libc.close(a)
out(case="dup", err=e, charge=ledger(), held=dev() - base)
libc.ioctl(b, CLOSE, ctypes.addressof(Close(h, 0)))
out(case="dup_gemclose", charge=ledger(), held=dev() - base)
# 2) PRIME export of a charged VRAM handle
h2, e2 = create(b, GIB)
pr = Prime(h2, 0, -1)
r = libc.ioctl(b, PRIME, ctypes.addressof(pr))
out(case="prime", rc=r, errno=ctypes.get_errno() if r else 0, charge=ledger())
libc.close(b)
out(case="closed", charge=ledger(), held=dev() - base)
# 3) a child inherits the render fd; the parent closes its copy
c = fresh()
h3, e3 = create(c, 2 * GIB)
rp, wp = os.pipe()
pid = os.fork()
if pid == 0:
    os.close(wp)
    os.read(rp, 1)
    os._exit(0)
os.close(rp)
libc.close(c)
out(case="inherited", charge=ledger(), held=dev() - base)
d = fresh()
h4, e4 = create(d, 3 * GIB)                  # quota 4 GiB: 2 (lingering, child alive) + 3 > 4
out(case="over_while_child", errno=e4)
os.close(wp)
os.waitpid(pid, 0)
h5, e5 = create(d, 3 * GIB)                  # the child is gone: its file's 2 GiB were freed
out(case="after_child", errno=e5, charge=ledger(), held=dev() - base)
libc.close(d)
out(case="end", charge=ledger(), held=dev() - base)
'''


def test_shim_gem_escapes_are_closed():
    """Round-3 review item 3 on the real render node: dup + close keeps the charge while the DRM
    file (and the device's VRAM) lives; a charged VRAM handle cannot be exported as a dma-buf;
    a parent closing an inherited fd leaves the charge until the child holding the file exits.
    Throughout, the ledger follows the device's own VRAM count."""
    from aliyun_gpushare_device_plugin_amd.utils.native import lib_path

    with S.SMI("auto") as smi:
        minor = smi.device(0).render_minor
    env = dict(os.environ, LD_PRELOAD=preload(lib_path("hipshim")), GPUSHARE_QUOTA_BYTES=str(4 * GIB),
               GPUSHARE_SHIM_LOG="1")
    r = subprocess.run([sys.executable, "-c", _GEM_ESCAPES, str(minor)], env=env, capture_output=True, text=True,
                       timeout=90)
    assert r.returncode == 0, r.stderr[-2000:]
    rows = {x["case"]: x for x in (json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{"))}
    tol = 128 * MIB
    assert rows["dup"]["err"] == 0 and rows["dup"]["charge"] == GIB
    assert abs(rows["dup"]["held"] - GIB) <= tol, rows           # the VRAM really is still allocated
    assert rows["dup_gemclose"]["charge"] == 0 and rows["dup_gemclose"]["held"] <= tol
    assert rows["prime"]["rc"] != 0 and rows["prime"]["errno"] == 13 and rows["prime"]["charge"] == GIB
    assert rows["closed"]["charge"] == 0 and rows["closed"]["held"] <= tol
    assert rows["inherited"]["charge"] == 2 * GIB and abs(rows["inherited"]["held"] - 2 * GIB) <= tol
    assert rows["over_while_child"]["errno"] == 12
    assert rows["after_child"]["errno"] == 0 and rows["after_child"]["charge"] == 3 * GIB
    assert abs(rows["after_child"]["held"] - 3 * GIB) <= tol
    assert rows["end"]["charge"] == 0 and rows["end"]["held"] <= tol


def test_quota_watchdog_catches_a_process_without_the_shim():
    """Round-2 review, isolation: a tenant process that drops the quota shim is still seen by
    the node-side watchdog (amdgpu DRM fdinfo, kernel-reported) and, in kill mode, ended."""
    import time

    from aliyun_gpushare_device_plugin_amd.quota.watchdog import QuotaWatchdog
    from aliyun_gpushare_device_plugin_amd.utils.metrics import PluginMetrics
    from tests.test_allocate_engine import StaticSource, mkpod

    code = ("import torch, sys, time\nx = torch.empty(6 << 30, dtype=torch.uint8, device='cuda')\n"
            "torch.cuda.synchronize()\nprint('held', flush=True)\ntime.sleep(60)\n")
    env = {k: v for k, v in os.environ.items() if k != "LD_PRELOAD"}
    child = subprocess.Popen([sys.executable, "-c", code], env=env, stdout=subprocess.PIPE, text=True)
    try:
        assert child.stdout.readline().strip() == "held"
        with S.SMI("auto") as smi:
            model = DeviceModel(smi.devices(), const.GIB, "nearest")
        pod = mkpod("tenant", 4, 0, 10, assigned="true", phase="Running", uid="uid-tenant")   # 4 GiB share
        m = PluginMetrics()
        wd = QuotaWatchdog(model, StaticSource([pod]), m, mode="report", slack_bytes=256 << 20,
                           pid_pod=lambda pid: "uid-tenant" if pid == child.pid else None)
        v = wd.scan()
        assert len(v) == 1 and v[0].gpu == 0, v
        assert 6 * GIB <= v[0].used <= 6 * GIB + 512 * MIB and v[0].allowed < 4.1 * GIB
        assert m.quota_violation.value(pod_uid="uid-tenant", gpu="0") > 1.5 * GIB
        wd.mode = "kill"
        v = wd.scan()
        assert v[0].killed == [child.pid]
        child.wait(timeout=20)
        assert child.returncode == -9
        time.sleep(0.5)
        assert wd.scan() == []
    finally:
        if child.poll() is None:
            child.kill()
            child.wait(timeout=20)


def test_dmem_limits_read_the_box_kernel_truthfully():
    """quota/dmem.py on the real cgroup v2 tree: it reports the dmem controller exactly when the
    kernel lists it, finds a VRAM region for every GPU when it does, and otherwise stays inactive
    (the test boxes' 6.18 kernel has no dmem controller: profiles/r3/dmem_probe.txt)."""
    from aliyun_gpushare_device_plugin_amd.quota.dmem import DmemLimits

    from .test_allocate_engine import StaticSource

    with S.SMI("auto") as smi:
        model = DeviceModel(smi.devices(), const.GIB, "nearest")
    try:
        with open("/sys/fs/cgroup/cgroup.controllers") as f:
            ctrl = "dmem" in f.read().split()
    except OSError:
        ctrl = False
    d = DmemLimits(model, StaticSource([]))
    assert d.controller_present() == ctrl
    if ctrl and d.regions():
        assert set(d.regions()) == {g.index for g in model.gpus}
    else:
        assert not d.available() and d.sync() == 0
