"""CPU tests of the quota shim against a stub HIP runtime (tests/native/fake_hip.c).

The stub has the same soname as ROCm's runtime (libamdhip64.so.7) and a 16 GiB "device" it
allocates from through emulated KFD ioctls, like ROCr does; the driver program is an ordinary
HIP client linked against it, run with the shim in LD_PRELOAD — exactly how a container
process sees it. The default mode charges at the KFD ioctl; GPUSHARE_SHIM_MODE=hip charges at
the HIP API. Real-hardware coverage of the same paths: tests/test_gpu_native.py (marked gpu).
"""
import json
import os
import subprocess
import sys
import uuid

import pytest
from aliyun_gpushare_device_plugin_amd.utils.native import preload

HERE = os.path.dirname(os.path.abspath(__file__))
GIB = 1 << 30
MIB = 1 << 20


@pytest.fixture(scope="module")
def stub(tmp_path_factory):
    d = tmp_path_factory.mktemp("fakehip")
    lib = d / "libamdhip64.so.7"
    subprocess.run(["gcc", "-shared", "-fPIC", "-O1", "-Wl,-soname,libamdhip64.so.7", "-o", str(lib),
                    os.path.join(HERE, "native", "fake_hip.c")], check=True)
    drv = d / "shim_driver"
    subprocess.run(["gcc", "-O1", "-pthread", "-o", str(drv), os.path.join(HERE, "native", "shim_driver.c"),
                    str(lib), f"-Wl,-rpath,{d}", "-ldl"], check=True)
    return d, drv


@pytest.fixture(scope="module")
def kfd_root(tmp_path_factory):
    """A KFD topology with one GPU (gpu_id 1) of 16 GiB, for quotas derived from units."""
    r = tmp_path_factory.mktemp("kfdroot")
    n = r / "sys/class/kfd/kfd/topology/nodes/1"
    (n / "mem_banks/0").mkdir(parents=True)
    (n / "gpu_id").write_text("1\n")
    (n / "mem_banks/0/properties").write_text(f"heap_type 1\nsize_in_bytes {16 * GIB}\n")
    return str(r)


def run(stub, shim, args, **env):
    d, drv = stub
    e = dict(os.environ)
    e.update({"LD_PRELOAD": shim, "LD_LIBRARY_PATH": str(d)})
    e.update({k: str(v) for k, v in env.items()})
    r = subprocess.run([str(drv), *map(str, args)], env=e, capture_output=True, text=True, timeout=30)
    return [json.loads(line) for line in r.stdout.splitlines() if line.startswith("{")], r


def ledger():
    return f"/gs-test-{uuid.uuid4().hex[:12]}"


def cleanup(name):
    try:
        os.unlink("/dev/shm" + name)
    except FileNotFoundError:
        pass


@pytest.mark.parametrize("mode", ["kfd", "hip"])
def test_quota_from_container_share(stub, native_shim, mode):
    # 4 of 16 units of a 16 GiB device -> 4 GiB quota
    out, _ = run(stub, native_shim, ["info", "alloc", 3 * GIB, "alloc", 2 * GIB, "info"],
                 ALIYUN_COM_GPU_MEM_CONTAINER=4, ALIYUN_COM_GPU_MEM_DEV=16, GPUSHARE_SHIM_MODE=mode)
    assert out[0]["total"] == 4 * GIB and out[0]["free"] == 4 * GIB
    assert out[1]["err"] == 0
    assert out[2]["err"] == 2                    # hipErrorOutOfMemory: 3 + 2 > 4
    assert out[3]["free"] == 1 * GIB and out[3]["total"] == 4 * GIB


def test_free_releases_charge(stub, native_shim):
    out, _ = run(stub, native_shim, ["alloc", 3 * GIB, "free", 0, "alloc", 3 * GIB, "info"],
                 GPUSHARE_QUOTA_BYTES=4 * GIB)
    assert [o["err"] for o in out[:3]] == [0, 0, 0]
    assert out[3]["free"] == 1 * GIB


def test_hip_mode_cdna4_granule_rounding(stub, native_shim):
    # HIP-API mode: 2 MiB allocation granule, a 1-byte hipMalloc costs 2 MiB, 2 MiB + 1 costs 4 MiB
    out, _ = run(stub, native_shim, ["mode", "alloc", 1, "info", "alloc", 2 * MIB + 1, "info"],
                 GPUSHARE_QUOTA_BYTES=64 * MIB, GPUSHARE_SHIM_MODE="hip")
    assert out[0]["mode"] == 1
    assert out[2]["free"] == 62 * MIB
    assert out[4]["free"] == 58 * MIB
    out, _ = run(stub, native_shim, ["alloc", 1, "info"], GPUSHARE_QUOTA_BYTES=64 * MIB,
                 GPUSHARE_ALLOC_GRANULE=4096, GPUSHARE_SHIM_MODE="hip")
    assert out[1]["free"] == 64 * MIB - 4096


@pytest.mark.parametrize("mode", ["kfd", "hip"])
def test_async_and_vmm_paths_are_charged(stub, native_shim, mode):
    out, _ = run(stub, native_shim, ["async", 3 * GIB, "async", 2 * GIB, "vmm", 2 * GIB, "vmm", GIB],
                 GPUSHARE_QUOTA_BYTES=4 * GIB, GPUSHARE_SHIM_MODE=mode)
    assert [o["err"] for o in out] == [0, 2, 2, 0]


def test_kfd_mode_is_default_and_charges_the_ioctl(stub, native_shim):
    out, _ = run(stub, native_shim, ["mode", "alloc", 1, "stats"], GPUSHARE_QUOTA_BYTES=64 * MIB)
    assert out[0]["mode"] == 0
    assert out[2]["used"] == 1          # the KFD allocation's size (the runtime rounds, not the shim)


def test_pool_retention_is_charged_until_trim(stub, native_shim):
    """hipMallocAsync pools keep freed blocks: HIP-level accounting forgot them at hipFreeAsync
    (round-1 review); at the KFD boundary they stay charged until the pool trims."""
    args = ["async", 3 * GIB, "freeasync", 0, "stats", "alloc", 2 * GIB, "trim", "stats", "alloc", 2 * GIB]
    out, _ = run(stub, native_shim, args, GPUSHARE_QUOTA_BYTES=4 * GIB)
    assert out[2]["used"] == 3 * GIB          # freed to the pool, still resident
    assert out[3]["err"] == 2                 # so 2 GiB more does not fit
    assert out[5]["used"] == 0 and out[6]["err"] == 0
    # the HIP-level mode under-counts exactly this case
    out, _ = run(stub, native_shim, args, GPUSHARE_QUOTA_BYTES=4 * GIB, GPUSHARE_SHIM_MODE="hip")
    assert out[2]["used"] == 0 and out[3]["err"] == 0


def test_runtime_internal_allocations_are_charged(stub, native_shim):
    """Scratch / code objects / staging: VRAM the runtime takes with no HIP allocation call."""
    out, _ = run(stub, native_shim, ["scratch", 3 * GIB, "alloc", 2 * GIB, "scratch", 2 * GIB, "stats"],
                 GPUSHARE_QUOTA_BYTES=4 * GIB)
    assert [o["err"] for o in out[:3]] == [0, 2, 2]
    assert out[3]["used"] == 3 * GIB and out[3]["denied"] == 2


def test_quota_from_units_and_kfd_topology(stub, native_shim, kfd_root):
    # no GPUSHARE_QUOTA_BYTES: 4 of 16 units of the GPU KFD reports (16 GiB) -> 4 GiB, resolved
    # at the first allocation (inside the runtime, before any hipMemGetInfo)
    out, _ = run(stub, native_shim, ["alloc", 3 * GIB, "alloc", 2 * GIB, "info"],
                 ALIYUN_COM_GPU_MEM_CONTAINER=4, ALIYUN_COM_GPU_MEM_DEV=16, GPUSHARE_KFD_SYSFS=kfd_root)
    assert [o["err"] for o in out[:2]] == [0, 2]
    assert out[2]["total"] == 4 * GIB and out[2]["free"] == 1 * GIB


def test_forked_child_starts_with_empty_table(stub, native_shim):
    """Round-1 review: the child inherited the parent's pointer map, so freeing an inherited
    pointer uncharged the child's slot (underflow) and the shared total."""
    name = ledger()
    try:
        out, r = run(stub, native_shim, ["alloc", GIB, "fork", 2 * GIB, "stats"], GPUSHARE_LEDGER=name,
                     GPUSHARE_QUOTA_BYTES=4 * GIB)
        child = next(o for o in out if o["op"] == "child")
        assert child["err"] == 0 and child["used"] == 3 * GIB            # parent's 1 + child's 2 (shared ledger)
        assert child["used_after_parent_frees"] == 3 * GIB             # inherited pointers: not the child's to uncharge
        st = [o for o in out if o["op"] == "stats"][-1]
        assert st["used"] == GIB                                         # child exited: its slot returned
    finally:
        cleanup(name)


def test_shim_links_no_cxx_runtime_and_old_glibc(native_shim):
    """Round-1 review: the shim is preloaded into arbitrary tenant images — no libstdc++ /
    libgcc_s dependency, and glibc symbol versions no newer than 2.17 (CentOS 7 baseline)."""
    dyn = subprocess.run(["readelf", "-d", native_shim], capture_output=True, text=True, check=True).stdout
    needed = {ln.split("[")[1].rstrip("]") for ln in dyn.splitlines() if "(NEEDED)" in ln}
    assert not {n for n in needed if n.startswith(("libstdc++", "libgcc_s"))}, needed
    syms = subprocess.run(["objdump", "-T", native_shim], capture_output=True, text=True, check=True).stdout
    import re
    vers = {tuple(int(x) for x in v.split(".")) for v in re.findall(r"GLIBC_([0-9.]+)\)", syms)}
    assert max(vers) <= (2, 17), sorted(vers)[-3:]
    assert "GLIBCXX" not in syms and "CXXABI" not in syms


def test_cgpu_disable_passes_through(stub, native_shim):
    out, _ = run(stub, native_shim, ["alloc", 10 * GIB, "info"], ALIYUN_COM_GPU_MEM_CONTAINER=1,
                 ALIYUN_COM_GPU_MEM_DEV=16, CGPU_DISABLE="true")
    assert out[0]["err"] == 0 and out[1]["total"] == 16 * GIB


def test_no_quota_env_passes_through(stub, native_shim):
    out, _ = run(stub, native_shim, ["alloc", 10 * GIB, "info"])
    assert out[0]["err"] == 0 and out[1]["total"] == 16 * GIB


def test_shared_ledger_across_processes(stub, native_shim):
    name = ledger()
    try:
        d, drv = stub
        env = dict(os.environ, LD_PRELOAD=preload(native_shim), LD_LIBRARY_PATH=str(d), GPUSHARE_LEDGER=name,
                   GPUSHARE_QUOTA_BYTES=str(4 * GIB))
        holder = subprocess.Popen([str(drv), "alloc", str(3 * GIB), "sleep", "3"], env=env,
                                  stdout=subprocess.PIPE, text=True)
        first = holder.stdout.readline()
        assert json.loads(first)["err"] == 0
        out, _ = run(stub, native_shim, ["alloc", 2 * GIB, "alloc", GIB, "info"], GPUSHARE_LEDGER=name,
                     GPUSHARE_QUOTA_BYTES=4 * GIB)
        assert out[0]["err"] == 2        # the other process holds 3 of 4 GiB
        assert out[1]["err"] == 0
        holder.wait(timeout=10)
        # holder exited cleanly: its charge was returned at exit
        out, _ = run(stub, native_shim, ["alloc", 3 * GIB], GPUSHARE_LEDGER=name, GPUSHARE_QUOTA_BYTES=4 * GIB)
        assert out[0]["err"] == 0
    finally:
        cleanup(name)


def test_crashed_process_charge_is_reclaimed(stub, native_shim):
    name = ledger()
    try:
        out, r = run(stub, native_shim, ["alloc", 3 * GIB, "crash"], GPUSHARE_LEDGER=name,
                     GPUSHARE_QUOTA_BYTES=4 * GIB)
        assert out[0]["err"] == 0 and r.returncode == 3   # _exit: no atexit cleanup ran
        out, _ = run(stub, native_shim, ["alloc", 3 * GIB], GPUSHARE_LEDGER=name, GPUSHARE_QUOTA_BYTES=4 * GIB)
        assert out[0]["err"] == 0                           # dead pid's 3 GiB reclaimed
    finally:
        cleanup(name)


def test_concurrent_threads_never_exceed_quota(stub, native_shim):
    """16 threads contend for a 64 MiB quota with 8 MiB allocations: the ledger's peak never
    exceeds the quota, every grant is returned, and denials are counted."""
    name = ledger()
    try:
        out, r = run(stub, native_shim, ["threads", 16, 400, 8 * MIB, "stats", "info"], GPUSHARE_LEDGER=name,
                     GPUSHARE_QUOTA_BYTES=64 * MIB)
        th, st, info = out
        assert th["ok"] + th["denied"] == 16 * 400 and th["ok"] > 0
        assert st["enabled"] == 1 and st["quota"] == 64 * MIB
        assert st["peak"] <= 64 * MIB and st["used"] == 0 and st["denied"] == th["denied"]
        assert info["free"] == 64 * MIB
    finally:
        cleanup(name)


@pytest.mark.parametrize("san", ["asan", "tsan"])
def test_shim_under_sanitizers(stub, tmp_path, san):
    """The shim built with -fsanitize=address,undefined / -fsanitize=thread (host code; GPU
    sanitizers are not available), run through the multi-process and multi-thread paths."""
    import sys
    sys.path.insert(0, os.path.join(HERE, "..", "native"))
    import build as nb
    lib = nb.build_hipshim(asan=san)[0]
    rt = subprocess.run(["gcc", f"-print-file-name=lib{san}.so"], capture_output=True, text=True).stdout.strip()
    if not os.path.exists(rt):
        pytest.skip(f"lib{san}.so not installed")
    d, drv = stub
    name = ledger()
    env = {"LD_PRELOAD": f"{rt}:{lib}", "LD_LIBRARY_PATH": str(d), "GPUSHARE_LEDGER": name,
           "GPUSHARE_QUOTA_BYTES": str(64 * MIB), "ASAN_OPTIONS": "detect_leaks=0:halt_on_error=1",
           "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1", "TSAN_OPTIONS": "halt_on_error=1:report_bugs=1"}
    try:
        e = dict(os.environ, **env)
        r = subprocess.run([str(drv), "threads", "8", "200", str(8 * MIB), "alloc", str(GIB), "alloc", str(MIB),
                            "free", "0", "gem", str(8 * MIB), "4", "gem", str(8 * MIB), "4", "gemclose", "1",
                            "closefd", "stats"], env=e, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-3000:]
        assert "ERROR: AddressSanitizer" not in r.stderr and "WARNING: ThreadSanitizer" not in r.stderr, r.stderr[-3000:]
        assert "runtime error" not in r.stderr, r.stderr[-3000:]
        out = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
        assert out[1]["err"] == 2 and out[2]["err"] == 0 and out[-1]["used"] == 0
        assert [o["err"] for o in out if o["op"] in ("gem", "gemclose", "closefd")] == [0, 0, 0, 0]
    finally:
        cleanup(name)


def test_file_backed_ledger_is_readable_by_the_plugin(stub, native_shim, tmp_path):
    """GPUSHARE_LEDGER_DIR: the ledger is a file the node agent reads (used / peak / denials)."""
    from aliyun_gpushare_device_plugin_amd.quota import ledger as L, ledger_name
    from aliyun_gpushare_device_plugin_amd.utils.metrics import PluginMetrics
    uid = "0b6f1c2e-aaaa-bbbb-cccc-0123456789ab"
    name = ledger_name(uid, 0)
    d, drv = stub
    env = dict(os.environ, LD_PRELOAD=preload(native_shim), LD_LIBRARY_PATH=str(d), GPUSHARE_LEDGER=name,
               GPUSHARE_LEDGER_DIR=str(tmp_path), GPUSHARE_QUOTA_BYTES=str(4 * GIB))
    holder = subprocess.Popen([str(drv), "alloc", str(3 * GIB), "alloc", str(2 * GIB), "sleep", "3"], env=env,
                              stdout=subprocess.PIPE, text=True)
    try:
        assert json.loads(holder.stdout.readline())["err"] == 0
        assert json.loads(holder.stdout.readline())["err"] == 2          # denied: 3 + 2 > 4 GiB
        st = L.read(str(tmp_path / (name.lstrip("/") + L.SUFFIX)))
        assert st is not None and st.pod_uid_key == L.uid_key(uid) and st.container_slot == 0
        assert (st.used, st.quota, st.peak, st.denied, st.processes) == (3 * GIB, 4 * GIB, 3 * GIB, 1, 1)
        m = PluginMetrics()
        L.collect(str(tmp_path), m, live_uids={uid})
        text = m.registry.render()
        assert f'gpushare_container_hbm_used_bytes{{container="0",pod_uid="{L.uid_key(uid)}"}} {float(3 * GIB)}' in text
        assert "gpushare_container_quota_denials" in text
    finally:
        holder.wait(timeout=10)
    # process gone and pod gone -> the collector removes the ledger
    L.collect(str(tmp_path), PluginMetrics(), live_uids=set())
    assert not list(tmp_path.glob("*.ledger"))


def test_per_container_ledger_dirs_and_gc_after_sigkill(stub, native_shim, tmp_path):
    """Round-2 review item 2: each container's shim writes into its own ledger directory (the
    only one mounted into it), and a SIGKILLed container's ledger — still showing its bytes as
    used — is removed once its pod is gone, not exported forever."""
    import signal
    import time

    from aliyun_gpushare_device_plugin_amd.quota import ledger as L, ledger_name
    from aliyun_gpushare_device_plugin_amd.utils.metrics import PluginMetrics
    root = tmp_path / "ledgers"
    ld = L.LedgerDir(str(root))
    ld.prepare()
    d, drv = stub
    procs, keys = [], {}
    for uid in ("uid-a", "uid-b"):
        lkey = ld.new_key(uid, 0)
        keys[uid] = lkey
        env = dict(os.environ, LD_PRELOAD=preload(native_shim), LD_LIBRARY_PATH=str(d), GPUSHARE_LEDGER=ledger_name(uid, 0),
                   GPUSHARE_LEDGER_DIR=ld.create(lkey, uid), GPUSHARE_QUOTA_BYTES=str(4 * GIB))
        procs.append(subprocess.Popen([str(drv), "alloc", str(1 * GIB), "sleep", "30"], env=env,
                                      stdout=subprocess.PIPE, text=True))
    try:
        for p in procs:
            assert json.loads(p.stdout.readline())["err"] == 0
        # each directory holds exactly its own container's ledger
        for uid, lkey in keys.items():
            assert [n for n in os.listdir(root / lkey)] == [ledger_name(uid, 0).lstrip("/") + L.SUFFIX]
        m = PluginMetrics()
        got = {st.lkey: st for st in L.collect(str(root), m, live_uids={"uid-a", "uid-b"})}
        assert got[keys["uid-a"]].used == got[keys["uid-b"]].used == 1 * GIB
        procs[0].send_signal(signal.SIGKILL)         # OOM-kill: the slot is never released
        procs[0].wait(timeout=10)
        st = L.read(str(root / keys["uid-a"] / (ledger_name("uid-a", 0).lstrip("/") + L.SUFFIX)))
        assert st.used == 1 * GIB
        # pod a deleted: its directory goes (after the grace period), b's stays
        left = {s.lkey for s in L.collect(str(root), m, live_uids={"uid-b"}, grace_s=0.0)}
        assert left == {keys["uid-b"]} and not (root / keys["uid-a"]).exists()
        assert 'pod_uid="uida"' not in m.registry.render()
        # placement truth: b's ledger is also owned by c (the pod really running it); b gone, c alive
        ld.add_owner(keys["uid-b"], "uid-c")
        time.sleep(0.01)
        left = {s.lkey for s in L.collect(str(root), m, live_uids={"uid-c"}, grace_s=0.0)}
        assert left == {keys["uid-b"]} and 'pod_uid="uidc"' in m.registry.render()
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
            p.wait(timeout=10)


def test_render_node_gem_vram_is_charged(stub, native_shim):
    """Round-2 review item 5: VRAM allocated on the container's render node
    (DRM_IOCTL_AMDGPU_GEM_CREATE, VRAM domain) is charged like KFD allocations: over quota it
    is refused with ENOMEM, GEM_CLOSE releases it, closing the render fd releases the rest;
    GTT-only buffer objects are not charged."""
    vram, gtt = 4, 2
    out, r = run(stub, native_shim, ["alloc", 1 * GIB, "gem", 2 * GIB, vram, "stats", "gem", 2 * GIB, vram,
                                     "gem", 8 * GIB, gtt, "stats", "gemclose", 1, "stats", "gem", 1 * GIB, vram,
                                     "closefd", "stats"],
                 GPUSHARE_QUOTA_BYTES=4 * GIB)
    assert out[0]["err"] == 0
    assert out[1]["err"] == 0 and out[2]["used"] == 3 * GIB
    assert out[3]["err"] == 12                               # ENOMEM: 3 + 2 > 4 GiB
    assert out[4]["err"] == 0 and out[5]["used"] == 3 * GIB  # GTT: not HBM, not charged
    assert out[6]["err"] == 0 and out[7]["used"] == 1 * GIB  # GEM_CLOSE of the 2 GiB VRAM object
    assert out[8]["err"] == 0 and out[9]["err"] == 0
    assert out[10]["used"] == 1 * GIB                        # fd closed: its GEM objects are gone


def test_hip_mode_runtime_init_under_shim_init_does_not_deadlock(stub, native_shim):
    """ADVICE (round 2): in hip mode without GPUSHARE_QUOTA_BYTES the shim's init calls the real
    hipMemGetInfo; if that starts the runtime, which allocates VRAM through the (interposed)
    KFD ioctl on the same thread, the ioctl must not wait on the shim's own once-control."""
    out, r = run(stub, native_shim, ["alloc", 1 * GIB, "info"], ALIYUN_COM_GPU_MEM_CONTAINER=4,
                 ALIYUN_COM_GPU_MEM_DEV=16, GPUSHARE_SHIM_MODE="hip", FAKE_HIP_INIT_KFD=1)
    assert r.returncode == 0, r.stderr
    assert out[0]["err"] == 0 and out[1]["total"] == 4 * GIB


def test_kfd_mode_allocation_during_shim_init_passes(stub, native_shim):
    out, r = run(stub, native_shim, ["info", "alloc", 1 * GIB, "stats"], GPUSHARE_QUOTA_BYTES=4 * GIB,
                 FAKE_HIP_INIT_KFD=1)
    assert r.returncode == 0 and out[1]["err"] == 0 and out[2]["used"] >= 1 * GIB


@pytest.mark.parametrize("backing", ["file", "shm"])
def test_ledger_survives_runtime_map_fixed_during_shim_init(stub, native_shim, tmp_path, backing):
    """Measured on MI355X (bench pod processes): the shim initialised inside ROCr's first VRAM
    ioctl, mapped its ledger into the range ROCr had just probed and unmapped, and ROCr then
    mapped that range MAP_FIXED and trimmed it — the ledger page vanished and the next charge
    faulted. The shim reserves the ledger's address range when it is loaded, before any runtime
    runs, and maps the ledger onto that reservation."""
    name = ledger()
    env = dict(GPUSHARE_LEDGER=name, GPUSHARE_QUOTA_BYTES=4 * GIB, FAKE_HIP_PROBE_FIXED=1, GPUSHARE_SHIM_DIAG=1)
    if backing == "file":
        env["GPUSHARE_LEDGER_DIR"] = str(tmp_path)
    try:
        out, r = run(stub, native_shim, ["scratch", 1 * GIB, "alloc", 2 * GIB, "alloc", 2 * GIB, "stats"], **env)
    finally:
        cleanup(name)
    assert r.returncode == 0, r.stderr
    assert [o["err"] for o in out[:3]] == [0, 0, 2]
    assert out[3]["used"] == 3 * GIB and out[3]["denied"] == 1


def _proc(tmp_path):
    root = tmp_path / "proc"
    root.mkdir(parents=True)
    return str(root)


def test_gem_charge_survives_dup_and_close(stub, native_shim, tmp_path):
    """Round-3 review item 3: GEM handles belong to the DRM file, not the fd number. dup(fd) +
    close(fd) leaves the file (and its VRAM) alive through the dup, so the charge stays; it is
    released when the last fd closes, and GEM_CLOSE through the dup releases a handle."""
    vram = 4
    out, r = run(stub, native_shim, ["drmfile", 71, "gem", GIB, vram, "gem", GIB, vram, "dup", "closefd", "stats",
                                     "swapdup", "gemclose", 2, "stats", "closefd", "stats"],
                 GPUSHARE_QUOTA_BYTES=4 * GIB, GPUSHARE_SHIM_PROC_ROOT=_proc(tmp_path))
    assert r.returncode == 0, r.stderr
    ops = {o["op"]: o for o in out}
    st = [o for o in out if o["op"] == "stats"]
    assert out[1]["err"] == out[2]["err"] == 0 and ops["closefd"]["err"] == 0
    assert st[0]["used"] == 2 * GIB              # the original fd closed, the dup holds the file
    assert st[1]["used"] == GIB                  # GEM_CLOSE through the dup: same DRM file
    assert st[2]["used"] == 0                    # the last fd closed: the file and its BOs are gone


def test_gem_charge_survives_a_parent_closing_an_inherited_fd(stub, native_shim, tmp_path):
    """A child inherits the render fd; the parent closing its copy does not free the file, so
    the charge lingers; once the child is gone it is released at the next re-check (before a
    denial, or when another fd of the file closes)."""
    vram = 4
    out, r = run(stub, native_shim, ["drmfile", 72, "gem", 2 * GIB, vram, "forkhold", "closefd", "stats",
                                     "drmfile", 73, "gem", 3 * GIB, vram, "killhold", "gem", 3 * GIB, vram, "stats"],
                 GPUSHARE_QUOTA_BYTES=4 * GIB, GPUSHARE_SHIM_PROC_ROOT=_proc(tmp_path))
    assert r.returncode == 0, r.stderr
    gems = [o for o in out if o["op"] == "gem"]
    st = [o for o in out if o["op"] == "stats"]
    assert gems[0]["err"] == 0
    assert st[0]["used"] == 2 * GIB              # the child still holds the DRM file
    assert gems[1]["err"] == 12                  # 2 + 3 > 4 GiB: the lingering file is still alive
    assert gems[2]["err"] == 0                   # child gone: re-checked before denying, released
    assert st[1]["used"] == 3 * GIB


def test_prime_export_of_charged_vram_is_refused(stub, native_shim, tmp_path):
    """A dma-buf export would keep the BO alive after GEM_CLOSE: refused for charged VRAM
    handles (EACCES); GTT handles export normally; GPUSHARE_SHIM_PRIME=keep exports and keeps the
    charge until the DRM file is gone."""
    vram, gtt = 4, 2
    args = ["drmfile", 74, "gem", GIB, vram, "gem", GIB, gtt, "prime", 1, "prime", 2, "gemclose", 1, "stats",
            "closefd", "stats"]
    out, r = run(stub, native_shim, args, GPUSHARE_QUOTA_BYTES=4 * GIB, GPUSHARE_SHIM_PROC_ROOT=_proc(tmp_path))
    assert r.returncode == 0, r.stderr
    pr = [o for o in out if o["op"] == "prime"]
    st = [o for o in out if o["op"] == "stats"]
    assert pr[0]["err"] == 13 and pr[1]["err"] == 0      # EACCES for VRAM; GTT is not HBM
    assert st[0]["used"] == 0                            # not exported: GEM_CLOSE released it
    out, r = run(stub, native_shim, args, GPUSHARE_QUOTA_BYTES=4 * GIB, GPUSHARE_SHIM_PRIME="keep",
                 GPUSHARE_SHIM_PROC_ROOT=_proc(tmp_path / "k"))
    pr = [o for o in out if o["op"] == "prime"]
    st = [o for o in out if o["op"] == "stats"]
    assert pr[0]["err"] == 0 and st[0]["used"] == GIB  # exported: GEM_CLOSE keeps the charge
    assert st[1]["used"] == 0                            # the DRM file closed: released


class FakeBroker:
    """The HBM broker's pod side (native/hbmbroker): answers one TAKE with ``granules`` fds, then
    records when the pod's connection ends (its granules would be scrubbed and lent again).
    ``stream``: [(delay_s, k), ...] answers a streaming TAKE with ``granules - sum(k)`` at once
    ("FDS <k0> <gran> <total> <limit>") and each k after its delay ("MORE <k> <gran>"); with
    ``hangup`` it closes the connection at the first delay instead (a broker that went away).
    After that it answers EXTEND with up to ``extra`` granules beyond the grant (``limit``: the
    pod's whole quota in granules, sent in the streaming header) and AVAIL with what is left."""

    def __init__(self, path, granules=4, gran=GIB, refuse=False, stream=None, hangup=False, extra=0, limit=None):
        import socket
        import threading

        self.granules, self.gran, self.refuse, self.stream, self.hangup = granules, gran, refuse, stream, hangup
        self.extra, self.limit = extra, limit if limit is not None else granules + extra
        self.requests = []
        self.took = None
        self.closed_at = None
        self.ls = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self.ls.bind(path)
        self.ls.listen(1)
        threading.Thread(target=self._serve, daemon=True).start()

    def _serve(self):
        import socket
        import time

        conn, _ = self.ls.accept()
        buf = b""
        while not buf.endswith(b"\n"):
            buf += conn.recv(1)
        self.took = buf.decode().strip()
        if self.refuse:
            conn.sendall(b"ERR timeout\n")
            conn.close()
            return
        def send(head, k):
            fds = [os.open("/dev/null", os.O_RDONLY) for _ in range(k)]
            conn.sendall(head.encode())
            if fds:
                socket.send_fds(conn, [b"f"], fds)
            for fd in fds:
                os.close(fd)

        if self.stream is not None:
            later = sum(k for _, k in self.stream)
            send(f"FDS {self.granules - later} {self.gran} {self.granules} {self.limit}\n", self.granules - later)
            for delay, k in self.stream:
                time.sleep(delay)
                if self.hangup:
                    conn.close()
                    self.closed_at = time.monotonic()
                    return
                try:
                    send(f"MORE {k} {self.gran}\n", k)
                except OSError:           # the pod already handed its arena back
                    break
        else:
            send(f"FDS {self.granules} {self.gran}\n", self.granules)
        buf = b""
        while True:
            try:
                c = conn.recv(1)
            except OSError:
                break
            if not c:
                break
            buf += c
            if not buf.endswith(b"\n"):
                continue
            line, buf = buf.decode().strip(), b""
            self.requests.append(line)
            if line.startswith("EXTEND "):
                j = min(int(line.split()[1]), self.extra)
                self.extra -= j
                send(f"XFDS {j} {self.gran}\n", j)
            elif line == "AVAIL":
                conn.sendall(f"AVAIL {self.extra}\n".encode())
        self.closed_at = time.monotonic()
        conn.close()


def test_broker_arena_serves_hipmalloc_from_the_granted_granules(stub, native_shim, tmp_path):
    """The pod's hipMalloc/hipFree come from its granted granules (first fit, coalescing), the
    pod sees the arena's rest as free, the arena counts against its quota, and the arena is
    handed back only once nothing in it is live; allocations after that go to the driver."""
    import time

    sock = str(tmp_path / "hbm.sock")
    b = FakeBroker(sock, granules=4)
    name = ledger()
    try:
        t0 = time.monotonic()
        out, r = run(stub, native_shim, ["alloc", 3 * GIB, "alloc", 512 * MIB, "arena", "free", 0, "alloc", 2 * GIB,
                                         "alloc", GIB, "alloc", GIB, "info", "stats", "arenarelease", "freeall",
                                         "arenarelease", "arena", "sleepms", 600, "alloc", MIB, "stats"],
                     GPUSHARE_QUOTA_BYTES=8 * GIB, GPUSHARE_LEDGER=name, GPUSHARE_HBM_BROKER=sock,
                     GPUSHARE_HBM_TOKEN="tok123")
        t_end = time.monotonic()
        assert r.returncode == 0, r.stderr
        assert b.took == "TAKE tok123 STREAM"               # streaming is the default; this broker answers whole
        a3, b512, arena, _, c2, d1, e1, info, st, rel_live, _, rel, arena_after, late, st_after = out
        assert a3["err"] == 0 and b512["err"] == 0
        assert arena == {"op": "arena", "on": 1, "size": 4 * GIB, "used": 3 * GIB + 512 * MIB}
        assert c2["err"] == 0 and c2["p"] == a3["p"]             # first fit reuses the freed range
        assert d1["err"] == 0 and d1["p"] == a3["p"] + 2 * GIB   # coalesced rest of it
        # the 4 GiB arena is full and the broker lends nothing beyond the grant: the driver's, charged
        assert e1["err"] == 0 and not a3["p"] <= e1["p"] < a3["p"] + 8 * GIB
        assert b.requests == []                                  # a whole-grant answer has no limit beyond it
        # what the pod can obtain: the arena's rest + the quota's rest (the stub's driver has room)
        assert info["total"] == 8 * GIB and info["free"] == 512 * MIB + 3 * GIB
        assert st["used"] == 5 * GIB                             # the arena (4) + the driver's 1
        assert rel_live["r"] == -1 and rel["r"] == 1             # released only once nothing is live
        assert arena_after["on"] == 0
        assert b.closed_at is not None and b.closed_at < t_end - 0.4   # handed back before exit
        assert late["err"] == 0 and MIB <= st_after["used"] < GIB   # arena uncharged; the driver, charged
    finally:
        cleanup(name)


def test_streaming_take_maps_the_first_granules_and_waits_for_the_rest(stub, native_shim, tmp_path):
    """A streaming TAKE (the default): the broker answers at once with the 1 granule of 4 it has
    free; the pod's runtime is up without waiting for the other 3. A 512 MiB allocation is served
    from it; a 2 GiB one waits for the MORE batches (0.3 s, then 0.2 s) and lands contiguously
    in the first granule's rest and the new ones; hipMemGetInfo reports the whole grant; the ledger holds the grant
    from the start."""
    import time

    sock = str(tmp_path / "hbm.sock")
    b = FakeBroker(sock, granules=4, stream=[(0.3, 1), (0.2, 2)])
    name = ledger()
    try:
        t0 = time.monotonic()
        out, r = run(stub, native_shim, ["alloc", 512 * MIB, "arena", "arenastream", "info", "stats", "alloc", 2 * GIB,
                                         "arenastream", "alloc", 2 * GIB, "arena", "arenastream"],
                     GPUSHARE_QUOTA_BYTES=8 * GIB, GPUSHARE_LEDGER=name, GPUSHARE_HBM_BROKER=sock,
                     GPUSHARE_HBM_TOKEN="tok")
        assert r.returncode == 0, r.stderr
        assert b.took == "TAKE tok STREAM"
        small, arena, s0, info, st, big, s1, last, arena2, s2 = out
        assert small["err"] == 0 and arena == {"op": "arena", "on": 1, "size": 4 * GIB, "used": 512 * MIB}
        assert s0["mapped"] == 1 and s0["granted"] == 4 and s0["waits"] == 0
        assert info["free"] == 4 * GIB - 512 * MIB + 4 * GIB                # the grant's rest + the quota's rest
        assert st["used"] == 4 * GIB                                         # the whole grant is charged
        assert big["err"] == 0 and big["p"] == small["p"] + 512 * MIB       # the granules join the first one's rest
        assert s1["mapped"] == 4 and s1["msgs"] == 2 and s1["waits"] >= 1 and s1["wait_ms"] >= 400
        assert last["err"] == 0 and not small["p"] <= last["p"] < small["p"] + 8 * GIB   # 1.5 GiB left: the driver
        assert arena2["used"] == 2 * GIB + 512 * MIB and s2["mapped"] == 4
        assert time.monotonic() - t0 < 10
    finally:
        cleanup(name)


def test_plain_take_and_a_stream_that_ends_early(stub, native_shim, tmp_path):
    """GPUSHARE_HBM_STREAM=0 asks for the whole grant in one answer. A stream whose broker goes
    away before the rest comes shrinks the grant to what was delivered, and the ledger with it."""
    sock = str(tmp_path / "hbm.sock")
    b = FakeBroker(sock, granules=2)
    name = ledger()
    try:
        out, r = run(stub, native_shim, ["alloc", GIB, "arena"], GPUSHARE_QUOTA_BYTES=4 * GIB, GPUSHARE_LEDGER=name,
                     GPUSHARE_HBM_BROKER=sock, GPUSHARE_HBM_TOKEN="plain", GPUSHARE_HBM_STREAM="0")
        assert r.returncode == 0, r.stderr
        assert b.took == "TAKE plain" and out[1]["size"] == 2 * GIB
    finally:
        cleanup(name)
    sock2 = str(tmp_path / "hbm2.sock")
    FakeBroker(sock2, granules=4, stream=[(0.1, 3)], hangup=True)    # 1 granule, then gone
    name = ledger()
    try:
        out, r = run(stub, native_shim, ["alloc", 512 * MIB, "alloc", 2 * GIB, "arena", "stats", "arenastream"],
                     GPUSHARE_QUOTA_BYTES=8 * GIB, GPUSHARE_LEDGER=name, GPUSHARE_HBM_BROKER=sock2,
                     GPUSHARE_HBM_TOKEN="short", GPUSHARE_HBM_MORE_WAIT_S="5")
        assert r.returncode == 0, r.stderr
        small, big, arena, st, s = out
        assert small["err"] == 0 and big["err"] == 0                 # the rest never came: the driver's
        assert arena["size"] == GIB and st["used"] == 3 * GIB        # grant and ledger shrank to 1 granule
        assert s["granted"] == s["mapped"] == 1
    finally:
        cleanup(name)


@pytest.mark.parametrize("version,free_kept,left", [(70051831, "1", 0), (70051831, "0", 3), (70253211, "1", 0)])
def test_arena_release_frees_the_kfd_imports_hip70_keeps(stub, native_shim, tmp_path, version, free_kept, left):
    """HIP 7.0 (PyTorch's runtime) never frees the KFD import of a released handle, so a broker
    granule stays referenced until the pod's process is torn down and the next pod waits for that
    (measured on MI355X: profiles/r5/dmabuf_refs/); the stub runtime does the same below 7.1. At
    gpushare_shim_arena_release() the shim frees the KFD imports the runtime kept (noted when it
    made them, during the arena's own imports). GPUSHARE_HBM_FREE_KEPT=0 leaves the runtime's
    behaviour; HIP 7.2 frees them itself. The broker side is on MI355X:
    tests/test_hbm_broker.py::test_a_released_arena_comes_back_while_the_tenant_lives."""
    sock = str(tmp_path / "hbm.sock")
    FakeBroker(sock, granules=3)
    name = ledger()
    try:
        out, r = run(stub, native_shim, ["alloc", GIB, "imports", "freeall", "arenarelease", "imports"],
                     GPUSHARE_QUOTA_BYTES=4 * GIB, GPUSHARE_LEDGER=name, GPUSHARE_HBM_BROKER=sock, GPUSHARE_HBM_TOKEN="t",
                     FAKE_HIP_VERSION=version, GPUSHARE_HBM_FREE_KEPT=free_kept, GPUSHARE_SHIM_LOG="1")
        assert r.returncode == 0, r.stderr
        a, live, _, rel, after = out
        assert a["err"] == 0 and live["live"] == 3 and rel["r"] == 1
        assert after["live"] == left, r.stderr
        if version < 70100000 and free_kept == "1":
            assert "freed 3 KFD imports the runtime kept" in r.stderr
    finally:
        cleanup(name)


@pytest.mark.parametrize("reserve", [True, False])
def test_the_fd_table_is_grown_at_load(native_shim, reserve):
    """The shim grows the process's fd table when it loads (still single-threaded), so receiving
    a broker arena's granule fds later never grows it in a multi-threaded pod, where each growth
    waits for an RCU grace period (115-210 ms measured on MI355X for 60-120 fds)."""
    import resource

    soft, _ = resource.getrlimit(resource.RLIMIT_NOFILE)
    env = dict(os.environ, LD_PRELOAD=preload(native_shim), GPUSHARE_SHIM_FD_RESERVE="1" if reserve else "0")
    out = subprocess.run(["cat", "/proc/self/status"], env=env, capture_output=True, text=True, check=True).stdout
    size = int(next(ln.split()[1] for ln in out.splitlines() if ln.startswith("FDSize:")))
    if reserve and soft >= 256:
        assert size >= min(soft, 2048), size
    else:
        assert size < 256, size


def test_a_forked_child_grows_its_fd_table_again(native_shim):
    """fork() gives the child an fd table only as large as its highest open fd: a pod process
    forked from a pre-started parent would grow it again at its TAKE, multi-threaded by then. The
    shim grows it in the child right after the fork."""
    import resource

    soft, _ = resource.getrlimit(resource.RLIMIT_NOFILE)
    if soft < 256:
        pytest.skip("RLIMIT_NOFILE below 256")
    code = ("import os\n"
            "pid = os.fork()\n"
            "if pid == 0:\n"
            "    print([l.split()[1] for l in open('/proc/self/status') if l.startswith('FDSize:')][0], flush=True)\n"
            "    os._exit(0)\n"
            "os.waitpid(pid, 0)\n")
    env = dict(os.environ, LD_PRELOAD=preload(native_shim))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True).stdout
    assert int(out.split()[0]) >= min(soft, 2048), out
    env["GPUSHARE_SHIM_FD_RESERVE"] = "0"
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True).stdout
    assert int(out.split()[0]) < 256, out


def test_broker_refusal_leaves_the_pod_on_the_driver(stub, native_shim, tmp_path):
    sock = str(tmp_path / "hbm.sock")
    b = FakeBroker(sock, refuse=True)
    name = ledger()
    try:
        out, r = run(stub, native_shim, ["alloc", GIB, "arena", "stats"], GPUSHARE_QUOTA_BYTES=4 * GIB,
                     GPUSHARE_LEDGER=name, GPUSHARE_HBM_BROKER=sock, GPUSHARE_HBM_TOKEN="nope")
        assert r.returncode == 0, r.stderr
        assert b.took == "TAKE nope STREAM"
        assert out[0]["err"] == 0 and out[1]["on"] == 0 and out[2]["used"] == GIB   # quota shim as before
    finally:
        cleanup(name)


@pytest.mark.parametrize("mode", ["whole", "stream"])
@pytest.mark.parametrize("san", ["asan", "tsan"])
def test_broker_arena_under_sanitizers(stub, tmp_path, san, mode):
    """Threads allocating and freeing from the broker arena at once, under ASan+UBSan / TSan:
    8 threads in a 2-granule arena, or ("stream") 3 threads of 1 GiB blocks in a 3-granule grant
    of which 1 granule is there at first and 2 arrive 0.2 s later, so two threads wait for the
    owed granules while the third allocates and frees."""
    import sys
    sys.path.insert(0, os.path.join(HERE, "..", "native"))
    import build as nb
    lib = nb.build_hipshim(asan=san)[0]
    rt = subprocess.run(["gcc", f"-print-file-name=lib{san}.so"], capture_output=True, text=True).stdout.strip()
    if not os.path.exists(rt):
        pytest.skip(f"lib{san}.so not installed")
    d, drv = stub
    sock = str(tmp_path / "hbm.sock")
    b = FakeBroker(sock, granules=2) if mode == "whole" else FakeBroker(sock, granules=3, stream=[(0.2, 2)])
    name = ledger()
    env = dict(os.environ, LD_PRELOAD=preload(rt, lib), LD_LIBRARY_PATH=str(d), GPUSHARE_LEDGER=name,
               GPUSHARE_QUOTA_BYTES=str(4 * GIB), GPUSHARE_HBM_BROKER=sock, GPUSHARE_HBM_TOKEN="t",
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               TSAN_OPTIONS="halt_on_error=1:report_bugs=1")
    try:
        nt, it, sz = (8, 300, 64 * MIB) if mode == "whole" else (3, 20, GIB)
        r = subprocess.run([str(drv), "threads", str(nt), str(it), str(sz), "arena", "arenarelease"], env=env,
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-3000:]
        out = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
        assert out[0]["ok"] == nt * it and out[0]["denied"] == 0
        assert out[1] == {"op": "arena", "on": 1, "size": (2 if mode == "whole" else 3) * GIB, "used": 0}
        assert out[2]["r"] == 1 and b.took == "TAKE t STREAM"
    finally:
        cleanup(name)


def test_broker_arena_larger_than_the_quota_is_not_used(stub, native_shim, tmp_path):
    """A grant bigger than the pod's quota (a misconfigured granter) must not lift the quota: the
    shim hands the granules back and the pod allocates from the driver under its quota."""
    sock = str(tmp_path / "hbm.sock")
    b = FakeBroker(sock, granules=4)
    name = ledger()
    try:
        out, r = run(stub, native_shim, ["alloc", GIB, "arena", "alloc", 3 * GIB, "stats"], GPUSHARE_QUOTA_BYTES=2 * GIB,
                     GPUSHARE_LEDGER=name, GPUSHARE_HBM_BROKER=sock, GPUSHARE_HBM_TOKEN="big")
        assert r.returncode == 0, r.stderr
        assert out[0]["err"] == 0 and out[1]["on"] == 0
        assert out[2]["err"] == 2 and out[3]["used"] == GIB
        import time
        for _ in range(50):
            if b.closed_at is not None:
                break
            time.sleep(0.02)
        assert b.closed_at is not None                           # the granules went back at once
    finally:
        cleanup(name)


def test_broker_arena_serves_stream_ordered_allocations(stub, native_shim, tmp_path):
    """hipMallocAsync and hipMallocFromPoolAsync (the default pool: PyTorch's
    cudaMallocAsync backend) come from the arena like hipMalloc; a hipFreeAsync'd block is reused
    once its stream got past the free (an event), and an allocation that needs it waits for that
    instead of going to the driver."""
    sock = str(tmp_path / "hbm.sock")
    FakeBroker(sock, granules=4)
    name = ledger()
    try:
        out, r = run(stub, native_shim, ["async", 2 * GIB, "poolasync", GIB, "arena", "freeasync", 0,
                                         "async", 2 * GIB, "arena", "stats", "info"],
                     GPUSHARE_QUOTA_BYTES=8 * GIB, GPUSHARE_LEDGER=name, GPUSHARE_HBM_BROKER=sock,
                     GPUSHARE_HBM_TOKEN="tok", FAKE_HIP_EVENT_MS=300)
        assert r.returncode == 0, r.stderr
        a2, p1, arena, _, again, arena2, st, info = out
        assert a2["err"] == 0 and p1["err"] == 0
        assert arena == {"op": "arena", "on": 1, "size": 4 * GIB, "used": 3 * GIB}
        assert again["err"] == 0 and again["p"] == a2["p"]          # waited for the stream, reused
        assert arena2["used"] == 3 * GIB
        assert st["used"] == 4 * GIB and st["denied"] == 0           # the arena only: nothing from the driver
        assert info["total"] == 8 * GIB and info["free"] == 5 * GIB  # the arena's rest + the quota's rest
    finally:
        cleanup(name)


@pytest.mark.parametrize("align_cap", [None, 2 * MIB])
def test_broker_arena_serves_vmm_pages(stub, native_shim, tmp_path, align_cap):
    """VMM the way PyTorch's expandable segments use it (a large reserved
    range, 20 MiB pages created and mapped one after another) is served from the arena: the
    range is aligned to the granule, its slots are backed by arena granules on demand (a page may
    straddle two), unmapping a slot's last page gives its granule back, and past the arena the
    pages come from the driver, charged, until the quota is out. ``align_cap``: the runtime
    returns ranges aligned to 2 MiB only, whatever alignment is asked for (HIP 7.x on MI355X):
    the shim reserves a granule more and uses the aligned part."""
    sock = str(tmp_path / "hbm.sock")
    FakeBroker(sock, granules=4)
    name = ledger()
    page = 20 * MIB
    n1 = 60                                          # 1.17 GiB: two slots
    try:
        args = ["alloc", MIB, "vres", 9 * GIB] + ["vpage", page] * n1 + ["vstats", "arena", "stats"]
        args += sum((["vdrop", k] for k in range(n1)), []) + ["vstats", "arena"]
        extra = {"FAKE_HIP_RESERVE_ALIGN_MAX": str(align_cap)} if align_cap else {}
        out, r = run(stub, native_shim, args, GPUSHARE_QUOTA_BYTES=8 * GIB, GPUSHARE_LEDGER=name,
                     GPUSHARE_HBM_BROKER=sock, GPUSHARE_HBM_TOKEN="tok", **extra)
        assert r.returncode == 0, r.stderr
        vres = out[1]
        assert vres == {"op": "vres", "err": 0, "aligned": 1}
        pages = out[2:2 + n1]
        assert all(p["err"] == 0 and p["map"] == 0 and p["access"] == 0 for p in pages)
        vs, arena, st = out[2 + n1:5 + n1]
        assert vs["windows"] == 1 and vs["creates"] == n1 and vs["real_pieces"] == 0
        assert vs["arena_maps"] == n1 + 1 and vs["slots_now"] == 2     # one page straddles the slots
        assert arena["used"] == 2 * GIB + MIB                          # two granules lent + the 1 MiB block
        assert st["used"] == 4 * GIB                                   # only the arena's charge
        drops = out[5 + n1:5 + 2 * n1]
        assert all(d == {"op": "vdrop", "unmap": 0, "release": 0} for d in drops)
        vs2, arena2 = out[5 + 2 * n1:]
        assert vs2["slots_now"] == 0 and arena2["used"] == MIB          # granules back in the arena
    finally:
        cleanup(name)


@pytest.mark.parametrize("refuse", [False, True])
def test_broker_arena_vmm_spills_to_the_driver_within_the_quota(stub, native_shim, tmp_path, refuse):
    """Past the arena, VMM pages come from the driver within the quota. ``refuse``: the runtime
    refuses the access call of a single driver page (HIP 7.x does, now and then); the shim sets
    it over the whole run of mappings ending at that page, which the runtime accepts."""
    sock = str(tmp_path / "hbm.sock")
    FakeBroker(sock, granules=4)
    name = ledger()
    half = GIB // 2
    try:
        args = ["vres", 12 * GIB] + ["vpage", half] * 17 + ["vstats", "stats", "info"]
        extra = {"FAKE_HIP_ACCESS_REFUSE_SIZE": str(half), "GPUSHARE_SHIM_LOG": "1"} if refuse else {}
        out, r = run(stub, native_shim, args, GPUSHARE_QUOTA_BYTES=8 * GIB, GPUSHARE_LEDGER=name,
                     GPUSHARE_HBM_BROKER=sock, GPUSHARE_HBM_TOKEN="tok", **extra)
        assert r.returncode == 0, r.stderr
        if refuse:   # each driver page: over the run from the window's start (4 arena slots, the pages before it)
            spans = [ln for ln in r.stderr.splitlines() if "refused; over the run from +0 " in ln]
            assert len(spans) == 8 and all(ln.endswith(": 0") for ln in spans), r.stderr
        pages = out[1:18]
        ok = [p for p in pages if p["err"] == 0]
        assert len(ok) == 16 and pages[16]["err"] == 2                 # 8 GiB: 4 arena + 4 driver, then OOM
        assert all(p["map"] == 0 for p in ok)
        vs, st, info = out[18:]
        assert vs["slots_now"] == 4 and vs["real_pieces"] == 8          # 8 half-GiB driver pages
        assert st["used"] == 8 * GIB and info["free"] == 0
    finally:
        cleanup(name)


@pytest.mark.parametrize("version,form", [(70051831, "address"), (70253211, "value")])
def test_broker_fds_are_imported_the_way_the_runtime_reads_them(stub, native_shim, tmp_path, version, form):
    """how a POSIX fd reaches hipMemImportFromShareableHandle is chosen by the
    runtime's version, not by probing errors. The stub runtime behaves like HIP 7.0 (reads the fd
    through the pointer, dies on a bare value) or 7.2 (takes the value, refuses an address)."""
    sock = str(tmp_path / "hbm.sock")
    FakeBroker(sock, granules=2)
    name = ledger()
    try:
        out, r = run(stub, native_shim, ["alloc", GIB, "arena"], GPUSHARE_QUOTA_BYTES=4 * GIB, GPUSHARE_LEDGER=name,
                     GPUSHARE_HBM_BROKER=sock, GPUSHARE_HBM_TOKEN="t", FAKE_HIP_VERSION=version, GPUSHARE_SHIM_LOG="2")
        assert r.returncode == 0, r.stderr
        assert out[1]["on"] == 1 and out[1]["size"] == 2 * GIB
        assert f"fds imported by {form}" in r.stderr
    finally:
        cleanup(name)


# ---- round 6: the whole quota usable, truthful free memory, frees that do not wait, IPC, fork and
# exit hygiene ------------------------------------------------
def test_extend_borrows_beyond_the_grant_then_the_driver_and_memgetinfo_tells_what_can_be_had(stub, native_shim,
                                                                                                tmp_path):
    """a pod can use its whole quota. Its grant is 4 granules of an 8 GiB quota
    (limit 8); past the grant the shim asks the broker for granules beyond it (EXTEND, the broker
    has 1 to lend), then uses the driver, charged to the same ledger. hipMemGetInfo reports what
    the pod can actually obtain: the arena's rest plus the quota's rest bounded by the driver's
    free memory and what the broker could lend (AVAIL), not the quota's rest alone."""
    sock = str(tmp_path / "hbm.sock")
    b = FakeBroker(sock, granules=4, stream=[], extra=1, limit=8)
    name = ledger()
    try:
        out, r = run(stub, native_shim, ["alloc", 3 * GIB, "info", "alloc", 3 * GIB // 2, "extra", "alloc", GIB, "extra",
                                         "arena", "stats", "info"],
                     GPUSHARE_QUOTA_BYTES=8 * GIB, GPUSHARE_LEDGER=name, GPUSHARE_HBM_BROKER=sock,
                     GPUSHARE_HBM_TOKEN="tok", FAKE_HIP_TOTAL_GIB=2)
        assert r.returncode == 0, r.stderr
        a3, info0, a15, x1, d1, x2, arena, st, info = out
        # before: 1 GiB of the arena + min(4 GiB of quota, 2 GiB driver + 1 granule to borrow)
        assert info0["free"] == GIB + 3 * GIB and info0["total"] == 8 * GIB
        assert a15["err"] == 0 and a15["p"] == a3["p"] + 3 * GIB          # the borrowed granule joins the tail
        assert x1["extends"] == 1 and x1["extended"] == 1 and x1["limit"] == 8 and x1["driver_allocs"] == 0
        assert d1["err"] == 0 and not a3["p"] <= d1["p"] < a3["p"] + 8 * GIB   # nothing left to borrow: the driver
        assert x2["driver_allocs"] == 1 and x2["driver_bytes"] == GIB
        assert arena["size"] == 5 * GIB and arena["used"] == 3 * GIB + 3 * GIB // 2
        assert st["used"] == 6 * GIB and st["denied"] == 0
        # after: 0.5 GiB of the arena + min(2 GiB of quota, 1 GiB the driver still has + 0 to borrow)
        assert info["free"] == GIB // 2 + GIB
        assert b.requests == ["AVAIL", "EXTEND 1", "EXTEND 1", "AVAIL"]
    finally:
        cleanup(name)


def test_extend_never_asks_beyond_the_quota_left(stub, native_shim, tmp_path):
    sock = str(tmp_path / "hbm.sock")
    b = FakeBroker(sock, granules=4, stream=[], extra=4, limit=8)
    name = ledger()
    try:
        # 4.75 GiB quota: 4 granules charged, 0.75 GiB left, no whole granule to borrow
        out, r = run(stub, native_shim, ["alloc", 4 * GIB, "alloc", GIB // 2, "extra", "stats"],
                     GPUSHARE_QUOTA_BYTES=4 * GIB + 3 * GIB // 4, GPUSHARE_LEDGER=name, GPUSHARE_HBM_BROKER=sock,
                     GPUSHARE_HBM_TOKEN="tok")
        assert r.returncode == 0, r.stderr
        a4, half, x, st = out
        assert a4["err"] == 0 and half["err"] == 0 and x["extends"] == 0 and x["driver_allocs"] == 1
        assert st["used"] == 4 * GIB + GIB // 2 and b.requests == []
    finally:
        cleanup(name)


def test_hipfree_of_an_arena_block_does_not_wait_for_the_device(stub, native_shim, tmp_path):
    """hipFree of an arena block used to synchronise the whole device. Now it
    records an event on every stream of the device (and the null stream) and returns; the block is
    reused once they have completed (here the stub's events complete 400 ms after they are
    recorded), and an allocation that needs the room waits for them instead of going to the driver."""
    sock = str(tmp_path / "hbm.sock")
    FakeBroker(sock, granules=4)
    name = ledger()
    try:
        out, r = run(stub, native_shim, ["alloc", 3 * GIB, "timefree", 0, "freestats", "arena", "timealloc", 4 * GIB,
                                         "arena", "freestats", "extra"],
                     GPUSHARE_QUOTA_BYTES=8 * GIB, GPUSHARE_LEDGER=name, GPUSHARE_HBM_BROKER=sock,
                     GPUSHARE_HBM_TOKEN="tok", FAKE_HIP_EVENT_MS=400)
        assert r.returncode == 0, r.stderr
        a3, tf, fs, arena, ta, arena2, fs2, x = out
        assert tf["err"] == 0 and tf["ms"] < 50, tf                        # returned without waiting
        assert fs["deferred"] == 1 and fs["pending"] == 1 and fs["device_waits"] == 0
        assert arena["used"] == 3 * GIB                                    # not reusable yet
        assert ta["err"] == 0 and ta["p"] == a3["p"] and ta["ms"] >= 250   # waited for the events, from the arena
        assert arena2["used"] == 4 * GIB and fs2["pending"] == 0 and x["driver_allocs"] == 0
    finally:
        cleanup(name)


def test_arena_memory_is_shared_between_processes_through_ipc_handles(stub, native_shim, tmp_path):
    """hipIpcGetMemHandle of arena memory (the runtime's own cannot export it)
    gives a handle another process of the pod opens: the exporter's shim sends the fds of the
    granules the allocation spans over its socket, the importer maps them (its import is freed again
    at hipIpcCloseMemHandle). hipMemGetAddressRange answers with the allocation, not the granule;
    hipMemRetainAllocationHandle gives no handle of arena memory (the broker's)."""
    d, drv = stub
    sock = str(tmp_path / "hbm.sock")
    FakeBroker(sock, granules=4)
    name = ledger()
    env = dict(os.environ, LD_PRELOAD=native_shim, LD_LIBRARY_PATH=str(d), GPUSHARE_QUOTA_BYTES=str(8 * GIB),
               GPUSHARE_LEDGER=name, GPUSHARE_HBM_BROKER=sock, GPUSHARE_HBM_TOKEN="tok")
    args = ["alloc", 3 * GIB // 2, "alloc", 2 * GIB, "ipcget", 1, "range", 0, 12345, "range", 1, GIB + 7, "retain", 1,
            "wait", "ipcstats"]
    exp = subprocess.Popen([str(drv), *map(str, args)], env={k: str(v) for k, v in env.items()},
                           stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        lines = [json.loads(exp.stdout.readline()) for _ in range(6)]
        a0, a1, h, r0, r1, ret = lines
        assert h["err"] == 0 and a1["err"] == 0
        assert r0 == {"op": "range", "err": 0, "base": a0["p"], "size": 3 * GIB // 2}
        assert r1 == {"op": "range", "err": 0, "base": a1["p"], "size": 2 * GIB}   # spans granules 1..3
        assert ret["err"] == 1                                                     # hipErrorInvalidValue
        out, r = run(stub, native_shim, ["ipcopen", h["handle"], "range", 0, 100, "ipcstats", "imports", "ipcclose", 0,
                                         "ipcstats", "imports"], GPUSHARE_QUOTA_BYTES=4 * GIB)
        assert r.returncode == 0, r.stderr
        op, rng, st, imp, cl, st2, imp2 = out
        assert op["err"] == 0 and rng["err"] == 0 and rng["base"] == op["p"] and rng["size"] == 2 * GIB
        assert st["opened"] == 1 and st["open_now"] == 1 and imp["live"] == 3    # granules 1, 2, 3 of the exporter
        assert cl["err"] == 0 and st2["open_now"] == 0 and imp2["live"] == 0
        bad = h["handle"][:24] + "ffffffff" + h["handle"][32:]                    # an export that does not exist
        out, r = run(stub, native_shim, ["ipcopen", bad])
        assert out[0]["err"] != 0
        exp.stdin.close()
        tail = json.loads(exp.stdout.readline())
        assert tail["exports"] == 1 and tail["served"] == 1
        assert exp.wait(10) == 0
    finally:
        if exp.poll() is None:
            exp.kill()
        cleanup(name)


def test_a_forked_child_does_not_keep_the_parents_granules(stub, native_shim, tmp_path):
    """A child forked by a pod process (a data-loader worker) inherits the broker connection and
    the granules' fds: it used to keep the parent's granules from the broker until it exited too.
    The shim closes its copies in the child at the fork: the broker sees the connection end when
    the parent exits."""
    import time

    sock = str(tmp_path / "hbm.sock")
    b = FakeBroker(sock, granules=2)
    name = ledger()
    try:
        t0 = time.monotonic()
        out, r = run(stub, native_shim, ["alloc", GIB, "forksleep", 3000, "alloc", MIB],
                     GPUSHARE_QUOTA_BYTES=4 * GIB, GPUSHARE_LEDGER=name, GPUSHARE_HBM_BROKER=sock, GPUSHARE_HBM_TOKEN="t")
        assert r.returncode == 0 and out[2]["err"] == 0, r.stderr
        for _ in range(100):
            if b.closed_at is not None:
                break
            time.sleep(0.02)
        assert b.closed_at is not None and b.closed_at - t0 < 2.5        # not the child's 3 s
    finally:
        cleanup(name)


@pytest.mark.parametrize("case", ["sigterm", "handler", "exit", "off"])
def test_fast_exit_hands_the_granules_back(stub, native_shim, tmp_path, case):
    """a pod stopped the way the kubelet stops it (SIGTERM, default action) or
    that just exits never calls gpushare_shim_arena_release(); the kernel would release its
    imports of the broker's granules only once it has torn the process down (300-380 ms on
    MI355X). The shim does it first: at SIGTERM it destroys the process's queues and frees the
    imports, then lets the signal end the process; at the end of a normal exit likewise. A program
    with its own SIGTERM handler keeps it; GPUSHARE_SHIM_FAST_EXIT=0 leaves it all to the kernel."""
    import signal
    import time

    d, drv = stub
    sock = str(tmp_path / "hbm.sock")
    b = FakeBroker(sock, granules=2)
    name = ledger()
    env = {k: str(v) for k, v in dict(os.environ, LD_PRELOAD=native_shim, LD_LIBRARY_PATH=str(d),
                                      GPUSHARE_QUOTA_BYTES=str(4 * GIB), GPUSHARE_LEDGER=name,
                                      GPUSHARE_HBM_BROKER=sock, GPUSHARE_HBM_TOKEN="t", GPUSHARE_SHIM_LOG="1",
                                      GPUSHARE_SHIM_FAST_EXIT="0" if case == "off" else "1").items()}
    args = ["alloc", GIB, "wait"] if case != "exit" else ["alloc", GIB]
    if case == "handler":
        args = ["sigterm_handler"] + args
    p = subprocess.Popen([str(drv), *map(str, args)], env=env, stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True)
    try:
        first = p.stdout.readline() if case != "handler" else (p.stdout.readline(), p.stdout.readline())[1]
        assert json.loads(first)["err"] == 0
        if case != "exit":
            p.send_signal(signal.SIGTERM)
        p.wait(20)                                   # stdin stays open: "wait" holds the process until the signal
        out, err = p.stdout.read(), p.stderr.read()
        if case in ("sigterm", "off"):
            assert p.returncode == -signal.SIGTERM, err
        else:
            assert p.returncode == 0, err
        fast = [ln for ln in err.splitlines() if "fast exit" in ln]
        if case == "sigterm":
            assert len(fast) == 1 and "fast exit (SIGTERM)" in fast[0] and "2 imports freed" in fast[0], err
        elif case == "exit":
            assert len(fast) == 1 and "fast exit (exit)" in fast[0] and "2 imports freed" in fast[0], err
        else:
            assert not fast, err
        if case == "handler":
            assert '"handled"' in out
        for _ in range(100):
            if b.closed_at is not None:
                break
            time.sleep(0.02)
        assert b.closed_at is not None
    finally:
        if p.poll() is None:
            p.kill()
        cleanup(name)
