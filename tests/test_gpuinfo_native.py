"""libgpushare_gpuinfo on CPU: fake backend (+fault injection), sysfs backend on a synthetic
KFD/DRM tree shaped like the one measured on MI355X, and the gpushare-smi CLI."""
import json
import os
import subprocess

import pytest
from aliyun_gpushare_device_plugin_amd.utils.native import preload

from aliyun_gpushare_device_plugin_amd.device import smi as S
from aliyun_gpushare_device_plugin_amd.utils.native import NATIVE_DIR


def test_fake_shorthand():
    with S.SMI("fake:8x288G") as s:
        assert s.backend == "fake" and s.count() == 8
        g = s.device(3)
        assert g.vram_total == 288 << 30 and g.gfx == "gfx950" and g.uuid.startswith("GPU-")
        assert s.link(0, 5).type == S.LINK_XGMI and s.link(0, 5).hops == 1
        assert s.link(2, 2).type == S.LINK_SELF


def test_fake_bytes_suffix():
    with S.SMI("fake:1x309220868096B") as s:
        assert s.device(0).vram_total == 309220868096


def test_fake_json_spec(tmp_path):
    spec = {"devices": [{"uuid": "GPU-aaaa", "vram_total": 4 << 30, "numa_node": 0, "render_minor": 130},
                        {"uuid": "GPU-bbbb", "vram_total": 4 << 30, "numa_node": 1}],
            "xgmi": [[0, 2], [2, 0]]}
    p = tmp_path / "spec.json"
    p.write_text(json.dumps(spec))
    with S.SMI(f"fake:{p}") as s:
        assert [d.uuid for d in s.devices()] == ["GPU-aaaa", "GPU-bbbb"]
        assert s.device(0).render_minor == 130 and s.device(1).numa_node == 1
        assert s.link(0, 1).type == S.LINK_PCIE


def test_fake_json_partitions_share_socket(tmp_path):
    """CPX-style partitions (same unique id) -> one socket in the model and the topology export."""
    from aliyun_gpushare_device_plugin_amd import const
    from aliyun_gpushare_device_plugin_amd.device.model import DeviceModel
    from aliyun_gpushare_device_plugin_amd.parallel.topology import build_topology
    devs = [{"uuid": f"GPU-p{i}", "vram_total": 288 << 30, "unique_id": 4096 + i // 2, "compute_partition": 2,
             "memory_partition": 1} for i in range(4)]
    p = tmp_path / "cpx.json"
    p.write_text(json.dumps({"devices": devs}))
    with S.SMI(f"fake:{p}") as s:
        assert [d.unique_id for d in s.devices()] == [4096, 4096, 4097, 4097]
        assert [g.units for g in DeviceModel(s.devices(), const.GIB).gpus] == [144] * 4
        topo = build_topology(s)
        assert [(g["socket"], g["partition_index"]) for g in topo["gpus"]] == [(0, 0), (0, 1), (1, 0), (1, 1)]


def test_fault_injection_events_and_membership():
    with S.SMI("fake:4x288G") as s:
        s.inject("unplug 2")
        ev = s.wait_event(1000)
        assert ev.kind == S.EV_UNPLUG and ev.index == 2
        assert s.refresh() == 3
        assert "GPU-fa6e000000000002" not in [d.uuid for d in s.devices()]
        s.inject("replug 2")
        assert s.wait_event(1000).kind == S.EV_REPLUG
        assert s.refresh() == 4
        s.inject("reset 1")
        assert [s.wait_event(1000).kind for _ in range(2)] == [S.EV_PRE_RESET, S.EV_POST_RESET]
        s.inject("ecc 0 3")
        assert s.wait_event(1000).kind == S.EV_ECC_UE
        s.refresh()
        assert s.device(0).ecc_ue == 3
        s.inject("linkdown 0 1")
        s.refresh()
        assert s.link(0, 1).type == S.LINK_PCIE and s.link(1, 0).type == S.LINK_PCIE
        assert s.link(0, 2).type == S.LINK_XGMI
        assert s.wait_event(10).kind == S.EV_LINK_DOWN
        assert s.wait_event(10) is None
        with pytest.raises(S.SMIError):
            s.inject("explode 0")


def test_unknown_backend_errors():
    with pytest.raises(S.SMIError):
        S.SMI("nvml")
    with pytest.raises(S.SMIError):
        S.SMI("fake:0x1G")


def _write(path, text):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        f.write(text)


def make_sysfs(root, ngpu=2):
    """Mimics the KFD/DRM layout read on an MI355X box (gpurun_out/probe)."""
    nodes = f"{root}/sys/class/kfd/kfd/topology/nodes"
    _write(f"{nodes}/0/properties", "cpu_cores_count 128\nsimd_count 0\n")
    for i in range(ngpu):
        n = 2 + i
        minor = 128 + 8 * i
        _write(f"{nodes}/{n}/properties",
               f"cpu_cores_count 0\nsimd_count 1024\nsimd_per_cu 4\ngfx_target_version 90500\n"
               f"location_id {0x0a00 + 0x1000 * i}\ndomain 0\ndrm_render_minor {minor}\n"
               f"hive_id 12051920080120582036\nunique_id {16966105145620891471 + i}\nnum_xcc 8\n")
        _write(f"{nodes}/{n}/mem_banks/0/properties", "heap_type 1\nsize_in_bytes 309220868096\n")
        links = [(0, 2, 20)] + [(2 + j, 11, 15) for j in range(ngpu) if j != i]
        for k, (to, typ, w) in enumerate(links):
            _write(f"{nodes}/{n}/io_links/{k}/properties",
                   f"type {typ}\nnode_from {n}\nnode_to {to}\nweight {w}\nmax_bandwidth 153600\n")
        dev = f"{root}/sys/class/drm/renderD{minor}/device"
        _write(f"{dev}/mem_info_vram_total", "309220868096\n")
        _write(f"{dev}/mem_info_vram_used", "297766912\n")
        _write(f"{dev}/product_name", "AMD Instinct MI355 OAM\n")
        _write(f"{dev}/numa_node", f"{i // 4}\n")
        _write(f"{dev}/current_compute_partition", "SPX\n")
        _write(f"{dev}/current_memory_partition", "NPS1\n")
        _write(f"{dev}/ras/umc_err_count", "ue: 0\nce: 2\n")


def test_sysfs_backend_on_synthetic_tree(tmp_path):
    make_sysfs(str(tmp_path), 3)
    with S.SMI(f"sysfs:{tmp_path}") as s:
        assert s.backend == "sysfs" and s.count() == 3
        g = s.device(0)
        assert g.uuid == "GPU-eb73b6bd5aa9074f" and g.bdf == "0000:0a:00.0"
        assert g.vram_total == 309220868096 and g.gfx == "gfx950" and g.num_cu == 256
        assert g.render_minor == 128 and g.name == "AMD Instinct MI355 OAM"
        assert g.compute_partition == 1 and g.memory_partition == 1 and g.ecc_ce == 2
        assert s.link(0, 1).type == S.LINK_XGMI and s.link(0, 1).hops == 1 and s.link(0, 1).weight == 15
        assert s.device(1).bdf == "0000:1a:00.0"
        st = s.health_status()
        assert st["ecc_api"] == 1 and st["ecc_reads_ok"] == 3 and st["ecc_reads_failed"] == 0
        assert st["events_api"] == 0 and st["refreshes"] >= 1       # sysfs: polling only
    os.remove(f"{tmp_path}/sys/class/drm/renderD136/device/ras/umc_err_count")
    with S.SMI(f"sysfs:{tmp_path}") as s:
        st = s.health_status()
        assert st["ecc_reads_ok"] == 2 and st["ecc_reads_failed"] == 1


def test_health_status_fake_backend():
    with S.SMI("fake:4x288G") as s:
        assert s.health_status()["events_armed"] == 0
        s.events_start()
        st = s.health_status()
        assert st["events_api"] == 1 and st["events_armed"] == 4 and st["ecc_reads_ok"] == 4


def test_sysfs_missing_tree_errors(tmp_path):
    with pytest.raises(S.SMIError):
        S.SMI(f"sysfs:{tmp_path}/nothing")


def test_smi_cli_json(native_gpuinfo, tmp_path):
    cli = os.path.join(NATIVE_DIR, "gpushare-smi")
    r = subprocess.run([cli, "--backend", "fake:2x4G", "--json"], capture_output=True, text=True, check=True)
    d = json.loads(r.stdout)
    assert d["backend"] == "fake" and len(d["devices"]) == 2 and d["links"][0][1]["type"] == S.LINK_XGMI
    r = subprocess.run([cli, "--backend", "fake:2x4G"], capture_output=True, text=True, check=True)
    assert "XGMI1" in r.stdout and "gfx950" in r.stdout


_SAN_SCRIPT = r"""
import threading
from aliyun_gpushare_device_plugin_amd.device import smi as S
with S.SMI("fake:8x288G") as s:
    assert s.count() == 8
    m = s.link_matrix()
    assert m[0][1].type == S.LINK_XGMI
    def poll():
        for _ in range(50):
            s.refresh()
    t = threading.Thread(target=poll)
    t.start()
    for k in range(4):
        s.inject(f"unplug {k}"); s.wait_event(1000)
        s.inject(f"replug {k}"); s.wait_event(1000)
        s.inject(f"reset {k}"); s.wait_event(1000); s.wait_event(1000)
        s.inject(f"linkdown {k} {k + 1}"); s.wait_event(1000)
    t.join()
    # close while another thread is blocked in wait_event: must wait for it, not free under it
    waiter = threading.Thread(target=lambda: s.wait_event(300))
    waiter.start()
    s.close()
    waiter.join()
    try:
        s.count()
        raise SystemExit("call after close did not raise")
    except S.SMIError:
        pass
print("SAN-OK")
"""


@pytest.mark.parametrize("san", ["asan", "tsan"])
def test_gpuinfo_under_sanitizers(san):
    """libgpushare_gpuinfo built with ASan+UBSan / TSan, exercised through fault injection with
    a concurrent refresh thread (the health monitor's pattern)."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "native", "build.py"), "gpuinfo", "--sanitize", san],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    rt = subprocess.run(["gcc", f"-print-file-name=lib{san}.so"], capture_output=True, text=True).stdout.strip()
    if not os.path.exists(rt):
        pytest.skip(f"lib{san}.so not installed")
    env = dict(os.environ, LD_PRELOAD=preload(rt), GPUSHARE_NATIVE_VARIANT=san, PYTHONPATH=root,
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               TSAN_OPTIONS="halt_on_error=1:report_signal_unsafe=0")
    r = subprocess.run([sys.executable, "-c", _SAN_SCRIPT], env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0 and "SAN-OK" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
    assert "ERROR: AddressSanitizer" not in r.stderr and "WARNING: ThreadSanitizer" not in r.stderr, r.stderr[-4000:]
    assert "runtime error" not in r.stderr, r.stderr[-4000:]
