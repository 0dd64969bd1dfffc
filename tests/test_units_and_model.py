"""Capacity math and the fake-device model (component C2)."""
import pytest

from aliyun_gpushare_device_plugin_amd import const
from aliyun_gpushare_device_plugin_amd.device.model import DeviceModel, fake_device_id, real_device_id
from aliyun_gpushare_device_plugin_amd.device.smi import GPU
from aliyun_gpushare_device_plugin_amd.utils import units as U

MI355X_BYTES = 309_220_868_096   # measured on MI355X (hipMemGetInfo / mem_info_vram_total)


def gpu(i, nbytes=MI355X_BYTES, numa=0, health=0):
    return GPU(index=i, uuid=f"GPU-{i:016x}", bdf=f"0000:{i:02x}:00.0", name="MI355X", gfx="gfx950",
               vram_total=nbytes, vram_used=0, numa_node=numa, render_minor=128 + i, kfd_node=2 + i,
               unique_id=i, hive_id=1, num_xcc=8, num_cu=256, compute_partition=1, memory_partition=1,
               ecc_ue=0, ecc_ce=0, health=health)


def test_units_for_mi355x():
    assert U.units_for_bytes(MI355X_BYTES, const.GIB, "nearest") == 288
    assert U.units_for_bytes(MI355X_BYTES, const.GIB, "floor") == 287
    assert U.units_for_bytes(MI355X_BYTES, const.MIB, "floor") == 294896
    assert U.units_for_bytes(4 << 30, const.GIB, "floor") == 4


def test_reference_unit_bug_not_reproduced():
    # the reference divides NVML *bytes* by 1024 and calls it GiB (nvidia.go:31-38)
    assert U.units_for_bytes(16 << 30, const.GIB) == 16 != (16 << 30) // 1024


def test_quota_is_proportional():
    assert U.quota_bytes(288, 288, MI355X_BYTES) == MI355X_BYTES
    assert U.quota_bytes(64, 288, MI355X_BYTES) == MI355X_BYTES * 64 // 288
    assert U.quota_bytes(0, 288, MI355X_BYTES) == 0


def test_normalize_unit_warns_and_defaults():
    assert U.normalize_unit("MiB") == "MiB"
    assert U.normalize_unit("TiB") == "GiB"


@pytest.mark.parametrize("q,v", [("2", 2), (64, 64), ("1k", 1000), ("1Ki", 1024), ("500m", 1), ("1.5", 2),
                                 ("2e3", 2000), ("0", 0)])
def test_parse_quantity(q, v):
    assert U.parse_quantity(q) == v


def test_fake_ids_roundtrip():
    fid = fake_device_id("GPU-abc", 7)
    assert fid == "GPU-abc-_-7" and real_device_id(fid) == "GPU-abc"


def test_model_device_list_and_topology():
    m = DeviceModel([gpu(0, numa=0), gpu(1, numa=1)], const.GIB, "nearest")
    devs = m.device_list()
    assert len(devs) == 576 and m.total_units() == 576
    assert devs[0].ID == "GPU-0000000000000000-_-0" and devs[0].health == const.HEALTHY
    assert devs[300].topology.nodes[0].ID == 1
    assert m.uuid_by_index(1) == "GPU-0000000000000001" and m.uuid_by_index(5) is None


def test_heterogeneous_uses_minimum_by_default():
    m = DeviceModel([gpu(0, 8 << 30), gpu(1, 4 << 30)], const.GIB, "floor")
    assert [g.units for g in m.gpus] == [4, 4]
    m2 = DeviceModel([gpu(0, 8 << 30), gpu(1, 4 << 30)], const.GIB, "floor", homogeneous=False)
    assert [g.units for g in m2.gpus] == [8, 4]


def test_gpu_subset_reindexes():
    m = DeviceModel([gpu(0), gpu(1), gpu(2)], const.GIB, gpu_indices=[1, 2])
    assert m.count() == 2 and m.gpus[0].uuid == "GPU-0000000000000001" and m.gpus[0].index == 0


def test_health_generation_and_recovery():
    m = DeviceModel([gpu(0, 4 << 30)], const.GIB)
    g0 = m.generation
    assert m.set_health(0, False, "reset")
    assert m.generation == g0 + 1
    assert all(d.health == const.UNHEALTHY for d in m.device_list())
    assert not m.set_health(0, False, "again")    # no change, no wake-up
    assert m.set_health(0, True, "recovered")
    assert all(d.health == const.HEALTHY for d in m.device_list())


def test_mib_mode_falls_back_to_gib_on_mi355x():
    """Round-1 review: MiB mode on 8 x MI355X (2.36 M fake devices) used to raise, and the
    plugin exited 1 -> DaemonSet crash loop. Now: GiB with a recorded reason; small GPUs keep MiB."""
    m = DeviceModel([gpu(i) for i in range(8)], const.MIB)
    assert m.unit == const.GIB and m.dev_units() == 288 and "MiB devices exceed" in m.unit_fallback
    small = DeviceModel([gpu(i, 4 << 30) for i in range(2)], const.MIB)
    assert small.unit == const.MIB and small.dev_units() == 4096 and not small.unit_fallback


def test_mib_fallback_end_to_end_and_impossible_config_parks(monkeypatch):
    """The plugin started with --memory-unit=MiB on an MI355X node registers in GiB and says so
    on the node; a node it can never advertise parks (exit code 0 on SIGTERM), never exits 1."""
    import dataclasses

    from aliyun_gpushare_device_plugin_amd.cluster import objects as O
    from aliyun_gpushare_device_plugin_amd.sim.cluster import SimCluster
    from aliyun_gpushare_device_plugin_amd.utils import units as U

    c = SimCluster([("n", "fake:2x309220868096B")])
    base = c._plugin_cfg
    c._plugin_cfg = lambda node: dataclasses.replace(base(node), memory_unit=const.MIB)
    with c:
        n = c.client.get_node("n")
        assert O.node_allocatable(n, const.RESOURCE_NAME) == 2 * 288
        assert O.annotations(n)[const.NODE_ANNOTATION_MEMORY_UNIT] == const.GIB
        assert c.manager("n").metrics.unit_fallback.value() == 1

    import signal
    import tempfile
    import threading
    import time

    from aliyun_gpushare_device_plugin_amd.device import smi as S
    from aliyun_gpushare_device_plugin_amd.plugin.manager import PluginConfig, SharedGPUManager

    monkeypatch.setattr(U, "MAX_FAKE_DEVICES_PER_NODE", 100)
    d = tempfile.mkdtemp(prefix="gs-park-", dir="/tmp")
    m = SharedGPUManager(PluginConfig(node_name="n", smi_backend="fake:1x288G", device_plugin_dir=d),
                         smi=S.SMI("fake:1x288G"))
    rc = []
    t = threading.Thread(target=lambda: rc.append(m.run(install_signals=False)), daemon=True)
    t.start()
    t0 = time.monotonic()
    while m.metrics.config_error.value() != 1 and time.monotonic() - t0 < 10:
        time.sleep(0.01)
    assert m.metrics.config_error.value() == 1 and t.is_alive()       # parked, not exited
    m.events.put(("signal", signal.SIGTERM))
    t.join(10)
    assert rc == [0]


def part(i, socket, cp=4, nps=1, nbytes=MI355X_BYTES):
    g = gpu(i, nbytes)
    return GPU(**{**g.__dict__, "unique_id": 0xabc0 + socket, "bdf": f"0000:{0x10 * socket:02x}:00.0",
                  "compute_partition": cp, "memory_partition": nps})


def test_partition_aware_divides_shared_hbm():
    """2 sockets in QPX x NPS1: 8 HIP devices, each reporting its socket's full HBM."""
    devs = [part(i, i // 4) for i in range(8)]
    m = DeviceModel(devs, const.GIB)
    assert m.count() == 8
    assert [g.units for g in m.gpus] == [72] * 8              # 288 GiB / 4 partitions
    assert [(g.socket, g.partition) for g in m.gpus] == [(s, p) for s in range(2) for p in range(4)]
    assert m.total_units() == 2 * 288                        # never more than the real HBM
    naive = DeviceModel(devs, const.GIB, partition_aware=False)
    assert naive.total_units() == 8 * 288                    # the 4x over-commit it prevents


def test_partition_aware_keeps_nps_split_memory():
    """NPS2 partitions report their own half of the HBM: taken as reported."""
    devs = [part(i, 0, cp=2, nps=2, nbytes=MI355X_BYTES // 2) for i in range(2)]
    assert [g.units for g in DeviceModel(devs, const.GIB).gpus] == [144, 144]
    spx = [gpu(i) for i in range(8)]                         # SPX: one device per socket
    assert DeviceModel(spx, const.GIB).total_units() == 8 * 288


def test_decode_ops_validate_on_host():
    import pytest
    import torch

    from aliyun_gpushare_device_plugin_amd.ops import decode as Dm

    kc = torch.zeros((2, 1, 256, 128), dtype=torch.bfloat16)
    with pytest.raises(ValueError):
        Dm.decode_attention(torch.zeros((2, 512), dtype=torch.bfloat16), kc, kc,
                            torch.zeros(2, dtype=torch.int32))                      # CPU tensors
    with pytest.raises(ValueError):
        Dm._check_cache(kc[:, :, :100], kc[:, :, :100])                              # Smax % 256
    with pytest.raises(ValueError):
        Dm.kv_append(torch.zeros((2, 128), dtype=torch.bfloat16), torch.zeros((2, 128), dtype=torch.bfloat16),
                     kc, kc, torch.zeros(2, dtype=torch.int64))
