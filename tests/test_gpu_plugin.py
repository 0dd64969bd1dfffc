"""BASELINE config 2 on real hardware: 1×MI355X advertised as 288 GiB, 4 pods × 64 GiB."""
import pytest

from aliyun_gpushare_device_plugin_amd import const
from aliyun_gpushare_device_plugin_amd.cluster import objects as O
from aliyun_gpushare_device_plugin_amd.sim.cluster import SimCluster

pytestmark = pytest.mark.gpu


def test_config2_binpack_on_real_mi355x():
    with SimCluster([("mi355x-node", "auto")]) as c:
        n = c.client.get_node("mi355x-node")
        assert O.node_allocatable(n, const.RESOURCE_COUNT) >= 1
        per_gpu = O.node_allocatable(n, const.RESOURCE_NAME) // O.node_allocatable(n, const.RESOURCE_COUNT)
        assert per_gpu == 288
        placed = []
        for i in range(4):
            pod, where, adm = c.run_pod(64)
            assert adm is not None and adm.error is None
            env = dict(adm.responses[0].envs)
            assert env[const.ENV_RESOURCE_BY_CONTAINER] == "64" and env[const.ENV_RESOURCE_BY_DEV] == "288"
            paths = {d.host_path for d in adm.responses[0].devices}
            assert const.KFD_DEVICE in paths and any(p.startswith("/dev/dri/renderD") for p in paths)
            placed.append(where)
        assert {g for _, g in placed} == {0}
        # 256 of 288 GiB used: a fifth 64 GiB pod must not fit on a single-GPU node
        _, where, _ = c.run_pod(64)
        assert where is None
        _, where, adm = c.run_pod(32)
        assert where is not None and adm.error is None


def test_hbm_arena_first_fit_and_player_on_slice():
    """bench.py's per-GPU arena: disjoint unit ranges, reuse after free, None when fragmented."""
    import torch
    from aliyun_gpushare_device_plugin_amd.models.gemm_player import GemmPlayer, HBMArena
    dev = torch.device("cuda", 0)
    arena = HBMArena(dev, 288)
    a = arena.alloc("a", 128)
    b = arena.alloc("b", 64)
    assert a.data_ptr() + a.numel() * 2 == b.data_ptr()          # contiguous, disjoint
    assert arena.alloc("c", 128) is None                          # only 96 units left
    arena.free("a")
    c = arena.alloc("c", 96)
    assert c.data_ptr() == a.data_ptr()                           # first fit reuses the hole
    p = GemmPlayer(0, dev, 1024, 1024, 1024, pool=b)
    p.run(3)
    p.synchronize()
    ref = p.a.float() @ p.b.float().t()
    assert (p.c.float() - ref).abs().max().item() < 0.05 * ref.abs().max().item()
    p.release()
