"""Kernel HBM limits through the dmem cgroup controller (quota/dmem.py) on a synthetic cgroup v2
tree: regions from dmem.capacity, the pod cgroup in both kubelet naming schemes, +dmem switched on
down the path, dmem.max following the (re-homed) placement, and an inactive no-op where the kernel
has no dmem controller. The GPU boxes' kernel (6.18, controllers: cpuset cpu io memory hugetlb pids
misc) has none, so this is the only place the writes are exercised (profiles/r3/dmem_probe.txt)."""
from aliyun_gpushare_device_plugin_amd import const
from aliyun_gpushare_device_plugin_amd.device.model import DeviceModel
from aliyun_gpushare_device_plugin_amd.quota.dmem import DmemLimits
from aliyun_gpushare_device_plugin_amd.utils.metrics import PluginMetrics

from .test_allocate_engine import StaticSource, mkpod
from .test_units_and_model import gpu

GIB = 1 << 30
UID_A = "0b6f1c2e-aaaa-bbbb-cccc-0123456789ab"
UID_B = "1c7e2d3f-dddd-eeee-ffff-0123456789ab"


def _tree(tmp_path, model, with_dmem=True):
    root = tmp_path / "cgroup"
    root.mkdir()
    (root / "cgroup.controllers").write_text("cpuset cpu io memory pids" + (" dmem" if with_dmem else "") + "\n")
    (root / "cgroup.subtree_control").write_text("cpu memory pids\n")
    if with_dmem:
        (root / "dmem.capacity").write_text("".join(f"drm/{g.bdf}/vram0 {g.vram_bytes}\n" for g in model.gpus)
                                            + "drm/0000:ff:00.0/vram0 1024\n")
    sysd = root / "kubepods.slice" / "kubepods-burstable.slice"
    a = sysd / f"kubepods-burstable-pod{UID_A.replace('-', '_')}.slice"
    a.mkdir(parents=True)
    for d in (root / "kubepods.slice", sysd):
        (d / "cgroup.subtree_control").write_text("cpu memory\n")
    (a / "cgroup.subtree_control").write_text("")
    fs = root / "kubepods" / "besteffort" / f"pod{UID_B}"
    fs.mkdir(parents=True)
    for d in (root / "kubepods", root / "kubepods" / "besteffort"):
        (d / "cgroup.subtree_control").write_text("")
    return root, a, fs


def _model():
    return DeviceModel([gpu(0, 16 * GIB), gpu(1, 16 * GIB)], const.GIB)        # 16 units per GPU


def _limits(path):
    out = {}
    for ln in (path / "dmem.max").read_text().splitlines():
        name, v = ln.split()
        out[name] = v if v == "max" else int(v)
    return out


def test_shares_become_dmem_max_on_both_cgroup_layouts(tmp_path):
    model = _model()
    root, a, b = _tree(tmp_path, model)
    pa = mkpod("a", 4, 1, 10, assigned="true", phase="Running", uid=UID_A)      # 4 GiB on GPU 1
    pb = mkpod("b", 8, 0, 11, assigned="true", phase="Running", uid=UID_B)      # 8 GiB on GPU 0
    m = PluginMetrics()
    d = DmemLimits(model, StaticSource([pa, pb]), m, cgroup_root=str(root))
    assert d.available()
    assert d.regions() == {0: f"drm/{model.gpu(0).bdf}/vram0", 1: f"drm/{model.gpu(1).bdf}/vram0"}
    assert d.sync() == 2
    r0, r1 = d.regions()[0], d.regions()[1]
    assert _limits(a) == {r1: 4 * GIB} and _limits(b) == {r0: 8 * GIB}     # other GPUs: kernel default
    for anc in (root, root / "kubepods.slice", root / "kubepods.slice" / "kubepods-burstable.slice",
                root / "kubepods", root / "kubepods" / "besteffort"):
        assert "dmem" in (anc / "cgroup.subtree_control").read_text()
    assert m.dmem_limited_pods.value() == 2


def test_limits_follow_a_rehomed_placement_and_forget_gone_pods(tmp_path):
    model = _model()
    root, a, _ = _tree(tmp_path, model)
    pa = mkpod("a", 4, 1, 10, assigned="true", phase="Running", uid=UID_A)
    src = StaticSource([pa])
    d = DmemLimits(model, src, cgroup_root=str(root))
    d.sync()
    (a / "dmem.max").write_text("")                       # unchanged placement: not rewritten
    d.sync()
    assert (a / "dmem.max").read_text() == ""
    pa["metadata"]["annotations"][const.ENV_RESOURCE_INDEX] = "0"            # placement truth moved it
    d.sync()
    assert _limits(a) == {d.regions()[0]: 4 * GIB, d.regions()[1]: "max"}   # old region back to max
    src.pods = []
    d.sync()
    assert d.applied == {}


def test_inactive_without_the_controller_or_regions(tmp_path):
    model = _model()
    root, a, _ = _tree(tmp_path, model, with_dmem=False)
    pa = mkpod("a", 4, 1, 10, assigned="true", phase="Running", uid=UID_A)
    d = DmemLimits(model, StaticSource([pa]), cgroup_root=str(root))
    assert not d.available() and d.sync() == 0 and not (a / "dmem.max").exists()
    assert DmemLimits(model, StaticSource([pa]), cgroup_root=str(root), mode="off").sync() == 0


def test_unplaced_or_foreign_pods_are_left_alone(tmp_path):
    model = _model()
    root, a, _ = _tree(tmp_path, model)
    pending = mkpod("a", 4, -1, 10, uid=UID_A)                                  # no GPU chosen yet
    d = DmemLimits(model, StaticSource([pending]), cgroup_root=str(root))
    assert d.sync() == 0 and not (a / "dmem.max").exists()
    other = mkpod("c", 4, 1, 10, assigned="true", phase="Running", uid="22222222-3333-4444-5555-666666666666")
    assert DmemLimits(model, StaticSource([other]), cgroup_root=str(root)).sync() == 0   # no cgroup here


def test_plugin_requests_prestart_when_limits_are_active(tmp_path):
    """With the controller present the allocator runs the limits before each container start, and
    the plugin asks the kubelet for PreStartContainer even without pod-resources."""
    from aliyun_gpushare_device_plugin_amd.plugin.server import DevicePluginServer

    from .test_allocate_engine import make

    pa = mkpod("a", 4, 1, 10, assigned="true", phase="Running", uid=UID_A)
    alloc, _, _ = make([pa], ngpu=2, gib=16)
    model = alloc.model
    root, a, _ = _tree(tmp_path, model)
    srv = DevicePluginServer(model, alloc, socket_path=str(tmp_path / "p.sock"))
    assert not srv.options().pre_start_required
    d = DmemLimits(model, alloc.pods, cgroup_root=str(root))
    alloc.prestart_hooks.append(d.sync)
    assert srv.options().pre_start_required
    alloc.prestart(None)
    assert _limits(a)[d.regions()[1]] == 4 * GIB
