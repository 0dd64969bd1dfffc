"""Node-side quota watchdog (quota/watchdog.py) on a synthetic /proc: kernel-reported HBM per
process (amdgpu DRM fdinfo) attributed to pods by cgroup, compared with their share."""
import os
import subprocess
import time

import pytest

from aliyun_gpushare_device_plugin_amd import const
from aliyun_gpushare_device_plugin_amd.device.model import DeviceModel
from aliyun_gpushare_device_plugin_amd.quota import watchdog as W
from aliyun_gpushare_device_plugin_amd.utils.metrics import PluginMetrics

from .test_allocate_engine import StaticSource, mkpod
from .test_units_and_model import gpu

GIB = 1 << 30
UID_A = "0b6f1c2e-aaaa-bbbb-cccc-0123456789ab"
UID_B = "1c7e2d3f-dddd-eeee-ffff-0123456789ab"


def _proc(root, pid, cgroup, clients):
    """clients: [(fd, client id, bytes, bdf)]"""
    d = root / str(pid)
    (d / "fdinfo").mkdir(parents=True)
    (d / "cgroup").write_text(cgroup)
    for fd, cid, n, bdf in clients:
        (d / "fdinfo" / str(fd)).write_text(
            f"pos:\t0\nflags:\t02100002\ndrm-driver:\tamdgpu\ndrm-pdev:\t{bdf}\ndrm-client-id:\t{cid}\n"
            f"drm-total-vram:\t{n // 1024} KiB\ndrm-resident-vram:\t{n // 1024} KiB\n")


def _setup(tmp_path, a_bytes, mode="report"):
    model = DeviceModel([gpu(0, 16 * GIB), gpu(1, 16 * GIB)], const.GIB)     # 16 units per GPU
    pa = mkpod("a", 4, 1, 10, assigned="true", phase="Running", uid=UID_A)   # 4 GiB on GPU 1
    pb = mkpod("b", 8, 1, 11, assigned="true", phase="Running", uid=UID_B)
    root = tmp_path / "proc"
    bdf1 = model.gpu(1).bdf
    _proc(root, 100, f"0::/kubepods.slice/kubepods-burstable.slice/kubepods-burstable-pod{UID_A.replace('-', '_')}"
                     ".slice/cri-containerd-abc.scope\n", [(5, "11", a_bytes, bdf1), (9, "11", a_bytes, bdf1)])
    _proc(root, 200, f"12:memory:/kubepods/burstable/pod{UID_B}/0123abcd\n", [(4, "12", 6 * GIB, bdf1)])
    _proc(root, 300, "0::/system.slice/sshd.service\n", [(3, "13", GIB, bdf1)])           # not a pod
    m = PluginMetrics()
    wd = W.QuotaWatchdog(model, StaticSource([pa, pb]), m, mode=mode, slack_bytes=64 << 20, proc=str(root),
                         kfd_proc=str(tmp_path / "nokfd"), pids=lambda: {100, 200, 300})
    return wd, m


def test_cgroup_forms_and_fdinfo_parsing(tmp_path):
    wd, _ = _setup(tmp_path, 3 * GIB)
    assert W.pod_of_pid(100, wd.proc) == UID_A and W.pod_of_pid(200, wd.proc) == UID_B
    assert W.pod_of_pid(300, wd.proc) is None
    assert W.drm_usage(100, wd.proc) == {"11": (3 * GIB, wd.model.gpu(1).bdf)}   # dup'ed fd counted once


def test_within_share_is_quiet_and_foreign_use_is_exported(tmp_path):
    wd, m = _setup(tmp_path, 3 * GIB)
    assert wd.scan() == []
    assert m.unaccounted_hbm.value(gpu="1") == GIB and m.unaccounted_hbm.value(gpu="0") == 0
    assert m.pod_hbm_used.value(pod_uid=UID_A, gpu="1") == 3 * GIB
    assert m.pod_hbm_used.value(pod_uid=UID_B, gpu="1") == 6 * GIB


def test_over_share_is_reported(tmp_path):
    wd, m = _setup(tmp_path, 5 * GIB)           # pod a: 5 GiB held, 4 GiB share
    v = wd.scan()
    assert len(v) == 1 and v[0].pod_uid == UID_A and v[0].gpu == 1
    assert v[0].used == 5 * GIB and v[0].allowed == 4 * GIB and v[0].killed == []
    assert m.quota_violation.value(pod_uid=UID_A, gpu="1") == GIB


def test_kill_mode_ends_the_largest_process(tmp_path):
    """kill: the violating pod's process is SIGKILLed (a real child here), like a cgroup OOM."""
    victim = subprocess.Popen(["sleep", "30"])
    try:
        wd, m = _setup(tmp_path, 5 * GIB, mode="kill")
        os.rename(tmp_path / "proc" / "100", tmp_path / "proc" / str(victim.pid))
        wd.pids = lambda: {victim.pid, 200, 300}
        v = wd.scan()                          # first sighting: confirmed on the next scan
        assert v[0].killed == [] and victim.poll() is None
        v = wd.scan()
        assert v[0].killed == [victim.pid] and m.quota_kills.value() == 1
        victim.wait(timeout=5)
        assert victim.returncode == -9
    finally:
        if victim.poll() is None:
            victim.kill()


def test_cgpu_disable_label_turns_it_off(tmp_path):
    wd, _ = _setup(tmp_path, 5 * GIB)
    wd.disabled = lambda: True
    assert wd.scan() == []


def test_bad_mode_rejected():
    with pytest.raises(ValueError):
        W.QuotaWatchdog(None, None, mode="evict")


def test_kill_mode_spares_a_pod_whose_placement_is_not_settled(tmp_path):
    """after a swapped equal-size admission the pod annotations are crossed until the
    placement patch lands. Kill mode reads the allocator's overlay (the truth already decided)
    and never kills a pod whose placement is still in flight."""
    victim = subprocess.Popen(["sleep", "30"])
    try:
        wd, m = _setup(tmp_path, 5 * GIB, mode="kill")
        os.rename(tmp_path / "proc" / "100", tmp_path / "proc" / str(victim.pid))
        wd.pids = lambda: {victim.pid, 200, 300}
        # pod a really holds an 8 GiB reservation on GPU 1 (the annotations still say 4 GiB):
        # the overlay of the queued placement fix makes the share right, so no violation at all
        wd.view = lambda pods: [p if p["metadata"]["uid"] != UID_A else
                                dict(p, spec={"containers": [{"name": "c", "resources": {"limits": {
                                    const.RESOURCE_NAME: "8"}}}]}) for p in pods]
        assert wd.scan() == [] and wd.scan() == []
        # a pod whose answer / placement patch is still in flight is reported, never killed
        wd.view = lambda pods: pods
        wd.settled = lambda uid: uid != UID_A
        for _ in range(3):
            v = wd.scan()
            assert len(v) == 1 and v[0].killed == []
        assert victim.poll() is None and m.quota_kills.value() == 0
        wd.settled = lambda uid: True          # settled and still over: killed
        assert wd.scan()[0].killed == [victim.pid]
        victim.wait(timeout=5)
    finally:
        if victim.poll() is None:
            victim.kill()
