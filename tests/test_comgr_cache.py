"""The node's trusted comgr cache (quota/comgr_cache.py, cli/comgrcache.py).

CPU: the Allocate answer mounts the sealed cache read-only with comgr's two variables (and
nothing on a cgpu-disabled node), sealing makes every entry read-only, a fill without a GPU
still seals and exits 0, and the DaemonSet fills it in an init container before the plugin
mounts it. GPU: a filled cache (comgr's own plus the whole-pipeline one,
tests/test_comgr_action_cache.py) takes the runtime's blit-kernel compile off a process's first
stream, a pod cannot write it, and a runtime it does not hold still starts (a miss compiles)."""
import json
import os
import stat
import subprocess
import sys

import pytest
import yaml

from aliyun_gpushare_device_plugin_amd import const
from aliyun_gpushare_device_plugin_amd.alloc.engine import Allocator, AllocatorOptions
from aliyun_gpushare_device_plugin_amd.device.model import DeviceModel
from aliyun_gpushare_device_plugin_amd.quota import ShimConfig, comgr_cache

from .test_allocate_engine import NODE, FakeClient, StaticSource, mkpod
from .test_units_and_model import gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _answer(tmp_path, **opts):
    model = DeviceModel([gpu(0, 64 << 30)], const.GIB)
    src = StaticSource([mkpod("c", 16, 0, 10)])
    al = Allocator(model, src, FakeClient(src), NODE,
                   AllocatorOptions(shim=ShimConfig(host_dir=str(tmp_path / "shim")), **opts))
    try:
        return al._container_response(0, 16, 16, "uid-c", 0, None)
    finally:
        al.close()


def test_the_answer_mounts_the_cache_read_only(tmp_path):
    cache = tmp_path / "comgr-cache"
    cache.mkdir()
    r = _answer(tmp_path, comgr_cache_dir=str(cache))
    m = [x for x in r.mounts if x.container_path == const.COMGR_CACHE_CONTAINER_DIR]
    assert len(m) == 1 and m[0].host_path == str(cache) and m[0].read_only
    assert r.envs[const.ENV_COMGR_CACHE] == "1"
    assert r.envs[const.ENV_COMGR_CACHE_DIR] == const.COMGR_CACHE_CONTAINER_DIR
    # the whole-pipeline cache: preloaded after the shim when it is installed next to it
    assert const.ENV_COMGR_ACTION_CACHE not in r.envs
    assert r.envs[const.ENV_LD_PRELOAD] == os.path.join(const.SHIM_CONTAINER_DIR, const.SHIM_LIB_NAME)
    (tmp_path / "shim").mkdir()
    (tmp_path / "shim" / const.COMGR_ACTION_LIB_NAME).write_bytes(b"")
    r = _answer(tmp_path, comgr_cache_dir=str(cache))
    assert r.envs[const.ENV_COMGR_ACTION_CACHE] == const.COMGR_CACHE_CONTAINER_DIR
    assert r.envs[const.ENV_LD_PRELOAD].split(":") == [
        os.path.join(const.SHIM_CONTAINER_DIR, n) for n in (const.SHIM_LIB_NAME, const.COMGR_ACTION_LIB_NAME)]
    assert const.ENV_COMGR_ACTION_CACHE not in _answer(tmp_path).envs
    # off unless configured, off on a cgpu-disabled node (its pods get nothing of the plugin's), and
    # off while the directory is not there (a hostPath mount of a missing path fails the container)
    for r in (_answer(tmp_path), _answer(tmp_path, comgr_cache_dir=str(cache), disable_cgpu=True),
              _answer(tmp_path, comgr_cache_dir=str(tmp_path / "missing"))):
        assert const.ENV_COMGR_CACHE not in r.envs
        assert not any(x.container_path == const.COMGR_CACHE_CONTAINER_DIR for x in r.mounts)


def test_seal_makes_every_entry_read_only_and_a_fresh_fill_starts_empty(tmp_path):
    d = tmp_path / "cc"
    (d / "sub").mkdir(parents=True)
    (d / "sub" / "entry").write_bytes(b"x" * 10)
    comgr_cache.seal(str(d))
    for root, dirs, files in os.walk(d):
        assert stat.S_IMODE(os.stat(root).st_mode) == 0o555
        for f in files:
            assert stat.S_IMODE(os.stat(os.path.join(root, f)).st_mode) == 0o444
    assert comgr_cache.entries(str(d)) == (1, 10)
    # no GPU here: every runtime fails to warm, the old entries are gone and the cache is sealed
    r = subprocess.run([sys.executable, "-m", "aliyun_gpushare_device_plugin_amd.cli.comgrcache", "--dir", str(d),
                        "--runtimes", "system"], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, PYTHONPATH=ROOT, HIP_VISIBLE_DEVICES="-1"))
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["sealed"] and out["files"] == 0 and not out["runtimes"]["system"]["ok"]
    assert stat.S_IMODE(os.stat(d).st_mode) == 0o555 and os.listdir(d) == []


def test_the_daemonset_fills_the_cache_before_the_plugin_mounts_it():
    with open(os.path.join(ROOT, "deploy", "device-plugin-ds.yaml")) as f:
        ds = next(d for d in yaml.safe_load_all(f) if d and d.get("kind") == "DaemonSet")
    spec = ds["spec"]["template"]["spec"]
    init = next(c for c in spec["initContainers"] if c["name"] == "comgr-cache")
    assert init["command"][0] == "gpushare-comgr-cache"
    cache = next(a.split("=", 1)[1] for a in init["command"] if a.startswith("--dir="))
    plugin = next(c for c in spec["containers"] if c["name"] == "gpushare")
    assert f"--comgr-cache-dir={cache}" in plugin["command"]
    # the same host directory in both (the gpushare-lib hostPath)
    mount = {m["mountPath"]: m["name"] for m in init["volumeMounts"]}
    assert any(cache.startswith(p) for p in mount) and all(m in {v["name"] for v in spec["volumes"]}
                                                          for m in mount.values())


# ---- on the GPU ----------------------------------------------------------------------------
POD = r"""
import json, os, sys, time
import torch
torch.cuda.init()
t0 = time.perf_counter()
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    x = torch.empty(1 << 20, device="cuda")
    x.zero_()
    x.fill_(2.0)
    y = x.cpu()
torch.cuda.synchronize()
ms = (time.perf_counter() - t0) * 1e3
write = None
d = os.environ.get("AMD_COMGR_CACHE_DIR")
if d:
    try:
        with open(os.path.join(d, "planted"), "w") as f:
            f.write("x")
        write = "allowed"
    except OSError:
        write = "denied"
try:                                   # the whole-pipeline cache's counters, when it is preloaded
    import ctypes
    a = (ctypes.c_uint64 * 5)()
    ctypes.CDLL(None).gpushare_comgr_cache_stats(a, 5)
    actions = dict(zip(("hits", "misses", "stores", "bypassed", "errors"), a))
except AttributeError:
    actions = None
print(json.dumps({"first_stream_ms": ms, "ok": float(y.sum()) == 2.0 * (1 << 20), "write": write, "actions": actions}))
"""


def _pod(cache_dir):
    import tempfile

    # a fresh container: comgr's own default cache ($XDG_CACHE_HOME/comgr) starts empty
    env = dict(os.environ, XDG_CACHE_HOME=tempfile.mkdtemp(prefix="pod-home-"))
    env.pop("AMD_COMGR_CACHE", None)
    env.pop("AMD_COMGR_CACHE_DIR", None)
    if cache_dir:
        env = comgr_cache.cache_env(cache_dir, env, lib=comgr_cache.action_lib())
    r = subprocess.run([sys.executable, "-c", POD], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def _snapshot(d):
    return {os.path.relpath(os.path.join(r, f), d): os.path.getsize(os.path.join(r, f))
            for r, _, fs in os.walk(d) for f in fs}


@pytest.mark.gpu
def test_a_pod_loads_its_blit_kernels_from_the_sealed_cache_and_cannot_write_it(tmp_path):
    d = str(tmp_path / "cc")
    w = comgr_cache.warm(d, ("system", "torch"))
    comgr_cache.seal(d)
    assert w["runtimes"]["system"]["ok"] and w["runtimes"]["torch"]["ok"] and w["files"] > 0, w
    before = _snapshot(d)
    plain = [_pod(None) for _ in range(2)]
    cached = [_pod(d) for _ in range(2)]
    # a miss falls through: a sealed cache holding nothing, the runtime compiles as without one
    empty = str(tmp_path / "empty")
    os.makedirs(empty)
    comgr_cache.seal(empty)
    miss = _pod(empty)
    res = {"cache": {"files": w["files"], "bytes": w["bytes"]}, "plain_ms": [p["first_stream_ms"] for p in plain],
           "cached_ms": [c["first_stream_ms"] for c in cached], "miss_ms": miss["first_stream_ms"],
           "write": [c["write"] for c in cached], "actions": [c["actions"] for c in cached],
           "action_entries": w["action_entries"]}
    print(json.dumps(res))
    assert all(p["ok"] for p in plain + cached) and miss["ok"]
    assert _snapshot(d) == before and os.listdir(empty) == []
    if os.geteuid() != 0:                    # (root ignores the mode bits; a container's mount is read-only)
        assert all(c["write"] == "denied" for c in cached) and miss["write"] == "denied"
    # every step of the runtime's compile from the cache (none compiled, none stored): the first
    # stream keeps only the runtime's own queue and code-object set-up
    assert w["action_entries"] >= 4 and all(c["actions"]["hits"] >= 4 and not c["actions"]["misses"]
                                             and not c["actions"]["stores"] for c in cached), res
    assert min(c["first_stream_ms"] for c in cached) + 80.0 < min(p["first_stream_ms"] for p in plain), res
