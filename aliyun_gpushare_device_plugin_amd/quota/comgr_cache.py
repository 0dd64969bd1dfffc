"""The node's trusted comgr cache: a shared pod's HIP runtime loads its blit kernels instead of
compiling them.

A HIP process builds its copy and fill ("blit") kernels with comgr at its first stream: ~56 ms of
``hipStreamCreate`` and ~60 ms of its first kernels on MI355X (``profiles/r5/comgr_cache/``:
140 -> 84 ms and 82 -> 24 ms with comgr's cache). comgr can keep what it built in a directory
(``AMD_COMGR_CACHE=1``, ``AMD_COMGR_CACHE_DIR``), keyed by its inputs and its own version, so a
process whose runtime matches an entry skips the compile.

A cache pods could write would let one pod plant code in every later pod's runtime. So here the
DaemonSet's init container fills it (``gpushare-comgr-cache``: ``warm`` runs the first-stream
work of each HIP runtime the node supports, the system one and the one PyTorch bundles, then
``seal`` makes it read-only), and the plugin (``--comgr-cache-dir``) mounts it read-only into
shared containers with the two variables set (``alloc/engine.py`` ``_container_base``). A
container whose runtime is not in it compiles as it would without the cache (comgr cannot store
the result: the mount is read-only) — a miss costs nothing extra.

comgr's cache holds only the codegen step; the rest of the runtime's compile (OpenCL source to
bitcode with the device libraries, link, link to an executable) still cost a pod ~70 ms of its
first stream. ``libgpushare_comgrcache.so`` (``native/comgrcache``) caches that whole pipeline in
the same directory (``gsa-*`` entries, keyed by the full content of each step's inputs): the fill
runs with it preloaded and ``GPUSHARE_COMGR_ACTION_CACHE_WRITE=1``, pods get it preloaded next to
the shim and only read. A pod's first stream: 84 -> 13 ms (``profiles/r6/first_stream/``).

The reference has nothing here: pod start-up cost is left to the runtime.
"""
from __future__ import annotations

import json
import os
import shutil
import stat
import subprocess
import sys
import time

# the first-stream work of PyTorch's bundled runtime (its own libamdhip64 / libamd_comgr)
_TORCH_WARM = r"""
import json, time, torch
t0 = time.perf_counter()
torch.cuda.init()
t1 = time.perf_counter()
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    x = torch.empty(1 << 20, device="cuda")
    x.zero_()
    x.fill_(1.0)
    y = x.clone()
    h = y.cpu()
    x.copy_(h.cuda(non_blocking=True))
torch.cuda.synchronize()
x.zero_()
torch.cuda.synchronize()
print(json.dumps({"ok": True, "runtime": "torch", "torch": torch.__version__, "hip": torch.version.hip,
                  "init_ms": (t1 - t0) * 1e3, "first_stream_ms": (time.perf_counter() - t1) * 1e3}))
"""

RUNTIMES = ("system", "torch")


ACTION_LIB = "libgpushare_comgrcache.so"


def action_lib() -> str | None:
    """The in-tree action cache library, or None where it was not built (no ROCm clang)."""
    from ..utils.native import NativeUnavailable, ensure_built

    try:
        return ensure_built("comgrcache")
    except NativeUnavailable:
        return None


def cache_env(cache_dir: str, base: dict | None = None, write: bool = False, lib: str | None = None) -> dict:
    """comgr's cache at ``cache_dir``; with ``lib``, the whole-pipeline cache preloaded too
    (``write``: this process fills it)."""
    env = dict(os.environ if base is None else base)
    env["AMD_COMGR_CACHE"] = "1"
    env["AMD_COMGR_CACHE_DIR"] = cache_dir
    if lib:
        env["GPUSHARE_COMGR_ACTION_CACHE"] = cache_dir
        if write:
            env["GPUSHARE_COMGR_ACTION_CACHE_WRITE"] = "1"
        env["LD_PRELOAD"] = ":".join(x for x in (lib, env.get("LD_PRELOAD", "")) if x)
    return env


def entries(cache_dir: str) -> tuple[int, int]:
    """(files, bytes) in the cache."""
    n = b = 0
    for root, _, files in os.walk(cache_dir):
        for f in files:
            try:
                b += os.path.getsize(os.path.join(root, f))
                n += 1
            except OSError:
                pass
    return n, b


def unseal(cache_dir: str) -> None:
    for root, dirs, _ in os.walk(cache_dir):
        os.chmod(root, 0o755)
        for d in dirs:
            os.chmod(os.path.join(root, d), 0o755)


def seal(cache_dir: str) -> None:
    """Read-only for everyone (files 0444, directories 0555); the mount into pods is read-only
    too, so neither a pod nor a process on the host with another uid can change an entry."""
    for root, dirs, files in os.walk(cache_dir, topdown=False):
        for f in files:
            os.chmod(os.path.join(root, f), stat.S_IRUSR | stat.S_IRGRP | stat.S_IROTH)
        for d in dirs:
            os.chmod(os.path.join(root, d), 0o555)
    os.chmod(cache_dir, 0o555)


def warm(cache_dir: str, runtimes=RUNTIMES, device: int = 0, timeout: float = 300.0, fresh: bool = True,
         actions: bool = True) -> dict:
    """Fill ``cache_dir`` with what each runtime in ``runtimes`` builds at its first stream;
    returns per-runtime results and the cache's size. ``fresh``: start from an empty cache (a
    DaemonSet restart after a ROCm upgrade drops entries no runtime on the node makes any more).
    ``actions``: fill the whole-pipeline cache too (when its library is built)."""
    if fresh and os.path.isdir(cache_dir):
        unseal(cache_dir)
        for e in os.listdir(cache_dir):
            p = os.path.join(cache_dir, e)
            shutil.rmtree(p) if os.path.isdir(p) and not os.path.islink(p) else os.unlink(p)
    os.makedirs(cache_dir, exist_ok=True)
    unseal(cache_dir)
    lib = action_lib() if actions else None
    env = cache_env(cache_dir, write=True, lib=lib)
    out: dict = {"dir": cache_dir, "runtimes": {}, "action_cache": bool(lib)}
    for rt in runtimes:
        t0 = time.perf_counter()
        if rt == "system":
            from ..utils.native import ensure_built

            cmd = [ensure_built("comgrwarm"), str(device)]
        elif rt == "torch":
            import importlib.util

            if importlib.util.find_spec("torch") is None:
                out["runtimes"][rt] = {"ok": False, "skipped": "PyTorch is not installed here"}
                continue
            cmd = [sys.executable, "-c", _TORCH_WARM]
        else:
            raise ValueError(f"unknown runtime {rt!r} (one of {', '.join(RUNTIMES)})")
        try:
            r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
            line = (r.stdout.strip().splitlines() or ["{}"])[-1]
            res = json.loads(line) if line.startswith("{") else {"ok": False}
            if r.returncode != 0:
                res = dict(res, ok=False, rc=r.returncode, stderr=r.stderr[-1000:])
        except (OSError, subprocess.TimeoutExpired, ValueError) as e:
            res = {"ok": False, "error": f"{type(e).__name__}: {e}"[:500]}
        res["wall_ms"] = round((time.perf_counter() - t0) * 1e3, 1)
        out["runtimes"][rt] = res
    out["files"], out["bytes"] = entries(cache_dir)
    out["action_entries"] = sum(1 for f in os.listdir(cache_dir) if f.startswith("gsa-"))
    return out
