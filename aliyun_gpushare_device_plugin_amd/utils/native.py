"""Locating (and, if needed, building) the in-tree native libraries.

All native artefacts live in ``<package>/_native`` so that they travel with the repository
snapshot to the GPU box and are visibly loaded from the tree (never from a JIT cache).
A missing library is an error, not a silent fallback: callers get ``NativeUnavailable``.
"""
from __future__ import annotations

import os
import subprocess
import sys
import threading

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE_DIR = os.path.join(PKG_DIR, "_native")
REPO_ROOT = os.path.dirname(PKG_DIR)
BUILD_SCRIPT = os.path.join(REPO_ROOT, "native", "build.py")

LIBS = {
    "gpuinfo": "libgpushare_gpuinfo.so",
    "hipshim": "libgpushare_hipquota.so",
    "dpserver": "libgpushare_dpserver.so",
    "kernels": "libgpushare_kernels.so",
    "hbmbroker": "gpushare-hbm-broker",
    "comgrwarm": "gpushare-comgr-warm",
    "comgrcache": "libgpushare_comgrcache.so",
    "comgrprobe": "gpushare-comgr-probe",
}

_lock = threading.Lock()


class NativeUnavailable(RuntimeError):
    pass


def preload(*libs: str) -> str:
    """LD_PRELOAD for a child process: ``libs`` first, then whatever this process already
    preloads (a profiler, the host's own libraries), which the child keeps."""
    return ":".join(x for x in (*libs, os.environ.get("LD_PRELOAD", "")) if x)


def lib_path(target: str) -> str:
    """``GPUSHARE_NATIVE_VARIANT=asan|tsan`` selects a sanitizer build (native/build.py
    --sanitize) from ``_native/<variant>/``; the matching runtime must be LD_PRELOADed."""
    variant = os.environ.get("GPUSHARE_NATIVE_VARIANT", "")
    if variant:
        return os.path.join(NATIVE_DIR, variant, LIBS[target])
    return os.path.join(NATIVE_DIR, LIBS[target])


SOURCES = {"gpuinfo": "gpuinfo", "hipshim": "hipshim", "dpserver": "dpserver", "kernels": "kernels",
           "hbmbroker": "hbmbroker", "comgrwarm": "comgrwarm", "comgrcache": "comgrcache",
           "comgrprobe": "comgrcache"}   # native/<dir>
BUILD_TARGET = {"comgrprobe": "comgrcache"}     # built by another target of native/build.py


def stale(target: str, path: str) -> bool:
    """The library is older than a source file of its ``native/<dir>`` (a test must never run
    a build of code that has since changed)."""
    src = os.path.join(REPO_ROOT, "native", SOURCES[target])
    try:
        built = os.path.getmtime(path)
        return any(os.path.getmtime(os.path.join(src, f)) > built for f in os.listdir(src)
                   if f.endswith((".c", ".cpp", ".h", ".hip", ".hpp")))
    except OSError:
        return False


def ensure_built(target: str, auto_build: bool | None = None) -> str:
    """Return the path of a native library, building it in-tree when it is missing or older
    than its sources.

    ``auto_build`` defaults to on unless ``GPUSHARE_NO_AUTOBUILD=1``.
    """
    path = lib_path(target)
    if auto_build is None:
        auto_build = os.environ.get("GPUSHARE_NO_AUTOBUILD", "") != "1"
    if os.path.exists(path) and not (auto_build and stale(target, path)):
        return path
    if auto_build and os.path.exists(BUILD_SCRIPT):
        with _lock:
            if not os.path.exists(path) or stale(target, path):
                variant = os.environ.get("GPUSHARE_NATIVE_VARIANT", "")
                extra = ["--sanitize", variant] if variant else []
                r = subprocess.run([sys.executable, BUILD_SCRIPT, BUILD_TARGET.get(target, target), *extra],
                                   capture_output=True, text=True)
                if r.returncode != 0:
                    raise NativeUnavailable(f"building {target} failed:\n{r.stdout}\n{r.stderr}")
    if not os.path.exists(path):
        raise NativeUnavailable(f"{LIBS[target]} not found in {NATIVE_DIR}; run `python native/build.py {target}`")
    return path
