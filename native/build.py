#!/usr/bin/env python3
"""Build every native component in-tree (outputs under the package's ``_native/`` dir).

Targets
  gpuinfo   libgpushare_gpuinfo.so + gpushare-smi (C++17, host only; librocm_smi64 is dlopen'ed)
  hipshim   libgpushare_hipquota.so  (C++17 LD_PRELOAD interposer over the HIP allocation API)
  dpserver  libgpushare_dpserver.so  (C++17 DevicePlugin gRPC server over libnghttp2, native Allocate fast path)
  hbmbroker gpushare-hbm-broker     (C++17 per-GPU HBM broker daemon over HIP VMM, host only)
  kernels   libgpushare_kernels.so   (hand-written HIP/CDNA4 kernels, hipcc --offload-arch=gfx950)
  probes    shim_probe               (HIP test helper run under the quota shim on hardware)
  comgrwarm gpushare-comgr-warm      (the system HIP runtime's first-stream work: fills the node's comgr cache)
  comgrcache libgpushare_comgrcache.so (clang: action cache in front of comgr, preloaded into pods) + gpushare-comgr-probe

Usage: python native/build.py [targets...] [--force] [--asan | --sanitize {asan,tsan}] [-j N]
The build is incremental (mtime based) so ``__graft_entry__.build()`` stays cheap.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shlex
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
OUT = os.path.join(ROOT, "aliyun_gpushare_device_plugin_amd", "_native")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")

CXX = shutil.which("g++") or "g++"
HIPCC = os.path.join(ROCM, "bin", "hipcc") if os.path.exists(os.path.join(ROCM, "bin", "hipcc")) else "hipcc"


def _src(*p):
    return os.path.join(HERE, *p)


def _newer(out, deps):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _run(cmd, verbose=True):
    if verbose:
        print("+", " ".join(shlex.quote(c) for c in cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise SystemExit(f"native build failed: {cmd[0]} exited {r.returncode}")
    return r


def _headers(d):
    return [os.path.join(d, f) for f in os.listdir(d) if f.endswith((".h", ".hpp", ".inc"))]


SANITIZERS = {
    # host-side only (GPU ASan / XNACK are not available on the pool)
    "asan": ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-O1"],
    "tsan": ["-fsanitize=thread", "-fno-omit-frame-pointer", "-O1"],
}


def _san(asan):
    """``asan`` is False/None, True (= "asan") or a SANITIZERS key."""
    if not asan:
        return None
    return "asan" if asan is True else asan


def build_gpuinfo(force=False, asan=False):
    d = _src("gpuinfo")
    lib = os.path.join(OUT, "libgpushare_gpuinfo.so")
    deps = [_src("gpuinfo", "gpuinfo.cpp")] + _headers(d)
    flags = ["-std=c++17", "-O2", "-fPIC", "-Wall", "-Wextra", "-Wno-unused-parameter", f"-I{d}"]
    san = _san(asan)
    if san:
        flags += SANITIZERS[san]
        lib = os.path.join(OUT, san, "libgpushare_gpuinfo.so")
    os.makedirs(os.path.dirname(lib), exist_ok=True)
    if force or _newer(lib, deps):
        _run([CXX, *flags, "-shared", "-o", lib, _src("gpuinfo", "gpuinfo.cpp"), "-ldl", "-pthread"])
    cli = os.path.join(os.path.dirname(lib), "gpushare-smi")
    if force or _newer(cli, [_src("gpuinfo", "smi_cli.cpp"), lib]):
        _run([CXX, *flags, "-o", cli, _src("gpuinfo", "smi_cli.cpp"), f"-L{os.path.dirname(lib)}",
              "-lgpushare_gpuinfo", "-Wl,-rpath,$ORIGIN", "-ldl", "-pthread"])
    return [lib, cli]


def hipshim_sources():
    """The quota shim's translation units (native/hipshim/shim.h lists what each one owns)."""
    d = _src("hipshim")
    return sorted(os.path.join(d, f) for f in os.listdir(d) if f.endswith(".cpp")) if os.path.isdir(d) else []


def build_hipshim(force=False, asan=False):
    d = _src("hipshim")
    srcs = hipshim_sources()
    if not srcs:
        return []
    lib = os.path.join(OUT, "libgpushare_hipquota.so")
    flags = ["-std=c++17", "-O2", "-fPIC", "-Wall", "-Wextra", "-Wno-unused-parameter",
             "-D__HIP_PLATFORM_AMD__", f"-I{ROCM}/include", f"-I{d}", "-fvisibility=hidden"]
    san = _san(asan)
    if san:
        flags += SANITIZERS[san]
        lib = os.path.join(OUT, san, "libgpushare_hipquota.so")
    os.makedirs(os.path.dirname(lib), exist_ok=True)
    if force or _newer(lib, srcs + _headers(d)):
        # Deliberately NOT linked against libamdhip64: the real entry points are resolved at
        # run time from whichever HIP runtime the process loaded (PyTorch bundles its own).
        # -static-libstdc++/-static-libgcc: the shim is preloaded into arbitrary tenant images,
        # whose libstdc++ may be older than ours (or absent); only glibc stays dynamic.
        # The shim uses no libstdc++ runtime at all (checked by tests/test_hipquota_shim.py) and
        # pins its glibc symbol versions to the 2.2.5 baseline; libdl/librt/libpthread stay
        # NEEDED for images whose glibc predates their merge into libc (2.34).
        static = [] if san else ["-static-libstdc++", "-static-libgcc", "-fno-exceptions", "-fno-rtti"]
        _run([CXX, *flags, "-shared", "-o", lib, *srcs, *static, "-Wl,--no-as-needed", "-l:libdl.so.2", "-l:librt.so.1",
              "-l:libpthread.so.0", "-Wl,--as-needed"])
    return [lib]


def _nghttp2_include():
    """Directory holding nghttp2/nghttp2.h (the dev headers, or the copy a Python distribution
    ships); the library itself is the system's libnghttp2.so.14."""
    for d in (os.environ.get("NGHTTP2_INCLUDE", ""), "/usr/include", "/usr/local/include", "/opt/conda/include"):
        if d and os.path.exists(os.path.join(d, "nghttp2", "nghttp2.h")):
            return d
    return None


def build_dpserver(force=False, asan=False):
    """libgpushare_dpserver.so: the DevicePlugin gRPC server with the native Allocate fast path
    (C++17 over libnghttp2)."""
    d = _src("dpserver")
    src = _src("dpserver", "dpserver.cpp")
    inc = _nghttp2_include()
    if not os.path.exists(src):
        return []
    if inc is None:
        print("dpserver: nghttp2/nghttp2.h not found (set NGHTTP2_INCLUDE); skipped", flush=True)
        return []
    lib = os.path.join(OUT, "libgpushare_dpserver.so")
    flags = ["-std=c++17", "-O2", "-fPIC", "-Wall", "-Wextra", "-Wno-unused-parameter", f"-I{d}",
             f"-I{inc}", "-fvisibility=hidden", "-fvisibility-inlines-hidden"]
    san = _san(asan)
    if san:
        flags += SANITIZERS[san]
        lib = os.path.join(OUT, san, "libgpushare_dpserver.so")
    os.makedirs(os.path.dirname(lib), exist_ok=True)
    srcs = [src, _src("dpserver", "h2client.cpp")]
    if force or _newer(lib, srcs + _headers(d)):
        _run([CXX, *flags, "-shared", "-o", lib, *srcs, "-l:libnghttp2.so.14", "-pthread"])
    return [lib]


def build_hbmbroker(force=False, asan=False):
    """gpushare-hbm-broker: lends each pod VMM granules of HBM it holds, scrubbed between pods
    (docs/HBM_TURNOVER.md). Host code built by g++; its scrub kernel (scrub.hip) is a gfx950 code
    object it loads at start."""
    src = _src("hbmbroker", "hbmbroker.cpp")
    if not os.path.exists(src):
        return []
    exe = os.path.join(OUT, "gpushare-hbm-broker")
    flags = ["-std=c++17", "-O2", "-Wall", "-Wextra", "-Wno-unused-parameter", "-D__HIP_PLATFORM_AMD__",
             f"-I{ROCM}/include"]
    san = _san(asan)
    if san:
        flags += SANITIZERS[san]
        exe = os.path.join(OUT, san, "gpushare-hbm-broker")
    os.makedirs(os.path.dirname(exe), exist_ok=True)
    if force or _newer(exe, [src]):
        _run([CXX, *flags, "-o", exe, src, f"-L{ROCM}/lib", "-lamdhip64", f"-Wl,-rpath,{ROCM}/lib", "-pthread"])
    # its scrub kernel: a gfx950 code object next to the executable, loaded with hipModuleLoad
    ksrc = _src("hbmbroker", "scrub.hip")
    co = os.path.join(os.path.dirname(exe), "gpushare-hbm-scrub.co")
    if os.path.exists(ksrc) and (force or _newer(co, [ksrc])):
        _run([HIPCC, "--genco", f"--offload-arch={ARCH}", "-O3", "-o", co, ksrc])
    return [exe, co] if os.path.exists(ksrc) else [exe]


def build_kernels(force=False, asan=False, jobs=4):
    d = _src("kernels")
    srcs = sorted(os.path.join(d, f) for f in os.listdir(d) if f.endswith(".hip")) if os.path.isdir(d) else []
    if not srcs:
        return []
    lib = os.path.join(OUT, "libgpushare_kernels.so")
    objdir = os.path.join(OUT, "obj")
    os.makedirs(objdir, exist_ok=True)
    hdrs = _headers(d)
    flags = ["-std=c++17", "-O3", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
             "-Wno-unused-result", f"-I{d}", "-D__HIP_PLATFORM_AMD__"]
    if _san(asan) == "asan":  # host-side sanitizers only; GPU ASan is not available on the pool
        flags += ["-Xarch_host", "-fsanitize=address", "-fno-omit-frame-pointer"]
    objs, todo = [], []
    for s in srcs:
        o = os.path.join(objdir, os.path.basename(s)[:-4] + ".o")
        objs.append(o)
        if force or _newer(o, [s] + hdrs):
            todo.append([HIPCC, *flags, "-c", s, "-o", o])
    with cf.ThreadPoolExecutor(max(1, jobs)) as ex:
        list(ex.map(_run, todo))
    if force or todo or _newer(lib, objs):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-o", lib, *objs])
    return [lib]


def build_probes(force=False, asan=False):
    """On-hardware test helpers (native/probes/*.hip): standalone HIP programs the GPU tests run
    under the quota shim (a plain executable, so LD_PRELOAD applies exactly as in a container)."""
    d = _src("probes")
    out = []
    if asan or not os.path.isdir(d):
        return out
    for f in sorted(os.listdir(d)):
        if not f.endswith(".hip"):
            continue
        exe = os.path.join(OUT, os.path.splitext(f)[0])
        if force or _newer(exe, [os.path.join(d, f)]):
            _run([HIPCC, "-std=c++17", "-O2", f"--offload-arch={ARCH}", "-o", exe, os.path.join(d, f), "-ldl"])
        out.append(exe)
    return out


def build_comgrwarm(force=False, asan=False):
    """gpushare-comgr-warm (native/comgrwarm): the first-stream work of a HIP process against the
    system runtime, run by the DaemonSet's init container to fill the node's comgr cache."""
    src = os.path.join(_src("comgrwarm"), "comgr_warm.cpp")
    exe = os.path.join(OUT, "gpushare-comgr-warm")
    if asan or not os.path.isfile(src):
        return []
    if force or _newer(exe, [src]):
        _run([HIPCC, "-std=c++17", "-O2", f"--offload-arch={ARCH}", "-o", exe, src])
    return [exe]


def build_comgrcache(force=False, asan=False):
    """libgpushare_comgrcache.so (native/comgrcache): the whole-pipeline cache in front of comgr
    that shared pods preload. Built with ROCm's clang: its dlsym must tail-call the C library's
    (``__attribute__((musttail))``, which g++ 11 lacks). gpushare-comgr-probe: the runtime's blit
    compile without a GPU (tests)."""
    d = _src("comgrcache")
    if not os.path.isdir(d):
        return []
    clang = os.path.join(ROCM, "llvm", "bin", "clang")
    lib = os.path.join(OUT, "libgpushare_comgrcache.so")
    srcs = [os.path.join(d, "comgr_dlsym.c"), os.path.join(d, "comgr_action_cache.cpp")]
    san = _san(asan)
    flags = ["-O2", "-fPIC", "-fvisibility=hidden", "-Wall", "-Wextra", f"-I{ROCM}/include"]
    if san:
        flags += SANITIZERS[san]
        lib = os.path.join(OUT, san, "libgpushare_comgrcache.so")
    os.makedirs(os.path.dirname(lib), exist_ok=True)
    if force or _newer(lib, srcs):
        import tempfile
        with tempfile.TemporaryDirectory() as tmp:
            objs = [os.path.join(tmp, "dlsym.o"), os.path.join(tmp, "cache.o")]
            # the dlsym thunk is never instrumented: a sanitizer runtime calls dlsym while it starts
            _run([clang, *[f for f in flags if f not in SANITIZERS.get(san or "", [])], "-c", "-o", objs[0], srcs[0]])
            _run([clang + "++", *flags, "-std=c++17", "-c", "-o", objs[1], srcs[1]])
            _run([clang + "++", *flags, "-shared", "-o", lib, *objs, "-ldl"])
    probe = os.path.join(os.path.dirname(lib), "gpushare-comgr-probe")
    psrc = os.path.join(d, "comgr_probe.cpp")
    if force or _newer(probe, [psrc]):
        _run([CXX, "-std=c++17", "-O2", "-Wall", f"-I{ROCM}/include", "-o", probe, psrc, "-ldl"])
    return [lib, probe]


TARGETS = {"gpuinfo": build_gpuinfo, "hipshim": build_hipshim, "dpserver": build_dpserver,
           "hbmbroker": build_hbmbroker, "kernels": build_kernels,
           "probes": build_probes, "comgrwarm": build_comgrwarm, "comgrcache": build_comgrcache}


def build(targets=None, force=False, asan=False, jobs=4):
    os.makedirs(OUT, exist_ok=True)
    built = []
    for t in targets or list(TARGETS):
        fn = TARGETS[t]
        built += fn(force=force, asan=asan, jobs=jobs) if t == "kernels" else fn(force=force, asan=asan)
    return built


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("targets", nargs="*", choices=[[], *TARGETS], default=None)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--asan", action="store_true", help="host-side ASan/UBSan variants under _native/asan")
    ap.add_argument("--sanitize", choices=sorted(SANITIZERS), default=None,
                    help="host-side sanitizer variant under _native/<name> (asan = ASan+UBSan, tsan = TSan)")
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 4))
    a = ap.parse_args(argv)
    for p in build(a.targets or None, a.force, a.sanitize or a.asan, a.jobs):
        print("built", os.path.relpath(p, ROOT))


if __name__ == "__main__":
    main()
