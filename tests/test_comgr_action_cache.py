"""The whole-pipeline cache in front of comgr (native/comgrcache, libgpushare_comgrcache.so).

comgr compiles on the CPU, so all of this runs here: ``gpushare-comgr-probe`` does the compile a
HIP runtime does for its blit kernels at a process's first stream (OpenCL source -> bitcode with
the device libraries -> link -> codegen -> executable for gfx950), loading comgr the way the
runtime does (dlopen + dlsym). Pinned: a fill stores every step, a reader gets byte-identical
executables from the cache without compiling and never writes, a corrupt entry falls through to
the real compile, the library is inert without its variable, and its dlsym keeps RTLD_NEXT
relative to the real caller (a tail call). On the GPU: tests/test_comgr_cache.py."""
import json
import os
import subprocess

import pytest

from aliyun_gpushare_device_plugin_amd.utils.native import NativeUnavailable, ensure_built

try:
    LIB = ensure_built("comgrcache")
    PROBE = ensure_built("comgrprobe")
except NativeUnavailable as e:   # no ROCm clang / comgr in this environment
    pytest.skip(f"comgr action cache not built: {e}", allow_module_level=True)


def _probe(cache=None, write=False, preload=True, variant="", logging=True, extra=None):
    env = {k: v for k, v in os.environ.items() if not k.startswith(("GPUSHARE_COMGR", "AMD_COMGR"))}
    if preload:
        env["LD_PRELOAD"] = LIB
    if cache is not None:
        env["GPUSHARE_COMGR_ACTION_CACHE"] = str(cache)
        env["GPUSHARE_COMGR_ACTION_CACHE_LOG"] = "1"
        if write:
            env["GPUSHARE_COMGR_ACTION_CACHE_WRITE"] = "1"
    env.update(extra or {})
    r = subprocess.run([PROBE, variant, "1" if logging else "0"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["ok"], out
    # "gpushare-comgr: action <kind> hit|miss <key> <ms> ms"
    out["log"] = [ln.split()[2:5] for ln in r.stderr.splitlines() if ln.startswith("gpushare-comgr: action")]
    return out


def _entries(d):
    return sorted(f for f in os.listdir(d) if f.startswith("gsa-"))


def test_a_fill_stores_every_step_and_a_reader_gets_the_same_executable_without_compiling(tmp_path):
    base = _probe(preload=False)
    assert base["cache"] is None
    d = tmp_path / "cache"
    d.mkdir()
    fill = _probe(d, write=True)
    assert fill["exe_digest"] == base["exe_digest"]
    assert fill["cache"] == {"hits": 0, "misses": 4, "stores": 4, "bypassed": 0, "errors": 0}
    assert len(_entries(d)) == 4 and not [f for f in os.listdir(d) if f.startswith(".gsa-tmp")]
    before = {f: os.path.getsize(d / f) for f in os.listdir(d)}
    for logging in (True, False):          # the runtime asks for logs; the key does not depend on them
        hit = _probe(d, logging=logging)
        assert hit["exe_digest"] == base["exe_digest"] and hit["exe_bytes"] == base["exe_bytes"]
        assert hit["cache"] == {"hits": 4, "misses": 0, "stores": 0, "bypassed": 0, "errors": 0}, hit
        assert [x[1] for x in hit["log"]] == ["hit"] * 4
    # a reader never writes, even a miss (another source) in a writable directory
    other = _probe(d, variant="another kernel set")      # (its bitcode is the same: later steps hit)
    assert other["cache"]["misses"] >= 1 and other["cache"]["stores"] == 0
    assert other["log"][0][:2] == ["12", "miss"]
    assert {f: os.path.getsize(d / f) for f in os.listdir(d)} == before
    # the compile itself (not the whole probe): milliseconds of LLVM against a file read
    assert hit["total_ms"] < base["total_ms"], (hit, base)


def test_a_corrupt_entry_falls_through_to_the_real_compile(tmp_path):
    d = tmp_path / "cache"
    d.mkdir()
    fill = _probe(d, write=True)
    last = fill["log"][-1]                  # the final link step: [kind, "miss", key]
    assert last[0] == "7"
    p = d / f"gsa-{last[2]}"
    b = bytearray(p.read_bytes())
    b[len(b) // 2] ^= 0xFF                  # checksum mismatch
    p.write_bytes(bytes(b))
    r = _probe(d)
    assert r["exe_digest"] == fill["exe_digest"]
    assert r["cache"]["hits"] == 3 and r["cache"]["misses"] == 1, r
    p.write_bytes(bytes(b[:40]))            # truncated
    assert _probe(d)["exe_digest"] == fill["exe_digest"]


def test_the_library_is_inert_without_its_variable_or_under_comgr_debugging(tmp_path):
    off = _probe(None)
    assert off["cache"] == {"hits": 0, "misses": 0, "stores": 0, "bypassed": 0, "errors": 0}
    d = tmp_path / "cache"
    d.mkdir()
    _probe(d, write=True)
    dbg = _probe(d, extra={"AMD_COMGR_EMIT_VERBOSE_LOGS": "1", "AMD_COMGR_REDIRECT_LOGS": "/dev/null"})
    assert dbg["cache"]["hits"] == 0 and dbg["exe_digest"] == off["exe_digest"]


NEXT_MAIN = r"""
#include <dlfcn.h>
#include <stdio.h>
void* gs_lookup_next(void);   /* in libgs_y.so */
int main(void) {
  void* p = gs_lookup_next();
  printf("%s\n", p ? "found" : "none");
  return 0;
}
"""
NEXT_X = "int gs_marker(void) { return 1; }\n"
NEXT_Y = r"""
#define _GNU_SOURCE
#include <dlfcn.h>
void* gs_lookup_next(void) { return dlsym(RTLD_NEXT, "gs_marker"); }
"""


def test_dlsym_keeps_rtld_next_relative_to_the_real_caller(tmp_path):
    """Preloaded in the order comgr-cache, X, Y: Y's dlsym(RTLD_NEXT, "gs_marker") must search
    after Y (nothing there defines it). Had the interposer called the C library's dlsym instead
    of jumping to it, the caller would be the comgr-cache library and X's gs_marker would come
    back."""
    for name, src in (("x", NEXT_X), ("y", NEXT_Y)):
        (tmp_path / f"{name}.c").write_text(src)
        subprocess.run(["gcc", "-shared", "-fPIC", "-o", str(tmp_path / f"libgs_{name}.so"), str(tmp_path / f"{name}.c"),
                        "-ldl"], check=True)
    (tmp_path / "main.c").write_text(NEXT_MAIN)
    exe = tmp_path / "main"
    subprocess.run(["gcc", "-o", str(exe), str(tmp_path / "main.c"), f"-L{tmp_path}", "-lgs_y",
                    f"-Wl,-rpath,{tmp_path}", "-ldl"], check=True)
    pre = ":".join([LIB, str(tmp_path / "libgs_x.so"), str(tmp_path / "libgs_y.so")])
    plain = subprocess.run([str(exe)], capture_output=True, text=True, check=True,
                           env=dict(os.environ, LD_PRELOAD=":".join(pre.split(":")[1:])))
    shimmed = subprocess.run([str(exe)], capture_output=True, text=True, check=True,
                             env=dict(os.environ, LD_PRELOAD=pre, GPUSHARE_COMGR_ACTION_CACHE=str(tmp_path)))
    assert plain.stdout.strip() == "none"
    assert shimmed.stdout.strip() == "none"


def test_the_cache_under_address_and_ub_sanitizers(tmp_path):
    """The library built with -fsanitize=address,undefined (its dlsym thunk left plain: the
    sanitizer runtime resolves its interceptors with dlsym before its shadow exists), through a
    fill, hits, and corrupt, truncated and foreign entries."""
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "native"))
    import build as nb

    lib = nb.build_comgrcache(asan="asan")[0]
    clang = os.path.join(nb.ROCM, "llvm", "bin", "clang")
    rt = subprocess.run([clang, "-print-file-name=libclang_rt.asan-x86_64.so"], capture_output=True,
                        text=True).stdout.strip()
    if not os.path.exists(rt):
        pytest.skip("clang's ASan runtime is not installed")
    d = tmp_path / "cache"
    d.mkdir()
    san = {"LD_PRELOAD": f"{rt}:{lib}", "ASAN_OPTIONS": "detect_leaks=0:halt_on_error=1",
           "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"}

    def run(write=False):
        env = dict(os.environ, GPUSHARE_COMGR_ACTION_CACHE=str(d), **san)
        if write:
            env["GPUSHARE_COMGR_ACTION_CACHE_WRITE"] = "1"
        r = subprocess.run([PROBE, "", "1"], capture_output=True, text=True, timeout=300, env=env)
        assert r.returncode == 0, r.stderr[-3000:]
        assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-3000:]
        return json.loads(r.stdout.strip().splitlines()[-1])

    digest = run(write=True)["exe_digest"]
    assert run()["cache"]["hits"] == 4
    entries = _entries(d)
    (d / entries[0]).write_bytes((d / entries[0]).read_bytes()[:-9])          # short by the checksum
    (d / entries[1]).write_bytes(b"GSCA0001" + b"\xff" * 64)                  # a count far past the end
    (d / entries[2]).write_bytes(b"")
    assert run()["exe_digest"] == digest
