"""Container entry point of the Llama-3-8B demo pod (BASELINE config 4).

Runs inside the environment the plugin's Allocate response created (quota shim preloaded),
loads a random-init Llama-3-8B, then runs prefill forwards for ``--seconds`` and prints JSON
lines: the quota it sees, the weight footprint, and tokens/s per interval. ``--probe-quota``
additionally tries to allocate past the quota and reports whether the shim refused it.
``--mode decode`` makes it a serving pod instead: a ``--seq`` token prompt is prefilled into a
KV cache and the pod then decodes greedily (one hipGraph replay per step, models/llama_serve.py);
a "step" is then one decode step of the whole batch and tokens/s counts generated tokens.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time


def _shim() -> dict | None:
    """The quota shim's ledger and arena counters (None without the shim): quota denials, the
    broker arena's size and use, granules borrowed beyond the grant, allocations that went to
    the driver."""
    import ctypes

    from .pod_worker import _shim_stats

    st = _shim_stats()
    if st is None:
        return None
    lib = ctypes.CDLL(None)
    try:
        f = lib.gpushare_shim_arena_stats
        f.argtypes = [ctypes.POINTER(ctypes.c_uint64)] * 2
        v = [ctypes.c_uint64() for _ in range(2)]
        if f(*(ctypes.byref(x) for x in v)):
            st.update(arena_bytes=v[0].value, arena_used=v[1].value)
        g = lib.gpushare_shim_arena_extra
        g.argtypes = [ctypes.POINTER(ctypes.c_uint64)] * 5
        w = [ctypes.c_uint64() for _ in range(5)]
        g(*(ctypes.byref(x) for x in w))
        st.update(zip(("extends", "extended", "driver_allocs", "driver_bytes", "limit_granules"), (x.value for x in w)))
        b = lib.gpushare_shim_arena_base
        b.restype = ctypes.c_uint64
        base = b()
        if base:
            st["arena_base_mod_mib"] = (base % (1 << 30)) >> 20
    except AttributeError:
        pass
    return st


_KFD_PROC: list = []


def _kfd_proc_dir() -> str | None:
    """This process's directory under ``/sys/class/kfd/kfd/proc``. KFD names it by the pid in the
    host's namespace, which is not ``os.getpid()`` inside a container; the process is then found
    by its PASID: the amdgpu VM that KFD took over is the one of the render node the runtime
    opened, and that file's fdinfo names it (``pasid:``)."""
    import glob

    if _KFD_PROC:
        return _KFD_PROC[0]
    d = f"/sys/class/kfd/kfd/proc/{os.getpid()}"
    if os.path.isdir(d):
        _KFD_PROC.append(d)
        return d
    pasids = set()
    for fd in os.listdir("/proc/self/fd"):
        try:
            if not os.readlink(f"/proc/self/fd/{fd}").startswith("/dev/dri/renderD"):
                continue
            with open(f"/proc/self/fdinfo/{fd}") as fh:
                for line in fh:
                    if line.startswith("pasid:"):
                        pasids.add(line.split(":", 1)[1].strip())
        except OSError:
            continue
    for p in glob.glob("/sys/class/kfd/kfd/proc/*/pasid"):
        try:
            with open(p) as fh:
                if fh.read().strip() in pasids:
                    _KFD_PROC.append(os.path.dirname(p))
                    return _KFD_PROC[0]
        except OSError:
            continue
    return None


def _evicted_ms() -> dict:
    """KFD's per-GPU count of how long this process's queues were evicted (ms): memory a KFD
    process maps being moved or validated by another process stops all of its queues."""
    import glob

    out = {}
    d = _kfd_proc_dir()
    if d is None:
        return out
    for f in glob.glob(f"{d}/stats_*/evicted_ms"):
        try:
            with open(f) as fh:
                out[f.split("/")[-2]] = int(fh.read().strip() or 0)
        except (OSError, ValueError):
            pass
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=20.0)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--seq", type=int, default=2048)
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--probe-quota", action="store_true")
    ap.add_argument("--start-file", default=None, help="wait for this file before timing (sync start)")
    ap.add_argument("--name", default="pod")
    ap.add_argument("--mode", default="prefill", choices=("prefill", "decode"))
    ap.add_argument("--decode-window", type=int, default=256, help="decode steps before rewinding to the prompt")
    ap.add_argument("--eager", action="store_true", help="decode: launch kernel by kernel instead of a hipGraph")
    ap.add_argument("--stream-priority", default=os.environ.get("GPUSHARE_STREAM_PRIORITY", "normal"),
                    choices=("normal", "high"), help="decode: the priority of the stream the steps run on")
    ap.add_argument("--graph", action="store_true",
                    help="decode: replay a hipGraph even under CU slots (default: eager when GPUSHARE_CU_SLOTS is "
                         "set, since graph replay in a CU-masked pod stalls next to a busy neighbour: "
                         "profiles/cu_mask/README.md)")
    a = ap.parse_args(argv)
    if os.environ.get("GPUSHARE_CU_SLOTS") and not a.graph:
        a.eager = True

    import torch

    from .llama import LlamaConfig, LlamaModel

    def emit(**kw):
        kw["pod"] = a.name
        print(json.dumps(kw), flush=True)

    free, total = torch.cuda.mem_get_info()
    sh0 = _shim() or {}
    emit(event="start", quota_total=total, free=free, ld_preload=os.environ.get("LD_PRELOAD", ""),
         shim_denied=sh0.get("denied"),                    # (the pod's ledger counts across its runs)
         container_units=os.environ.get("ALIYUN_COM_GPU_MEM_CONTAINER"),
         dev_units=os.environ.get("ALIYUN_COM_GPU_MEM_DEV"))
    cfg = LlamaConfig.llama3_8b(n_layers=a.layers)
    model = LlamaModel(cfg, "cuda", seed=hash(a.name) & 0xffff)
    tok = torch.randint(0, cfg.vocab, (a.batch, a.seq), device="cuda")
    srv = None
    if a.mode == "decode":
        from .llama_serve import LlamaServer

        srv = LlamaServer(model, a.batch, a.seq + a.decode_window + 1, priority=a.stream_priority)
        srv.prefill(tok)
        if not a.eager:
            srv.capture()
        if srv.stream is not None:                    # every step on it, no per-step hand-off
            torch.cuda.synchronize()
            torch.cuda.set_stream(srv.stream)
    else:
        model.forward(tok)
    torch.cuda.synchronize()
    emit(event="loaded", weight_bytes=model.weight_bytes(), params=cfg.n_params())
    if a.probe_quota:
        free, total = torch.cuda.mem_get_info()
        d0 = (_shim() or {}).get("denied") or 0
        try:
            x = torch.empty(int(free * 1.5) // 2, dtype=torch.bfloat16, device="cuda")
            emit(event="quota_probe", over_quota_alloc="allowed")
            del x
        except torch.OutOfMemoryError:
            emit(event="quota_probe", over_quota_alloc="denied",
                 probe_denied=((_shim() or {}).get("denied") or 0) - d0)
        torch.cuda.empty_cache()
    ev0 = _evicted_ms()
    emit(event="ready", evicted_ms=ev0, kfd_proc=_kfd_proc_dir())
    if a.start_file:
        while not os.path.exists(a.start_file):
            time.sleep(0.01)
    t0 = time.perf_counter()
    n = 0
    tokens = a.batch * a.seq if srv is None else a.batch
    last = t0
    lat = []
    while time.perf_counter() - t0 < a.seconds:
        ti = time.perf_counter()
        if srv is None:
            model.forward(tok)
        else:
            if srv.host_len >= srv.max_ctx:
                srv.rewind(a.seq)
            srv.step(use_graph=not a.eager)
        torch.cuda.synchronize()
        n += 1
        now = time.perf_counter()
        lat.append(now - ti)
        if now - last > 5.0:
            emit(event="progress", iters=n, tokens_per_s=n * tokens / (now - t0))
            last = now
    dt = time.perf_counter() - t0
    flops = (model.flops_per_token(a.seq) * tokens * n if srv is None
             else 2.0 * (cfg.n_params() - cfg.vocab * cfg.d_model) * tokens * n)
    lat.sort()

    def q(f):
        return round(lat[min(len(lat) - 1, int(f * (len(lat) - 1) + 0.5))] * 1e3, 2) if lat else None

    emit(event="done", iters=n, seconds=dt, tokens_per_s=n * tokens / dt, tflops=flops / dt / 1e12,
         peak_mem=torch.cuda.max_memory_allocated(), lat_p50_ms=q(0.5), lat_p99_ms=q(0.99),
         lat_max_ms=round(lat[-1] * 1e3, 2) if lat else None,
         cus=torch.cuda.get_device_properties(0).multi_processor_count,
         cu_slots=os.environ.get("GPUSHARE_CU_SLOTS"), shim=_shim(),
         evicted_ms={k: v - ev0.get(k, 0) for k, v in _evicted_ms().items()})
    return 0


if __name__ == "__main__":
    sys.exit(main())
