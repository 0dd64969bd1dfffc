"""A pod's container process for the bench and the demos: one OS process per pod, started the
way the container runtime starts it — with the Allocate response's env and the quota shim in
``LD_PRELOAD`` — running bf16 MFMA GEMM traffic inside its HBM quota.

Lifecycle (JSON lines on stdin/stdout):

* **standby** — the interpreter is up and torch is imported, but nothing has touched the GPU
  (the analogue of a container whose image is pulled and whose process is created). Prints
  ``{"event": "standby"}``. Standbys are fresh interpreters, or children forked from one
  interpreter that imported torch once (``--zygote``, ``zygote()``).
* ``{"cmd": "start", "env": {...}, "gemm": 4096, "burst": 8, "fill": 0.85}`` — the pod was
  admitted: the Allocate env (quota, ledger, visible GPU) is applied *before* the HIP runtime
  initialises, so the shim (preloaded since exec, initialised lazily at the first KFD ioctl)
  enforces this pod's quota. The worker reads its quota back through ``hipMemGetInfo``, holds
  ``fill`` of it (the pod's resident model state) plus a GEMM working set, runs one GEMM and
  prints ``{"event": "ready", "init_ms": ..., "quota": ..., ...}``. With ``"two_phase": true``
  it stops after the runtime is up (``{"event": "inited"}``) and allocates on ``{"cmd": "alloc"}``.
* traffic — bursts of ``burst`` GEMMs on the hand-written gfx950 kernel until told to stop;
  ``{"cmd": "stats"}`` answers ``{"event": "stats", "gemms": n, "t": ...}`` between bursts.
* ``{"cmd": "stop"}`` — frees everything (its HBM is back on the device when ``done`` is
  printed, before the process exits), prints ``{"event": "done", ...}`` and exits 0.
* ``{"cmd": "exit"}`` — the program just ends: a normal process exit (the C runtime's exit: atexit
  handlers, library destructors) with nothing freed and no arena release, as a pod whose main
  returns. A SIGTERM (the kubelet's stop) takes the default action: the process ends at once.

The reference's demo pod is ``cheyang/gpu-player:v2`` (``demo/binpack-1/binpack-1.yaml:39``);
``player_main.py`` is the long-running container entry point, this is its benchable form.
"""
from __future__ import annotations

import ctypes
import json
import os
import queue
import sys
import threading
import time


def _send(obj) -> None:
    sys.stdout.write(json.dumps(obj) + "\n")
    sys.stdout.flush()


def _shim_stats() -> dict | None:
    try:
        f = ctypes.CDLL(None).gpushare_shim_stats
    except AttributeError:
        return None
    f.argtypes = [ctypes.POINTER(ctypes.c_uint64)] * 4
    vals = [ctypes.c_uint64() for _ in range(4)]
    if not f(*(ctypes.byref(v) for v in vals)):
        return None
    return dict(zip(("used", "quota", "denied", "peak"), (v.value for v in vals)))


def _arena_timing() -> dict | None:
    """Where the quota shim's broker TAKE spent its time (ms), or None without an arena."""
    try:
        f = ctypes.CDLL(None).gpushare_shim_arena_timing
    except AttributeError:
        return None
    f.argtypes = [ctypes.POINTER(ctypes.c_uint64)] * 3
    vals = [ctypes.c_uint64() for _ in range(3)]
    if not f(*(ctypes.byref(v) for v in vals)):
        return None
    return dict(zip(("connect", "wait", "map"), (round(v.value / 1e6, 3) for v in vals)))


def _arena_stream() -> dict | None:
    """A streaming TAKE after it returned: allocations that waited for granules the broker still
    owed, the MORE batches and their import + map time, granules mapped of the grant."""
    try:
        f = ctypes.CDLL(None).gpushare_shim_arena_stream
    except AttributeError:
        return None
    f.argtypes = [ctypes.POINTER(ctypes.c_uint64)] * 9
    v = [ctypes.c_uint64() for _ in range(9)]
    if not f(*(ctypes.byref(x) for x in v)):
        return None
    out = {"waits": v[0].value, "wait_ms": round(v[1].value / 1e6, 3), "msgs": v[2].value,
           "map_ms": round(v[3].value / 1e6, 3), "mapped": v[4].value, "granted": v[5].value,
           "first": v[6].value, "first_reserve_ms": round(v[7].value / 1e6, 3),
           "first_access_ms": round(v[8].value / 1e6, 3)}
    try:
        g = ctypes.CDLL(None).gpushare_shim_arena_first
        g.argtypes = [ctypes.POINTER(ctypes.c_uint64)] * 3
        w = [ctypes.c_uint64() for _ in range(3)]
        if g(*(ctypes.byref(x) for x in w)):
            out["first_import_ms"] = round(w[0].value / 1e6, 3)
            out["first_map_ms"] = round(w[1].value / 1e6, 3)
            out["answer_ms"] = round(w[2].value / 1e6, 3)
    except AttributeError:
        pass
    return out


def _arena_release():
    """With an HBM broker arena (quota shim + GPUSHARE_HBM_BROKER), hand its granules back now
    that everything is freed, rather than at process exit. None without an arena."""
    try:
        f = ctypes.CDLL(None).gpushare_shim_arena_release
    except AttributeError:
        return None
    f.restype = ctypes.c_int
    r = f()
    if r == -1:
        # still live in the arena: torch's BLAS workspaces outlive empty_cache()
        import torch

        try:
            torch._C._cuda_clearCublasWorkspaces()
        except (AttributeError, RuntimeError):
            pass
        torch.cuda.empty_cache()
        r = f()
    return None if r == 0 else r == 1


def _nice() -> None:
    cpus = os.environ.get("GS_POD_CPUS", "")
    if cpus:
        # the node's pod CPUs: the ones its daemons do not have reserved (kubelet reservedSystemCPUs)
        try:
            os.sched_setaffinity(0, {int(c) for c in cpus.split(",") if c})
        except (OSError, ValueError):
            pass
    nice = int(os.environ.get("GS_POD_NICE", "0") or 0)
    if nice > 0:
        # a node runs its daemons (kubelet, device plugin) ahead of container workloads
        # (system-reserved CPU); the pod's start-up must not starve the plugin's watch
        os.nice(nice)


def zygote(ctl_fd: int) -> int:
    """Fork standby pod processes from one interpreter that imported torch once (``--zygote FD``).

    Each request on the control socket ``ctl_fd`` carries two fds, the child's stdin and stdout.
    The zygote forks, and the child serves them as a standby pod exactly as ``main`` does. The
    zygote answers the child's pid. Nothing here touches the GPU: the child's HIP runtime starts
    after its ``start`` command, with the pod's env. The zygote exits when the socket closes.
    A fresh interpreter per standby costs ~1.5 s of CPU (the torch import). At 4 pods/s that is
    6 cores taken from the pods starting at the same time; a fork costs milliseconds."""
    import signal
    import socket

    _nice()
    import torch  # noqa: F401

    ctl = socket.socket(fileno=ctl_fd)
    signal.signal(signal.SIGCHLD, signal.SIG_IGN)          # the kernel reaps the children
    while True:
        try:
            msg, fds, _, _ = socket.recv_fds(ctl, 16, 2)
        except OSError:
            return 0
        if not msg:
            return 0
        if len(fds) != 2:
            for fd in fds:
                os.close(fd)
            continue
        sys.stdout.flush()
        pid = os.fork()
        if pid == 0:
            try:
                ctl.close()
                signal.signal(signal.SIGCHLD, signal.SIG_DFL)
                os.dup2(fds[0], 0)
                os.dup2(fds[1], 1)
                for fd in fds:
                    os.close(fd)
                rc = _pod()
            except BaseException:  # noqa: BLE001 - a child never returns into the zygote's loop
                import traceback

                traceback.print_exc()
                rc = 1
            sys.stdout.flush()
            os._exit(rc or 0)
        for fd in fds:
            os.close(fd)
        ctl.sendall(f"{pid}\n".encode())


def _release_timing() -> dict | None:
    """Where the quota shim's last arena release spent its time (ms), or None without the shim."""
    try:
        f = ctypes.CDLL(None).gpushare_shim_arena_release_timing
    except AttributeError:
        return None
    f.argtypes = [ctypes.POINTER(ctypes.c_uint64)] * 5
    v = [ctypes.c_uint64() for _ in range(5)]
    if not f(*(ctypes.byref(x) for x in v)):
        return None
    return dict(zip(("sync", "unmap", "addr_free", "release", "kfd_free"), (round(x.value / 1e6, 3) for x in v)))


def main() -> int:
    if len(sys.argv) > 2 and sys.argv[1] == "--zygote":
        return zygote(int(sys.argv[2]))
    _nice()
    import torch  # noqa: F401 - imported in standby: the expensive part of a process start

    return _pod()


def _pod() -> int:
    import torch

    _send({"event": "standby", "pid": os.getpid()})
    line = sys.stdin.readline()
    if not line:
        return 0
    cmd = json.loads(line)
    if cmd.get("cmd") != "start":
        return 0
    os.environ.update({k: str(v) for k, v in (cmd.get("env") or {}).items()})
    g = int(cmd.get("gemm", 4096))
    burst = int(cmd.get("burst", 8))
    fill = float(cmd.get("fill", 0.0))

    t0 = time.perf_counter()
    torch.cuda.init()
    dev = torch.device("cuda", 0)
    t_rt = time.perf_counter()
    torch.empty(1, device=dev)                                 # context + runtime up (+ the arena's TAKE)
    t_up = time.perf_counter()
    free, quota = torch.cuda.mem_get_info(dev)                 # = the pod's quota under the shim
    take = _arena_timing()
    from .gemm_player import GemmPlayer

    if cmd.get("two_phase"):
        # the container is up before the GPU has room for its state (the driver may still be
        # wiping the HBM a retired pod freed): report, then allocate on "alloc"
        _send({"event": "inited", "init_ms": round((time.perf_counter() - t0) * 1e3, 3),
               "runtime_ms": round((t_up - t_rt) * 1e3, 3), "cuda_init_ms": round((t_rt - t0) * 1e3, 3),
               "take_ms": take})
        nxt = json.loads(sys.stdin.readline() or "{}")
        if nxt.get("cmd") != "alloc":
            return 0
    work = 3 * g * g * 2
    hold_bytes = max(0, int(quota * fill) - work)
    # resident state as a model holds it: many tensors (2 GiB each), not one block — amdgpu wipes
    # each freed buffer before returning it, so a pod's HBM comes back piecewise on release
    chunk = int(cmd.get("chunk", 2 << 30))
    t_hold = time.perf_counter()
    hold, chunk_ms = [], []
    for off in range(0, hold_bytes, chunk):
        t = time.perf_counter()
        hold.append(torch.empty(min(chunk, hold_bytes - off) // 2, dtype=torch.bfloat16, device=dev))
        chunk_ms.append(round((time.perf_counter() - t) * 1e3, 2))
    hold_ms = (time.perf_counter() - t_hold) * 1e3
    player = GemmPlayer(work, dev, g, g, g, touch_fraction=1.0, seed=os.getpid() & 0xffff)
    player.run(1)
    player.synchronize()
    init_ms = (time.perf_counter() - t0) * 1e3
    _send({"event": "ready", "init_ms": round(init_ms, 3), "quota": quota, "free_at_start": free,
           "held": hold_bytes + work, "hold_ms": round(hold_ms, 3), "hold_chunk_ms": chunk_ms, "shim": _shim_stats(),
           "stream": _arena_stream()})

    ctl: "queue.Queue" = queue.Queue()

    def reader():
        for ln in sys.stdin:
            try:
                c = json.loads(ln)
            except ValueError:
                continue
            c["_t"] = time.perf_counter()
            ctl.put(c)
        ctl.put({"cmd": "stop"})                                # parent went away

    threading.Thread(target=reader, daemon=True).start()
    # wait for each burst on a blocking-sync event: the thread sleeps until the GPU signals
    # instead of spinning a core (HIP's default) — co-located pods and the node's control plane
    # share the host's CPUs
    burst_done = torch.cuda.Event(blocking=True)
    gemms = 1
    t_start = time.time()
    t_asked = None
    while True:
        try:
            c = ctl.get_nowait()
        except queue.Empty:
            c = None
        if c is not None:
            if c.get("cmd") == "stats":
                _send({"event": "stats", "gemms": gemms, "t": time.time()})
            elif c.get("cmd") == "stop":
                t_asked = c.get("_t", time.perf_counter())
                break
            elif c.get("cmd") == "exit":
                sys.stdout.flush()
                ctypes.CDLL(None).exit(0)       # (a forked standby has no interpreter to unwind into)
            continue
        player.run(burst)
        burst_done.record(player.stream)
        burst_done.synchronize()
        gemms += burst
    # where a stop's time goes: the rest of the burst in flight when it came, freeing, the arena
    t_stop = time.perf_counter()
    player.release()
    st = _shim_stats()
    del hold, player
    torch.cuda.synchronize()
    torch.cuda.empty_cache()      # HBM back to the device now, not at process exit
    t_freed = time.perf_counter()
    # the broker arena (if any) is handed back first: its granules are on the ledger while it is
    # mapped, so the ledger read before the release would count them as a residue
    released = _arena_release()
    t_rel = time.perf_counter()
    after = _shim_stats()
    _send({"event": "done", "gemms": gemms, "t": time.time(), "seconds": time.time() - t_start, "shim": st,
           "used_after_release": (after or {}).get("used"), "arena_released": released,
           "stop_ms": {"burst_in_flight": round((t_stop - (t_asked or t_stop)) * 1e3, 3), "free": round((t_freed - t_stop) * 1e3, 3),
                       "arena_release": round((t_rel - t_freed) * 1e3, 3)},
           "release_ms": _release_timing() if released else None})
    # everything is freed and reported: leave without the interpreter's and torch's teardown
    # (hundreds of ms). The kernel still tears the process down, and only then do its last
    # references to an HBM broker's granules go (the broker quarantines them until then)
    sys.stdout.flush()
    if os.environ.get("GS_POD_CLEAN_EXIT") == "1":
        return 0          # a tool in the process (a profiler) writes its output at a normal exit
    os._exit(0)


if __name__ == "__main__":
    sys.exit(main())
