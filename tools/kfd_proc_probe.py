"""What the node can see of a process's HBM from outside it (no shim): KFD's per-process sysfs
(``/sys/class/kfd/kfd/proc/<pid>/vram_<gpu_id>``) and the DRM fdinfo of its render-node fds
(``/proc/<pid>/fdinfo/<fd>``: ``drm-memory-vram`` / ``drm-total-vram`` ...). Allocates through
HIP (KFD) and through a raw amdgpu GEM_CREATE on the render node and prints both views after
each step, one JSON line per step. Input for quota/watchdog.py.

    python tools/kfd_proc_probe.py
"""
from __future__ import annotations

import ctypes
import json
import os
import time

GIB = 1 << 30


def kfd_view(pid: int) -> dict:
    d = f"/sys/class/kfd/kfd/proc/{pid}"
    out = {}
    try:
        for n in sorted(os.listdir(d)):
            if n.startswith("vram_"):
                with open(os.path.join(d, n)) as f:
                    out[n] = int(f.read().strip() or 0)
    except OSError as e:
        out["error"] = str(e)
    return out


def fdinfo_view(pid: int) -> list:
    rows = []
    base = f"/proc/{pid}/fdinfo"
    for fd in sorted(os.listdir(base), key=int):
        try:
            with open(os.path.join(base, fd)) as f:
                lines = f.read().splitlines()
        except OSError:
            continue
        drm = {k.strip(): v.strip() for k, _, v in (ln.partition(":") for ln in lines) if k.startswith("drm-")}
        if drm:
            try:
                target = os.readlink(f"/proc/{pid}/fd/{fd}")
            except OSError:
                target = "?"
            rows.append({"fd": int(fd), "target": target, **drm})
    return rows


def main():
    import torch

    pid = os.getpid()
    ls = sorted(os.listdir("/sys/class/kfd/kfd/proc")) if os.path.isdir("/sys/class/kfd/kfd/proc") else None

    def emit(step, **kw):
        print(json.dumps({"step": step, "kfd": kfd_view(pid), "fdinfo": fdinfo_view(pid), **kw}), flush=True)

    print(json.dumps({"kfd_proc_dir_entries": ls[:20] if ls else ls, "cgroup": open("/proc/self/cgroup").read()}),
          flush=True)
    torch.cuda.init()
    torch.empty(1, device="cuda")
    torch.cuda.synchronize()
    emit("hip_init")
    x = torch.empty(8 * GIB, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    time.sleep(0.2)
    emit("hip_8GiB")
    from aliyun_gpushare_device_plugin_amd.device.smi import SMI

    with SMI("auto") as s:
        minor = s.device(0).render_minor
    libc = ctypes.CDLL(None, use_errno=True)
    libc.ioctl.argtypes = [ctypes.c_int, ctypes.c_ulong, ctypes.c_void_p]
    fd = os.open(f"/dev/dri/renderD{minor}", os.O_RDWR)

    class Create(ctypes.Structure):
        _fields_ = [("bo_size", ctypes.c_uint64), ("alignment", ctypes.c_uint64), ("domains", ctypes.c_uint64),
                    ("domain_flags", ctypes.c_uint64)]
    a = Create(2 * GIB, 4096, 0x4, 0)
    r = libc.ioctl(fd, (3 << 30) | (32 << 16) | (ord("d") << 8) | 0x40, ctypes.addressof(a))
    time.sleep(0.2)
    emit("gem_2GiB", rc=r, errno=ctypes.get_errno(), gem_fd=fd)
    del x
    torch.cuda.empty_cache()
    time.sleep(0.2)
    emit("hip_freed")
    os.close(fd)
    time.sleep(0.2)
    emit("gem_fd_closed")


if __name__ == "__main__":
    main()
