"""SIGQUIT stack dump (reference ``coredump.go:10-30``, wired at ``gpumanager.go:97-101``).

The reference writes every goroutine's stack to ``/etc/kubernetes/go_<YYYYmmddHHMMSS>.txt``,
a path its DaemonSet never mounts. Here the directory is configurable
(default: a writable temp dir) and the dump includes every Python thread plus the native
frames ``faulthandler`` can see.
"""
from __future__ import annotations

import faulthandler
import os
import sys
import tempfile
import threading
import time
import traceback


def dump_dir() -> str:
    return os.environ.get("GPUSHARE_DUMP_DIR") or tempfile.gettempdir()


def stack_trace() -> str:
    frames = sys._current_frames()
    names = {t.ident: t.name for t in threading.enumerate()}
    out = []
    for ident, frame in frames.items():
        out.append(f"--- thread {names.get(ident, '?')} ({ident}) ---\n")
        out.extend(traceback.format_stack(frame))
    return "".join(out)


def coredump(path: str | None = None) -> str:
    if path is None:
        path = os.path.join(dump_dir(), "gpushare_" + time.strftime("%Y%m%d%H%M%S") + ".txt")
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    tmp = path + ".partial"          # written in full, then renamed: readers never see half a dump
    with open(tmp, "w") as f:
        f.write(stack_trace())
        f.write("\n--- faulthandler (native view) ---\n")
        f.flush()
        faulthandler.dump_traceback(file=f, all_threads=True)
    os.replace(tmp, path)
    return path
