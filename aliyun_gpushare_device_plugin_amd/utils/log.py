"""glog-compatible leveled logging.

The reference logs through glog with verbosity gates ``V(1)`` lifecycle, ``V(4)`` candidate
pods, ``V(5)`` all pods, ``V(6)`` per-pod decisions, ``V(8)`` raw kubelet lists
(``gpumanager.go:34-57``, ``allocate.go:69-77``, ``podmanager.go:194,270,313-320``,
``podutils.go:79-86``) and the DaemonSet runs ``-logtostderr --v=5``
(``device-plugin-ds.yaml:31-32``). ``V(n)`` here follows the same contract so operators'
muscle memory carries over; output is one line per record, optionally JSON-structured.
"""
from __future__ import annotations

import json
import logging
import os
import sys
import threading
import time

_VERBOSITY = int(os.environ.get("GPUSHARE_V", "0"))
_JSON = os.environ.get("GPUSHARE_LOG_JSON", "") == "1"
_lock = threading.Lock()

# ``logger`` carries the level gate (tests quiet it with ``logger.setLevel``); records are
# written by the lean emitter below instead of logging.Handler: Allocate logs two lines per
# call, and the stdlib path (findCaller + LogRecord + handler lock) costs ~150 us a line.
logger = logging.getLogger("gpushare")
_stream = None
_pid = os.getpid()
_sec_cache = [-1, ""]
_LEVELS = {logging.INFO: ("I", "info"), logging.WARNING: ("W", "warning"), logging.ERROR: ("E", "error")}


def _emit(levelno: int, msg, args, fields, depth: int = 2) -> None:
    if levelno < logger.getEffectiveLevel():
        return
    if args:
        try:
            msg = msg % args
        except (TypeError, ValueError):
            msg = f"{msg} {args!r}"
    f = sys._getframe(depth)
    src = f"{os.path.basename(f.f_code.co_filename)}:{f.f_lineno}"
    now = time.time()
    code, name = _LEVELS.get(levelno, ("I", "info"))
    if _JSON:
        d = {"ts": round(now, 6), "level": name, "msg": str(msg), "src": src,
             "thread": threading.current_thread().name}
        d.update(fields or {})
        line = json.dumps(d, default=str)
    else:
        sec = int(now)
        if _sec_cache[0] != sec:
            _sec_cache[0], _sec_cache[1] = sec, time.strftime("%m%d %H:%M:%S", time.localtime(sec))
        line = f"{code}{_sec_cache[1]}.{int((now - sec) * 1e6):06d} {_pid:>7} {src}] {msg}"
    with _lock:
        if _flusher is not None and levelno < logging.WARNING:
            # buffered INFO (like glog's): no write(2) on the caller's path — a syscall there
            # hands the GIL to whichever thread is busy (Allocate's latency); the flusher
            # thread writes within _FLUSH_S, and WARNING+ flushes everything at once
            _buf.append(line)
            _buf_bytes[0] += len(line)
            if _buf_bytes[0] < _BUF_MAX:
                return
        else:
            _buf.append(line)
    # outside _lock: flush() takes _wlock, then _lock — the only order either lock is nested in
    # (taking _wlock while holding _lock deadlocked against the flusher thread)
    flush()


_buf: list[str] = []
_buf_bytes = [0]
_BUF_MAX = 1 << 16
_FLUSH_S = 0.05
_flusher = None


_wlock = threading.Lock()      # orders writes; taken before _lock, never while holding it


def _take_locked() -> str:
    if not _buf:
        return ""
    data = "\n".join(_buf) + "\n"
    _buf.clear()
    _buf_bytes[0] = 0
    return data


def _write(data: str) -> None:
    st = _stream or sys.stderr
    try:
        st.write(data)
        st.flush()
    except (OSError, ValueError):
        pass


def flush() -> None:
    """Write buffered lines. The buffer is swapped under the emit lock and written outside
    it, so a logging caller never waits for the flusher's write(2)."""
    with _wlock:
        with _lock:
            data = _take_locked()
        if data:
            _write(data)


def _flush_loop(stop: threading.Event) -> None:
    while not stop.wait(_FLUSH_S):
        flush()
    flush()


def setup(verbosity: int | None = None, json_lines: bool | None = None, stream=None,
          buffered: bool | None = None) -> None:
    """``buffered``: INFO lines are written by a background thread every 50 ms (WARNING and
    above, and process exit, flush at once) — the plugin daemon turns it on."""
    global _VERBOSITY, _JSON, _stream, _pid, _flusher
    if buffered and _flusher is None:
        import atexit

        stop = threading.Event()
        _flusher = threading.Thread(target=_flush_loop, args=(stop,), name="log-flush", daemon=True)
        _flusher.start()
        atexit.register(lambda: (stop.set(), flush()))
    elif buffered is False and _flusher is not None:
        flush()
        _flusher = None
    with _lock:
        if verbosity is not None:
            _VERBOSITY = int(verbosity)
        if json_lines is not None:
            _JSON = bool(json_lines)
        if stream is not None:
            _stream = stream
        _pid = os.getpid()
        logger.propagate = False
        logger.setLevel(logging.DEBUG if _VERBOSITY > 0 else logging.INFO)


def verbosity() -> int:
    return _VERBOSITY


class _V:
    __slots__ = ("on",)

    def __init__(self, on: bool):
        self.on = on

    def __bool__(self) -> bool:
        return self.on

    def info(self, msg, *args, **fields):
        if self.on:
            _emit(logging.INFO, msg, args, fields)


def V(level: int) -> _V:
    """``if V(4): ...`` / ``V(4).info("...")`` exactly like glog."""
    return _V(_VERBOSITY >= level)


def info(msg, *args, **fields):
    _emit(logging.INFO, msg, args, fields)


def warning(msg, *args, **fields):
    _emit(logging.WARNING, msg, args, fields)


def error(msg, *args, **fields):
    _emit(logging.ERROR, msg, args, fields)


setup()
