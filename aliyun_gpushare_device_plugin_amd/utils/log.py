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

logger = logging.getLogger("gpushare")


class _Fmt(logging.Formatter):
    _LVL = {"DEBUG": "D", "INFO": "I", "WARNING": "W", "ERROR": "E", "CRITICAL": "F"}

    def format(self, r: logging.LogRecord) -> str:
        if _JSON:
            d = {"ts": round(r.created, 6), "level": r.levelname.lower(), "msg": r.getMessage(),
                 "src": f"{r.filename}:{r.lineno}", "thread": r.threadName}
            d.update(getattr(r, "fields", {}) or {})
            return json.dumps(d, default=str)
        t = time.strftime("%m%d %H:%M:%S", time.localtime(r.created))
        us = int((r.created % 1) * 1e6)
        return (f"{self._LVL.get(r.levelname, 'I')}{t}.{us:06d} {os.getpid():>7} "
                f"{r.filename}:{r.lineno}] {r.getMessage()}")


def setup(verbosity: int | None = None, json_lines: bool | None = None, stream=None) -> None:
    global _VERBOSITY, _JSON
    with _lock:
        if verbosity is not None:
            _VERBOSITY = int(verbosity)
        if json_lines is not None:
            _JSON = bool(json_lines)
        if not logger.handlers:
            h = logging.StreamHandler(stream or sys.stderr)
            h.setFormatter(_Fmt())
            logger.addHandler(h)
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
            logger.info(msg, *args, stacklevel=2, extra={"fields": fields} if fields else None)


def V(level: int) -> _V:
    """``if V(4): ...`` / ``V(4).info("...")`` exactly like glog."""
    return _V(_VERBOSITY >= level)


def info(msg, *args, **fields):
    logger.info(msg, *args, stacklevel=2, extra={"fields": fields} if fields else None)


def warning(msg, *args, **fields):
    logger.warning(msg, *args, stacklevel=2, extra={"fields": fields} if fields else None)


def error(msg, *args, **fields):
    logger.error(msg, *args, stacklevel=2, extra={"fields": fields} if fields else None)


setup()
