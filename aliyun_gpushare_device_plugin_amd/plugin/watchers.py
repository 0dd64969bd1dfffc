"""File-system and OS-signal watchers (component C10; reference ``watchers.go:10-32``).

``FSWatcher`` uses Linux inotify through ctypes (no fsnotify equivalent installed) and falls
back to polling the directory when inotify is unavailable. Events are delivered to a queue
shared with the signal watcher so the lifecycle loop has one ``select``-like wait point.
"""
from __future__ import annotations

import ctypes
import ctypes.util
import os
import queue
import select
import signal
import struct
import threading

IN_CREATE = 0x00000100
IN_DELETE = 0x00000200
IN_MOVED_TO = 0x00000080
IN_NONBLOCK = 0o4000
IN_CLOEXEC = 0o2000000
_EVENT_HDR = struct.Struct("iIII")


class FSEvent:
    __slots__ = ("name", "op")

    def __init__(self, name: str, op: str):
        self.name, self.op = name, op

    def __repr__(self):
        return f"FSEvent({self.name!r}, {self.op})"


class FSWatcher:
    def __init__(self, directory: str, out: "queue.Queue", poll_interval: float = 0.5):
        self.dir = directory
        self.out = out
        self.poll_interval = poll_interval
        self._stop = threading.Event()
        self._fd = -1
        self.mode = "polling"
        libc_name = ctypes.util.find_library("c")
        try:
            libc = ctypes.CDLL(libc_name, use_errno=True)
            fd = libc.inotify_init1(IN_NONBLOCK | IN_CLOEXEC)
            if fd >= 0:
                wd = libc.inotify_add_watch(fd, os.fsencode(directory), IN_CREATE | IN_DELETE | IN_MOVED_TO)
                if wd >= 0:
                    self._fd, self.mode = fd, "inotify"
                else:
                    os.close(fd)
        except (OSError, AttributeError):
            pass
        self._thread = threading.Thread(target=self._run, name="fswatch", daemon=True)
        self._thread.start()

    def _run(self):
        if self._fd >= 0:
            while not self._stop.is_set():
                r, _, _ = select.select([self._fd], [], [], 0.2)
                if not r:
                    continue
                try:
                    data = os.read(self._fd, 65536)
                except BlockingIOError:
                    continue
                off = 0
                while off + _EVENT_HDR.size <= len(data):
                    _wd, mask, _cookie, ln = _EVENT_HDR.unpack_from(data, off)
                    name = data[off + _EVENT_HDR.size: off + _EVENT_HDR.size + ln].rstrip(b"\0").decode()
                    off += _EVENT_HDR.size + ln
                    op = "create" if mask & (IN_CREATE | IN_MOVED_TO) else "delete"
                    self.out.put(("fs", FSEvent(os.path.join(self.dir, name), op)))
            return
        seen = self._snapshot()
        while not self._stop.wait(self.poll_interval):
            cur = self._snapshot()
            for n, ino in cur.items():
                if seen.get(n) != ino:
                    self.out.put(("fs", FSEvent(os.path.join(self.dir, n), "create")))
            for n in seen.keys() - cur.keys():
                self.out.put(("fs", FSEvent(os.path.join(self.dir, n), "delete")))
            seen = cur

    def _snapshot(self):
        out = {}
        try:
            for e in os.scandir(self.dir):
                try:
                    out[e.name] = e.inode()
                except OSError:
                    pass
        except OSError:
            pass
        return out

    def close(self):
        self._stop.set()
        self._thread.join(timeout=1.0)
        if self._fd >= 0:
            os.close(self._fd)
            self._fd = -1


def watch_signals(out: "queue.Queue", sigs=(signal.SIGHUP, signal.SIGINT, signal.SIGTERM, signal.SIGQUIT)):
    """``newOSWatcher`` (``watchers.go:27-32``). Must be called from the main thread."""
    prev = {}

    def handler(signum, _frame):
        out.put(("signal", signum))

    for s in sigs:
        prev[s] = signal.signal(s, handler)
    return prev
