"""The buffered logger: a WARNING written while the flusher thread writes must not deadlock.

The emitter and the flusher each nest two locks; they once took them in opposite orders, which
hung a restarted plugin inside the engine's start-up warning (found by the chaos test in
``test_durability.py``).
"""
from __future__ import annotations

import threading
import time

from aliyun_gpushare_device_plugin_amd.utils import log


class _SlowStream:
    def __init__(self):
        self.lines = 0

    def write(self, data):
        time.sleep(0.0005)          # widen the window in which the writer holds its lock
        self.lines += data.count("\n")

    def flush(self):
        pass


def test_warnings_and_the_flusher_do_not_deadlock():
    saved_stream = log._stream
    stream = _SlowStream()
    log.setup(stream=stream, buffered=True)
    stop = threading.Event()

    def flusher():
        while not stop.is_set():
            log.flush()

    def warner(n):
        for i in range(400):
            log.info("info %d %d", n, i)
            log.warning("warn %d %d", n, i)

    try:
        threads = [threading.Thread(target=flusher, daemon=True)]
        threads += [threading.Thread(target=warner, args=(n,), daemon=True) for n in range(3)]
        for t in threads:
            t.start()
        for t in threads[1:]:
            t.join(30)
            assert not t.is_alive(), "a logging caller deadlocked against the flusher"
        stop.set()
        threads[0].join(30)
        assert not threads[0].is_alive()
        log.flush()
        assert stream.lines == 3 * 400 * 2
    finally:
        stop.set()
        log.setup(buffered=False)
        log._stream = saved_stream
