"""The DevicePlugin gRPC service served by ``libgpushare_dpserver.so`` (native/dpserver).

Reference ``pkg/gpu/nvidia/server.go`` serves the kubelet with grpc-go, natively. The Python
grpcio server (``plugin/server.py``) spent most of a kubelet-side Allocate in its own
machinery — a C-core poller thread hands each call to an executor thread, each taking the
interpreter lock — while the engine's prepared answer took ~0.1 ms (``bench.py``
``allocate_breakdown_p50_ms``). Here the HTTP/2 + gRPC framing runs in C++ (libnghttp2), and:

* the common Allocate is answered in the library from the engine's published table of
  prepared answers (``alloc/native_table.py`` ``attach_native``): claim, journal record, reply — the
  interpreter is not entered; the claim reaches the engine right after for the write-behind
  PATCH;
* every other request (the options, PreStartContainer, GetPreferredAllocation, and each
  Allocate the table cannot answer exactly as the engine would) is handed to handler threads
  here, which run the same servicer code as the grpcio server;
* ListAndWatch streams are fed from the device model by one thread.

Same interface as ``DevicePluginServer``; ``--grpc-server=python`` keeps the grpcio one.
"""
from __future__ import annotations

import ctypes
import json
import struct
import threading

from ..alloc.engine import AllocationError
from ..api import v1beta1 as api
from ..utils import log
from ..utils.native import ensure_built
from .server import DevicePluginServer, dial

_lib = None
_lib_mu = threading.Lock()
# Calls that wait (for a request, for a claim) release the interpreter lock while they do; the
# quick ones (reply, publish, version hooks, block/take) keep it: a ctypes call that drops the
# GIL has to queue behind whichever Python thread took it meanwhile to get it back (measured:
# ~0.3 ms per reply under load), which is longer than the call itself
_WAITING = {"gs_dp_start", "gs_dp_stop", "gs_dp_next", "gs_dp_taken_next", "gs_dp_fast_journal_open"}


class _Lib:
    """The library bound twice: ``ctypes.CDLL`` (GIL released) for the waiting calls,
    ``ctypes.PyDLL`` (GIL kept) for the rest."""

    def __init__(self, path: str):
        free, held = ctypes.CDLL(path), ctypes.PyDLL(path)
        P, I, I64, U64, B = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint64, ctypes.c_char_p
        for name, res, args in _SIGNATURES(P, I, I64, U64, B):
            fn = getattr(free if name in _WAITING else held, name)
            fn.restype, fn.argtypes = res, args
            setattr(self, name, fn)
            if name == "gs_dp_taken_next":           # the non-blocking drain keeps the GIL
                poll = held.gs_dp_taken_next
                poll.restype, poll.argtypes = res, args
                self.gs_dp_taken_poll = poll


def load():
    """The loaded library (built in-tree when missing or stale); raises NativeUnavailable."""
    global _lib
    with _lib_mu:
        if _lib is None:
            _lib = _Lib(ensure_built("dpserver"))
    return _lib


def _SIGNATURES(P, I, I64, U64, B):
    C = ctypes.c_char_p
    return (("gs_dp_start", P, [B, C, I]),
            ("gs_dp_stop", None, [P]),
            ("gs_dp_next", I64, [P, I, C, I, C, I, ctypes.POINTER(I), ctypes.POINTER(I64)]),
            ("gs_dp_reply", I, [P, I64, I, B, C, I]),
            ("gs_dp_set_devices", I, [P, C, I]),
            ("gs_dp_fast_publish", I, [P, C, I]),
            ("gs_dp_set_version", None, [P, U64]),
            ("gs_dp_set_gen", None, [P, U64]),
            ("gs_dp_fast_block", None, [P]),
            ("gs_dp_fast_unblock", None, [P]),
            ("gs_dp_fast_take", None, [P, B]),
            ("gs_dp_set_fast_wait_us", None, [P, I]),
            ("gs_dp_set_watch_wait_us", None, [P, I]),
            ("gs_dp_spin", None, [P, I]),
            ("gs_dp_taken_next", I, [P, I, C, I]),
            ("gs_dp_taken_pending", I, [P]),
            ("gs_dp_fast_journal_open", I, [P, B, U64]),
            ("gs_dp_fast_journal_used", U64, [P]),
            ("gs_dp_fast_journal_prefault", None, [P]),
            ("gs_dp_fast_journal_rotate", I, [P]),
            ("gs_dp_stats", I, [P, C, I]))


class NativeFast:
    """The engine's handle on the server's fast path (``Allocator.attach_native``)."""

    def __init__(self, lib, h):
        self.lib, self.h = lib, h
        self.spin_us = 0
        self._buf = ctypes.create_string_buffer(1 << 20)

    def publish(self, blob: bytes) -> None:
        if self.lib.gs_dp_fast_publish(self.h, blob, len(blob)) != 0:
            log.error("native fast table rejected (%d bytes)", len(blob))

    def set_version(self, v: int) -> None:
        self.lib.gs_dp_set_version(self.h, v)

    def set_gen(self, g: int) -> None:
        self.lib.gs_dp_set_gen(self.h, g)

    def block(self) -> None:
        self.lib.gs_dp_fast_block(self.h)

    def unblock(self) -> None:
        self.lib.gs_dp_fast_unblock(self.h)

    def take(self, uid: str) -> None:
        self.lib.gs_dp_fast_take(self.h, uid.encode())

    def pending(self) -> int:
        return self.lib.gs_dp_taken_pending(self.h)

    def taken_next(self, timeout_ms: int):
        """(uid, AllocateRequest bytes, wall time, handler ns, arrival CLOCK_MONOTONIC ns, watch-wait
        ns, table-wait ns); () on timeout; None once stopped."""
        fn = self.lib.gs_dp_taken_poll if timeout_ms <= 0 else self.lib.gs_dp_taken_next
        n = fn(self.h, timeout_ms, self._buf, len(self._buf))
        if n == 0:
            return ()
        if n < 0:
            if n == -2:
                self._buf = ctypes.create_string_buffer(len(self._buf) * 4)
                return ()
            return None
        b = ctypes.string_at(self._buf, n)
        (lu,) = struct.unpack_from("<I", b, 0)
        uid = b[4:4 + lu].decode()
        (lr,) = struct.unpack_from("<I", b, 4 + lu)
        o = 8 + lu
        req = b[o:o + lr]
        return (uid, req) + struct.unpack_from("<dQqQQ", b, o + lr)

    def journal_open(self, path: str, nbytes: int) -> None:
        if self.lib.gs_dp_fast_journal_open(self.h, path.encode(), nbytes) != 0:
            raise OSError(f"cannot map the native Allocate journal {path}")

    def journal_used(self) -> int:
        return self.lib.gs_dp_fast_journal_used(self.h)

    def spin(self, us: int) -> None:
        self.lib.gs_dp_spin(self.h, us)

    def journal_prefault(self) -> None:
        self.lib.gs_dp_fast_journal_prefault(self.h)

    def journal_rotate(self) -> None:
        self.lib.gs_dp_fast_journal_rotate(self.h)


class _Ctx:
    """What the servicer code uses of a grpc ServicerContext."""

    def __init__(self):
        self.callbacks = []

    def add_callback(self, fn) -> bool:
        self.callbacks.append(fn)
        return True


class NativeDevicePluginServer(DevicePluginServer):
    # fast_wait_us: how long an Allocate that finds the table one pod-cache change behind waits
    # for the engine to republish it before going to the engine's full path (~0.3 ms itself);
    # watch_wait_us: how long one that no candidate matches waits for the plugin's pod watch
    # to deliver the pod (the kubelet's watch can be ahead) before the engine's path
    # spin_us: after a pod was published into the table, the connection threads busy-poll this
    # long for the kubelet's Allocate instead of sleeping (0 = never)
    def __init__(self, *a, handler_threads: int = 4, fast_wait_us: int = 300, watch_wait_us: int = 2000,
                 spin_us: int = 0, **kw):
        super().__init__(*a, **kw)
        self.handler_threads = handler_threads
        self.fast_wait_us = fast_wait_us
        self.watch_wait_us = watch_wait_us
        self.spin_us = spin_us
        self._h = None
        self._lib = None
        self._threads: list[threading.Thread] = []
        self.fast: NativeFast | None = None

    # -- lifecycle --------------------------------------------------------------------------
    def start(self):
        self._cleanup()
        import os

        os.makedirs(os.path.dirname(self.socket), exist_ok=True)
        lib = self._lib = load()
        err = ctypes.create_string_buffer(512)
        h = lib.gs_dp_start(self.socket.encode(), err, len(err))
        if not h:
            raise RuntimeError(f"native device-plugin server: {err.value.decode()}")
        self._h = h
        lib.gs_dp_set_fast_wait_us(h, self.fast_wait_us)
        lib.gs_dp_set_watch_wait_us(h, self.watch_wait_us)
        self._push_devices()
        self.fast = NativeFast(lib, h)
        self.fast.spin_us = self.spin_us
        self.allocator.attach_native(self.fast)
        for i in range(self.handler_threads):
            t = threading.Thread(target=self._handle_loop, name=f"dp-native-{i}", daemon=True)
            t.start()
            self._threads.append(t)
        t = threading.Thread(target=self._devices_loop, name="dp-native-law", daemon=True)
        t.start()
        self._threads.append(t)
        dial(self.socket, 5.0).close()      # confirm the server answers (server.go:130-135)
        log.info("Starting to serve on %s (native server)", self.socket)

    def stop(self, grace: float = 0.5):
        self.stopped.set()
        self.model.notify_all()
        if self._h is not None:
            if self.allocator.native is self.fast:
                self.allocator.detach_native()
            self._lib.gs_dp_stop(self._h)
            for t in self._threads:
                t.join(timeout=2.0)
            self._h = None
        self._cleanup()

    def stats(self) -> dict:
        if self._h is None:
            return {}
        buf = ctypes.create_string_buffer(2048)
        n = self._lib.gs_dp_stats(self._h, buf, len(buf))
        return json.loads(buf.value.decode()) if n > 0 else {}

    # -- ListAndWatch -------------------------------------------------------------------------
    def _push_devices(self) -> None:
        body = api.ListAndWatchResponse(devices=self.model.device_list()).SerializeToString()
        self._lib.gs_dp_set_devices(self._h, body, len(body))
        self.metrics.listandwatch_sends.inc()

    def _devices_loop(self):
        gen = self.model.generation
        while not self.stopped.is_set():
            new = self.model.wait_change(gen, timeout=0.5)
            if new != gen and not self.stopped.is_set():
                gen = new
                self._push_devices()

    # -- requests the library hands over ----------------------------------------------------------
    def _handle_loop(self):
        lib, h = self._lib, self._h
        meth = ctypes.create_string_buffer(256)
        body = ctypes.create_string_buffer(8 << 20)
        n, t_in = ctypes.c_int(), ctypes.c_int64()
        while not self.stopped.is_set():
            rid = lib.gs_dp_next(h, 200, meth, len(meth), body, len(body), ctypes.byref(n), ctypes.byref(t_in))
            if rid == 0:
                continue
            if rid < 0:
                return
            # string_at copies the request only (``.raw`` would copy the whole 8 MiB buffer)
            self._handle(rid, meth.value.decode(), ctypes.string_at(body, n.value))

    def _handle(self, rid: int, method: str, raw: bytes) -> None:
        lib, h = self._lib, self._h
        ctx = _Ctx()
        status, msg, out = 0, None, b""
        try:
            name = method.rsplit("/", 1)[-1]
            if name == "Allocate":
                r = self.allocator.allocate_raw(api.AllocateRequest.FromString(raw), defer=ctx.add_callback)
                out = r if isinstance(r, bytes) else r.SerializeToString()
            elif name == "GetDevicePluginOptions":
                out = self.options().SerializeToString()
            elif name == "GetPreferredAllocation":
                out = self.allocator.preferred(api.PreferredAllocationRequest.FromString(raw)).SerializeToString()
            elif name == "PreStartContainer":
                self.allocator.prestart(api.PreStartContainerRequest.FromString(raw))
                out = api.PreStartContainerResponse().SerializeToString()
            else:
                status, msg = 12, f"unknown method {method}"
        except AllocationError as e:
            status, msg = 9, str(e)                 # FAILED_PRECONDITION, as the grpcio servicer
        except Exception as e:  # noqa: BLE001 - what grpcio answers for a handler exception
            log.warning("%s failed: %s", method, e)
            status, msg = 2, f"Exception calling application: {e}"
        lib.gs_dp_reply(h, rid, status, msg.encode() if msg else None, out, len(out))
        for fn in ctx.callbacks:
            try:
                fn()
            except Exception as e:  # noqa: BLE001
                log.warning("post-reply callback failed: %s", e)


def available() -> bool:
    try:
        load()
        return True
    except Exception:  # noqa: BLE001
        return False


__all__ = ["NativeDevicePluginServer", "NativeFast", "available", "load"]
