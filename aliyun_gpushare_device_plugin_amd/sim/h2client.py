"""The simulated kubelet's device-manager client in C++ (``gs_h2c_*`` in libgpushare_dpserver).

The kubelet calls the plugin through grpc-go; the simulator's Python grpcio client spent
~0.3 ms of every Allocate round trip in its own machinery (a completion-queue thread, the
interpreter lock), which the real kubelet does not. ``NativeUnaryClient`` sends the call and
reads the reply in C++ (libnghttp2) and stamps both ends there, so the kubelet-side latency
the bench reports is the plugin's and the transport's. ``GS_SIM_KUBELET_CLIENT=python`` keeps
the grpcio client.
"""
from __future__ import annotations

import ctypes
import os
import threading


class UnaryError(Exception):
    def __init__(self, status: int, message: str):
        super().__init__(f"grpc status {status}: {message}")
        self.status, self.message = status, message


class NativeUnaryClient:
    _lib = None
    _mu = threading.Lock()

    @classmethod
    def lib(cls):
        with cls._mu:
            if cls._lib is None:
                from ..utils.native import ensure_built

                lib = ctypes.CDLL(ensure_built("dpserver"))      # calls wait on the socket: GIL released
                lib.gs_h2c_connect.restype, lib.gs_h2c_connect.argtypes = ctypes.c_void_p, [ctypes.c_char_p]
                I, C, I64 = ctypes.c_int, ctypes.c_char_p, ctypes.c_int64
                for fn in (lib.gs_h2c_unary, lib.gs_h2c_call):
                    fn.restype = I
                    fn.argtypes = [ctypes.c_void_p, C, C, I, C, I, ctypes.POINTER(I), ctypes.POINTER(I),
                                   C, I, C, I, I, ctypes.POINTER(I64), ctypes.POINTER(I64)]
                lib.gs_h2c_close.restype, lib.gs_h2c_close.argtypes = None, [ctypes.c_void_p]
                cls._lib = lib
        return cls._lib

    @staticmethod
    def wanted() -> bool:
        if os.environ.get("GS_SIM_KUBELET_CLIENT", "native") == "python":
            return False
        try:
            NativeUnaryClient.lib()
            return True
        except Exception:  # noqa: BLE001 - no library: the grpcio client
            return False

    def __init__(self, socket_path: str):
        self.l = self.lib()
        self.path = socket_path
        self.h = None
        self._connect()
        self._out = ctypes.create_string_buffer(4 << 20)
        self._msg = ctypes.create_string_buffer(1024)
        self._stamp = ctypes.create_string_buffer(64)

    def _connect(self):
        if self.h:
            self.l.gs_h2c_close(self.h)
        self.h = self.l.gs_h2c_connect(self.path.encode())
        if not self.h:
            raise ConnectionError(f"cannot connect to {self.path}")

    def unary(self, path: str, request: bytes, timeout: float = 10.0, framed: bool = False):
        """(reply bytes, handler stamp "in,out" or "", t_send ns, t_recv ns); UnaryError on a
        non-OK status, ConnectionError on a transport failure. A connection the plugin closed
        (restart) is re-dialled once, as a grpc channel reconnects to its socket. ``framed``:
        ``request`` is the whole DATA payload, sent without adding the gRPC length prefix."""
        try:
            return self._unary(path, request, timeout, framed)
        except ConnectionError:
            self._connect()
            return self._unary(path, request, timeout, framed)

    def _unary(self, path: str, request: bytes, timeout: float, framed: bool = False):
        if not self.h:
            self._connect()
        n, st = ctypes.c_int(), ctypes.c_int()
        ts, tr = ctypes.c_int64(), ctypes.c_int64()
        fn = self.l.gs_h2c_call if framed else self.l.gs_h2c_unary
        rc = fn(self.h, path.encode(), request, len(request), self._out, len(self._out),
                                 ctypes.byref(n), ctypes.byref(st), self._msg, len(self._msg), self._stamp,
                                 len(self._stamp), int(timeout * 1000), ctypes.byref(ts), ctypes.byref(tr))
        if rc != 0:
            raise ConnectionError(f"{path}: transport error")
        if st.value != 0:
            raise UnaryError(st.value, self._msg.value.decode(errors="replace"))
        return ctypes.string_at(self._out, n.value), self._stamp.value.decode(), ts.value, tr.value

    def close(self):
        if self.h:
            self.l.gs_h2c_close(self.h)
            self.h = None
