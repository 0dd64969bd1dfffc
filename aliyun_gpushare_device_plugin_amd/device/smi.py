"""ctypes binding of ``libgpushare_gpuinfo`` (native/gpuinfo/gpuinfo.h).

This is the L0 hardware binding layer — the MI355X replacement for go-nvml (reference
``nvidia.go:44-86``, ``gpumanager.go:36-47``). The Python side never parses sysfs itself:
everything hardware-facing is in C++.
"""
from __future__ import annotations

import ctypes
import dataclasses
import json
import threading

from ..utils.native import ensure_built

GS_HEALTHY, GS_UNHEALTHY, GS_MISSING = 0, 1, 2
LINK_NONE, LINK_PCIE, LINK_XGMI, LINK_SELF = 0, 1, 2, 3
LINK_NAMES = {LINK_NONE: "none", LINK_PCIE: "pcie", LINK_XGMI: "xgmi", LINK_SELF: "self"}

EV_NONE, EV_VMFAULT, EV_THERMAL, EV_PRE_RESET, EV_POST_RESET = 0, 1, 2, 3, 4
EV_UNPLUG, EV_REPLUG, EV_ECC_UE, EV_LINK_DOWN, EV_LINK_UP = 10, 11, 12, 13, 14
EVENT_NAMES = {EV_NONE: "none", EV_VMFAULT: "vmfault", EV_THERMAL: "thermal", EV_PRE_RESET: "pre_reset",
               EV_POST_RESET: "post_reset", EV_UNPLUG: "unplug", EV_REPLUG: "replug", EV_ECC_UE: "ecc_ue",
               EV_LINK_DOWN: "link_down", EV_LINK_UP: "link_up"}


class _Device(ctypes.Structure):
    _fields_ = [("index", ctypes.c_int32), ("kfd_node", ctypes.c_int32), ("render_minor", ctypes.c_int32),
                ("numa_node", ctypes.c_int32), ("health", ctypes.c_int32),
                ("compute_partition", ctypes.c_int32), ("memory_partition", ctypes.c_int32),
                ("num_xcc", ctypes.c_int32), ("num_cu", ctypes.c_int32), ("gfx_version", ctypes.c_int32),
                ("unique_id", ctypes.c_uint64), ("hive_id", ctypes.c_uint64), ("vram_total", ctypes.c_uint64),
                ("vram_used", ctypes.c_uint64), ("ecc_ue", ctypes.c_uint64), ("ecc_ce", ctypes.c_uint64),
                ("uuid", ctypes.c_char * 40), ("bdf", ctypes.c_char * 16), ("name", ctypes.c_char * 64),
                ("gfx", ctypes.c_char * 16)]


class _Link(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int32), ("hops", ctypes.c_int32), ("weight", ctypes.c_int32),
                ("reserved", ctypes.c_int32), ("max_bandwidth_mbps", ctypes.c_uint64)]


class _HealthStatus(ctypes.Structure):
    _fields_ = [(f, ctypes.c_int32) for f in ("events_api", "events_armed", "events_last_status", "ecc_api",
                                               "ecc_reads_ok", "ecc_reads_failed", "ecc_last_status", "refreshes")]


class _Event(ctypes.Structure):
    _fields_ = [("index", ctypes.c_int32), ("kind", ctypes.c_int32), ("message", ctypes.c_char * 96)]


@dataclasses.dataclass(frozen=True)
class GPU:
    index: int
    uuid: str
    bdf: str
    name: str
    gfx: str
    vram_total: int
    vram_used: int
    numa_node: int
    render_minor: int
    kfd_node: int
    unique_id: int
    hive_id: int
    num_xcc: int
    num_cu: int
    compute_partition: int
    memory_partition: int
    ecc_ue: int
    ecc_ce: int
    health: int

    @property
    def render_node(self) -> str | None:
        return f"/dev/dri/renderD{self.render_minor}" if self.render_minor >= 0 else None


@dataclasses.dataclass(frozen=True)
class Link:
    type: int
    hops: int
    weight: int
    max_bandwidth_mbps: int

    @property
    def type_name(self) -> str:
        return LINK_NAMES.get(self.type, "none")


@dataclasses.dataclass(frozen=True)
class Event:
    index: int
    kind: int
    message: str

    @property
    def name(self) -> str:
        return EVENT_NAMES.get(self.kind, str(self.kind))


_lib = None
_lib_lock = threading.Lock()


def _load():
    global _lib
    with _lib_lock:
        if _lib is None:
            lib = ctypes.CDLL(ensure_built("gpuinfo"))
            lib.gs_open.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p)]
            lib.gs_close.argtypes = [ctypes.c_void_p]
            lib.gs_close.restype = None
            lib.gs_backend_name.argtypes = [ctypes.c_void_p]
            lib.gs_backend_name.restype = ctypes.c_char_p
            lib.gs_last_error.restype = ctypes.c_char_p
            for fn in ("gs_refresh", "gs_device_count", "gs_inaccessible_count", "gs_events_start"):
                getattr(lib, fn).argtypes = [ctypes.c_void_p]
            lib.gs_get_device.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(_Device)]
            lib.gs_get_link.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_Link)]
            lib.gs_wait_event.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(_Event)]
            lib.gs_inject.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
            lib.gs_probe.argtypes = [ctypes.c_void_p, ctypes.c_int]
            lib.gs_health_status.argtypes = [ctypes.c_void_p, ctypes.POINTER(_HealthStatus)]
            lib.gs_to_json.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]
            if lib.gs_abi_version() != 2:
                raise RuntimeError("libgpushare_gpuinfo ABI mismatch")
            _lib = lib
    return _lib


class SMIError(RuntimeError):
    pass


class SMI:
    """One open backend. Thread-safe: the C++ side locks its device table, and this wrapper
    makes ``close()`` safe against calls in flight on other threads (the health monitor
    blocks in ``wait_event`` while the manager may shut down) — close marks the handle
    closing, waits for in-flight calls to return, and only then frees it; later calls raise
    ``SMIError`` instead of touching freed memory (found by the ASan run in
    tests/test_gpuinfo_native.py)."""

    CLOSE_WAIT_S = 30.0

    def __init__(self, spec: str = "auto"):
        self._lib = _load()
        h = ctypes.c_void_p()
        if self._lib.gs_open(spec.encode(), ctypes.byref(h)) != 0:
            raise SMIError(f"gs_open({spec!r}): {self._lib.gs_last_error().decode()}")
        self._h = h
        self._cv = threading.Condition()
        self._active = 0
        self._closing = False
        self.spec = spec

    def _enter(self):
        with self._cv:
            if self._h is None or self._closing:
                raise SMIError("SMI handle is closed")
            self._active += 1
            return self._h

    def _exit(self):
        with self._cv:
            self._active -= 1
            if self._active == 0:
                self._cv.notify_all()

    def _call(self, fn, *args):
        h = self._enter()
        try:
            return fn(h, *args)
        finally:
            self._exit()

    def close(self):
        cv = getattr(self, "_cv", None)
        if cv is None:
            return
        with cv:
            if self._h is None or self._closing:
                return
            self._closing = True
            cv.wait_for(lambda: self._active == 0, timeout=self.CLOSE_WAIT_S)
            if self._active:
                # a native call is stuck: leak the handle rather than free it under the call
                return
            self._lib.gs_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def backend(self) -> str:
        return self._call(self._lib.gs_backend_name).decode()

    def _err(self, what):
        raise SMIError(f"{what}: {self._lib.gs_last_error().decode()}")

    def refresh(self) -> int:
        n = self._call(self._lib.gs_refresh)
        if n < 0:
            self._err("gs_refresh")
        return n

    def count(self) -> int:
        return self._call(self._lib.gs_device_count)

    def inaccessible(self) -> int:
        return self._call(self._lib.gs_inaccessible_count)

    def device(self, i: int) -> GPU:
        d = _Device()
        if self._call(self._lib.gs_get_device, i, ctypes.byref(d)) != 0:
            self._err(f"gs_get_device({i})")
        return GPU(index=d.index, uuid=d.uuid.decode(), bdf=d.bdf.decode(), name=d.name.decode(),
                   gfx=d.gfx.decode(), vram_total=d.vram_total, vram_used=d.vram_used, numa_node=d.numa_node,
                   render_minor=d.render_minor, kfd_node=d.kfd_node, unique_id=d.unique_id, hive_id=d.hive_id,
                   num_xcc=d.num_xcc, num_cu=d.num_cu, compute_partition=d.compute_partition,
                   memory_partition=d.memory_partition, ecc_ue=d.ecc_ue, ecc_ce=d.ecc_ce, health=d.health)

    def devices(self) -> list[GPU]:
        return [self.device(i) for i in range(self.count())]

    def link(self, i: int, j: int) -> Link:
        L = _Link()
        if self._call(self._lib.gs_get_link, i, j, ctypes.byref(L)) != 0:
            self._err(f"gs_get_link({i},{j})")
        return Link(L.type, L.hops, L.weight, L.max_bandwidth_mbps)

    def link_matrix(self) -> list[list[Link]]:
        n = self.count()
        return [[self.link(i, j) for j in range(n)] for i in range(n)]

    def events_start(self):
        self._call(self._lib.gs_events_start)

    def health_status(self) -> dict:
        """What the health path has on this backend: event notification armed on how many
        devices, ECC counters read at the last refresh (``gs_health_status``)."""
        st = _HealthStatus()
        if self._call(self._lib.gs_health_status, ctypes.byref(st)) < 0:
            self._err("gs_health_status")
        return {f: int(getattr(st, f)) for f, _ in _HealthStatus._fields_}

    def wait_event(self, timeout_ms: int) -> Event | None:
        ev = _Event()
        rc = self._call(self._lib.gs_wait_event, int(timeout_ms), ctypes.byref(ev))
        if rc < 0:
            self._err("gs_wait_event")
        if rc == 0:
            return None
        return Event(ev.index, ev.kind, ev.message.decode(errors="replace"))

    def probe(self, i: int) -> bool | None:
        """Is device ``i`` working, beyond being enumerated: True / False, None = no probe on
        this backend (``gs_probe``: amdgpu's gpu_metrics, refused while the GPU is in reset)."""
        rc = self._call(self._lib.gs_probe, int(i))
        if rc == -2:
            self._err(f"gs_probe({i})")
        return None if rc < 0 else rc == 1

    def inject(self, cmd: str):
        if self._call(self._lib.gs_inject, cmd.encode()) != 0:
            self._err(f"gs_inject({cmd!r})")

    def to_json(self) -> dict:
        h = self._enter()
        try:
            n = self._lib.gs_to_json(h, None, 0)
            buf = ctypes.create_string_buffer(n + 1)
            self._lib.gs_to_json(h, buf, n + 1)
        finally:
            self._exit()
        return json.loads(buf.value.decode())
