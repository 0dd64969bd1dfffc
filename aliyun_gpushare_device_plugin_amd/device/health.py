"""Live GPU health with recovery (component C3, re-designed).

The reference's ``watchXIDs`` is commented out ("FIXME: re-implement for new nvml
interface", ``nvidia.go:97-153``) so ``--health-check`` is a no-op, and a device that went
Unhealthy could never come back (``server.go:188``). Its intended policy: fatal XID events
mark the GPU unhealthy, application XIDs 31/43/45 are ignored (``nvidia.go:134``), an event
without a device marks every GPU unhealthy (``:138-143``).

MI355X policy, driven by the SMI event stream (rocm_smi event notification: VM fault,
thermal throttle, GPU pre/post reset — ``rocm_smi.h:319-323``) plus periodic re-enumeration:

================  ==============================================================
event             effect
================  ==============================================================
VM fault          application error (≙ XID 31/43) → ignored, counted
thermal throttle  informational → ignored, counted
pre-reset         Unhealthy ("resetting")
post-reset        Healthy again (unless still missing)
unplug / missing  Unhealthy, present=False (index kept: IDX annotations stay valid)
replug / back     Healthy, present=True
ECC UE increase   Unhealthy until a reset
xGMI link down    topology re-export (device stays Healthy)
================  ==============================================================

Recovery never depends on one event arriving (the reference's "no way to recover",
``server.go:188``; one lost POST_RESET would strand a whole 288 GiB GPU). The poll also ends
a mark when it sees the reset itself:

* "GPU reset in progress" (a pre-reset without its post-reset): Healthy again once the GPU is
  present *and working* on ``settle_polls`` consecutive polls. An MI355X stays enumerated in
  sysfs and SMI during a mode-1 reset, so being listed proves nothing: the functional probe
  (``SMI.probe``: amdgpu's gpu_metrics table, which the driver refuses while the GPU is in
  reset) must succeed on each of those polls. A device that is listed but failing the probe
  stays Unhealthy, and its count starts again; a backend with no probe falls back to presence;
* a GPU that left the enumeration and came back is Healthy again once it passes the probe;
* an ECC uncorrectable-error mark clears on an *observed* reset: a pre-reset event (then as
  above), the GPU leaving and re-joining the enumeration, or its UE counters going backwards
  (a reset cleared them) — the UE baseline restarts from the value read then.
"""
from __future__ import annotations

import threading
import time

from ..utils import log
from . import smi as S
from .model import DeviceModel


class HealthMonitor:
    def __init__(self, smi: S.SMI, model: DeviceModel, poll_interval: float = 5.0,
                 on_change=None, on_topology_change=None, on_sample=None, settle_polls: int = 2):
        self.smi, self.model = smi, model
        self.poll_interval = poll_interval
        self.settle_polls = max(1, settle_polls)
        # uuid -> "reset" (pre-reset seen, waiting for post-reset or settle_polls good polls,
        # counted in _settle) | "gone" (left the enumeration: its return is a reset)
        self._marks: dict[str, str] = {}
        self._settle: dict[str, int] = {}
        self._ecc_last: dict[str, int] = {}      # uuid -> UE count at the previous poll
        self.on_change = on_change
        self.on_topology_change = on_topology_change
        # on_sample(model_index, smi_device) after every poll: per-GPU HBM used for the
        # gpushare_hbm_used_bytes gauge
        self.on_sample = on_sample
        self.degraded: str = ""            # why health detection is weaker than it should be
        self._stop = threading.Event()
        self._threads: list[threading.Thread] = []
        self._ecc_baseline = {}
        self.events_seen: list[S.Event] = []
        self.status: dict = {}
        self.ignored = 0
        self._lock = threading.Lock()
        for g in smi.devices():
            self._ecc_baseline[g.uuid] = g.ecc_ue

    def start(self):
        self.smi.events_start()
        try:
            self.status = self.smi.health_status()
        except Exception as e:  # noqa: BLE001 - an older library without the call
            self.status = {}
            log.warning("health status unavailable: %s", e)
        st = self.status
        if st and st.get("events_armed", 0) < self.smi.count():
            # typically the plugin container cannot open /dev/kfd (not privileged / no device
            # cgroup grant): resets are then only seen by the poll, seconds late
            self.degraded = (f"SMI event notification armed on {st.get('events_armed', 0)}/{self.smi.count()} GPUs "
                             f"(status {st.get('events_last_status', 0)})")
            log.error("%s: resets/VM faults on the others are seen by polling only; check that the plugin "
                      "container can open /dev/kfd (privileged DaemonSet)", self.degraded)
        if st and st.get("ecc_reads_failed", 0):
            log.warning("ECC counters unreadable on %d GPU(s) (status %d): uncorrectable-error health is blind there",
                        st["ecc_reads_failed"], st.get("ecc_last_status", 0))
        for target, name in ((self._event_loop, "health-events"), (self._poll_loop, "health-poll")):
            t = threading.Thread(target=target, name=name, daemon=True)
            t.start()
            self._threads.append(t)
        if self.on_sample is not None:
            for g in self.model.gpus:           # first sample now, not one poll interval later
                d = next((x for x in self.smi.devices() if x.uuid == g.uuid), None)
                if d is not None:
                    self.on_sample(g.index, d)
        return self

    def stop(self):
        self._stop.set()
        for t in self._threads:
            t.join(timeout=2.0)

    @property
    def ready(self) -> bool:
        return not self.degraded

    # -- helpers --------------------------------------------------------------------------
    def _set(self, index: int, healthy: bool, reason: str, present: bool | None = None):
        if index < 0 or index >= self.model.count():
            return
        if self.model.set_health(index, healthy, reason, present) and self.on_change:
            self.on_change(index, healthy, reason)

    def _model_index_of_smi(self, smi_index: int) -> int:
        try:
            uuid = self.smi.device(smi_index).uuid
        except S.SMIError:
            return -1
        g = self.model.by_uuid(uuid)
        return g.index if g else -1

    # -- event stream ---------------------------------------------------------------------
    def handle_event(self, ev: S.Event):
        with self._lock:
            self.events_seen.append(ev)
        k = ev.kind
        if k in (S.EV_VMFAULT, S.EV_THERMAL):
            self.ignored += 1
            log.info("GPU event %s on %d ignored (application-level)", ev.name, ev.index)
            return
        if k in (S.EV_LINK_DOWN, S.EV_LINK_UP):
            if self.on_topology_change:
                self.on_topology_change(ev)
            return
        if k in (S.EV_UNPLUG, S.EV_REPLUG):
            self.poll_once()   # membership changes are resolved by re-enumeration
            return
        targets = range(self.model.count()) if ev.index < 0 else [self._model_index_of_smi(ev.index)]
        for idx in targets:
            g = self.model.gpu(idx)
            if k == S.EV_PRE_RESET:
                if g is not None:
                    with self._lock:
                        self._marks[g.uuid] = "reset"
                        self._settle[g.uuid] = 0
                self._set(idx, False, "GPU reset in progress")
            elif k == S.EV_POST_RESET:
                if g is not None:
                    try:
                        working = self.smi.probe(ev.index) if ev.index >= 0 else None
                    except S.SMIError:
                        working = None
                    if working is False:
                        # the event came, the GPU does not work yet: the poll clears the mark once it does
                        with self._lock:
                            self._marks[g.uuid] = "reset"
                            self._settle[g.uuid] = 0
                        continue
                    with self._lock:
                        self._marks.pop(g.uuid, None)
                    self._ecc_baseline[g.uuid] = self._current_ecc(g.uuid, self._ecc_baseline.get(g.uuid, 0))
                    if g.present:
                        self._set(idx, True, "recovered after reset")
            elif k == S.EV_ECC_UE:
                self.poll_once()

    def _current_ecc(self, uuid: str, dflt: int) -> int:
        for d in self.smi.devices():
            if d.uuid == uuid:
                return d.ecc_ue
        return dflt

    def _event_loop(self):
        while not self._stop.is_set():
            try:
                ev = self.smi.wait_event(200)
            except S.SMIError as e:
                log.warning("SMI event wait failed: %s", e)
                time.sleep(1.0)
                continue
            if ev is not None:
                self.handle_event(ev)

    # -- polling --------------------------------------------------------------------------
    def poll_once(self):
        try:
            self.smi.refresh()
            present = {d.uuid: d for d in self.smi.devices()}
        except S.SMIError as e:
            log.warning("SMI refresh failed: %s", e)
            return
        smi_index = {d.uuid: i for i, d in enumerate(self.smi.devices())} if self._marks else {}
        for g in self.model.gpus:
            d = present.get(g.uuid)
            mark0 = self._marks.get(g.uuid)
            working = None
            if d is not None and mark0 is not None:
                try:
                    working = self.smi.probe(smi_index[g.uuid])
                except (S.SMIError, KeyError):
                    working = False
            with self._lock:
                if d is None:
                    self._marks[g.uuid] = "gone"
                    self._settle.pop(g.uuid, None)
                    mark, settled = "gone", 0
                else:
                    mark = self._marks.get(g.uuid)
                    # a poll counts towards the settle only when the GPU works, not just answers
                    settled = (self._settle.get(g.uuid, 0) + 1 if working is not False else 0) if mark == "reset" else 0
                    if mark == "reset":
                        self._settle[g.uuid] = settled
            if d is None:
                self._set(g.index, False, "device missing", present=False)
                continue
            if self.on_sample is not None:
                self.on_sample(g.index, d)
            base = self._ecc_baseline.setdefault(g.uuid, d.ecc_ue)
            last = self._ecc_last.get(g.uuid, d.ecc_ue)
            self._ecc_last[g.uuid] = d.ecc_ue
            why = None
            if mark is not None and working is False:
                # listed, but not working yet (still in reset): stays Unhealthy, the count restarts
                self._set(g.index, False, "GPU reset in progress (enumerated, not answering the functional probe)",
                          present=True)
                continue
            if d.ecc_ue < last:
                why = f"uncorrectable ECC counters went back ({last}->{d.ecc_ue}): reset observed"
            elif mark == "gone":
                why = "device back"
            elif mark == "reset" and settled >= self.settle_polls:
                why = (f"working on {settled} polls after a reset (post-reset event not seen)" if working
                       else f"answering SMI on {settled} polls after a reset (post-reset event not seen; no probe here)")
            if why is not None:
                # an observed reset: the UE baseline restarts from what the GPU reports now
                with self._lock:
                    self._marks.pop(g.uuid, None)
                    self._settle.pop(g.uuid, None)
                self._ecc_baseline[g.uuid] = base = d.ecc_ue
            if d.ecc_ue > base:
                self._set(g.index, False, f"uncorrectable ECC errors {base}->{d.ecc_ue}", present=True)
            elif why is not None:
                self._set(g.index, True, why, present=True)
            elif mark is None and not g.healthy and g.reason.startswith("uncorrectable ECC"):
                pass                      # stays marked until a reset is observed
            elif not g.present:
                self._set(g.index, True, "device back", present=True)

    def _poll_loop(self):
        while not self._stop.wait(self.poll_interval):
            self.poll_once()
