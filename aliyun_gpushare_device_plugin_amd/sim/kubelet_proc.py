"""The fake kubelet as its own OS process (bench and latency tests).

A real kubelet is a separate process; running ``FakeKubelet`` inside the bench's interpreter
makes its gRPC client share one GIL with the bench's pod-fleet pumps, admission service and
fake scheduler, and the kubelet-side Allocate latency it reports then measures that contention,
not the plugin. Here the kubelet's device manager (registration server, ListAndWatch, device-ID
bookkeeping, ``Allocate`` calls and their timing) runs in a child interpreter; the parent
drives it over JSON lines on the child's stdin/stdout. Only the pipe hop is added, outside the
timed RPC.

Child protocol (one JSON object per line, one reply per request)::

    {"op": "admit", "pod": {...}}          -> {"uid", "responses": [b64 ContainerAllocateResponse],
                                               "latencies": [s], "device_ids": [[id]], "error"}
    {"op": "release", "uid": "..."}        -> {"ok": true}
    {"op": "registered", "timeout": s}     -> {"ok": bool}   (wait for Register + first ListAndWatch)
    {"op": "clear_registered"}             -> {"ok": true}
    {"op": "allocated"}                    -> {"ids": [...]}
    {"op": "options"}                      -> {"preferred": bool | null}
"""
from __future__ import annotations

import argparse
import base64
import json
import subprocess
import sys
import threading

from ..api import v1beta1 as api
from .kubelet import Admission


class _Registered:
    """``threading.Event``-shaped view of the child's registration state."""

    def __init__(self, proxy: "KubeletProcess"):
        self._p = proxy

    def wait(self, timeout: float | None = None) -> bool:
        return bool(self._p._call({"op": "registered", "timeout": 30.0 if timeout is None else timeout})["ok"])

    def clear(self):
        self._p._call({"op": "clear_registered"})

    def is_set(self) -> bool:
        return self.wait(0.0)


class _Options:
    def __init__(self, preferred: bool):
        self.get_preferred_allocation_available = preferred


class KubeletProcess:
    """Drop-in for ``FakeKubelet`` in ``SimCluster(kubelet="process")``: admit / release /
    registered / allocated_ids / options. ``serve_pods`` (kubelet pod source) stays in-process
    only."""

    def __init__(self, plugin_dir: str, api_url: str, node: str, env: dict | None = None, preexec_fn=None):
        self.dir, self.api_url, self.node = plugin_dir, api_url, node
        self._env, self._preexec = env, preexec_fn
        self._proc: subprocess.Popen | None = None
        self._mu = threading.Lock()
        self.registered = _Registered(self)

    def start(self) -> "KubeletProcess":
        self._proc = subprocess.Popen(
            [sys.executable, "-m", "aliyun_gpushare_device_plugin_amd.sim.kubelet_proc", "--dir", self.dir,
             "--apiserver", self.api_url, "--node", self.node],
            stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, bufsize=1, env=self._env,
            preexec_fn=self._preexec)
        line = self._proc.stdout.readline()
        if json.loads(line or "{}").get("event") != "listening":
            raise RuntimeError("fake kubelet process failed to start")
        return self

    def _call(self, req: dict) -> dict:
        with self._mu:
            if self._proc is None or self._proc.poll() is not None:
                raise RuntimeError("fake kubelet process is not running")
            self._proc.stdin.write(json.dumps(req) + "\n")
            self._proc.stdin.flush()
            line = self._proc.stdout.readline()
        if not line:
            raise RuntimeError("fake kubelet process exited")
        return json.loads(line)

    def admit(self, pod: dict, timeout: float = 10.0) -> Admission:
        r = self._call({"op": "admit", "pod": pod, "timeout": timeout})
        return Admission(r["uid"], [api.ContainerAllocateResponse.FromString(base64.b64decode(b))
                                    for b in r["responses"]], r["latencies"], r["device_ids"], r["error"],
                         [tuple(x) for x in r.get("splits", [])])

    def release(self, pod_uid: str):
        self._call({"op": "release", "uid": pod_uid})

    def allocated_ids(self) -> set:
        return set(self._call({"op": "allocated"})["ids"])

    @property
    def options(self):
        p = self._call({"op": "options"})["preferred"]
        return None if p is None else _Options(p)

    def stop(self):
        if self._proc is None:
            return
        try:
            self._proc.stdin.close()
        except OSError:
            pass
        try:
            self._proc.wait(timeout=10)
        except subprocess.TimeoutExpired:
            self._proc.kill()
            self._proc.wait(timeout=10)
        self._proc = None


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--dir", required=True)
    ap.add_argument("--apiserver", required=True)
    ap.add_argument("--node", required=True)
    a = ap.parse_args(argv)
    from ..cluster.client import APIClient, KubeConfig
    from .kubelet import FakeKubelet

    kl = FakeKubelet(a.dir, APIClient(KubeConfig(a.apiserver)), a.node).start()
    out = sys.stdout

    def send(obj):
        out.write(json.dumps(obj) + "\n")
        out.flush()

    send({"event": "listening"})
    try:
        for line in sys.stdin:
            req = json.loads(line)
            op = req.get("op")
            if op == "admit":
                adm = kl.admit(req["pod"], timeout=req.get("timeout", 10.0))
                send({"uid": adm.pod_uid, "latencies": adm.latencies, "device_ids": adm.device_ids,
                      "error": adm.error, "splits": adm.splits,
                      "responses": [base64.b64encode(r.SerializeToString()).decode() for r in adm.responses]})
            elif op == "release":
                kl.release(req["uid"])
                send({"ok": True})
            elif op == "registered":
                send({"ok": kl.registered.wait(req.get("timeout", 30.0))})
            elif op == "clear_registered":
                kl.registered.clear()
                send({"ok": True})
            elif op == "allocated":
                send({"ids": sorted(kl.allocated_ids())})
            elif op == "options":
                send({"preferred": None if kl.options is None else bool(kl.options.get_preferred_allocation_available)})
            else:
                send({"error": f"unknown op {op!r}"})
    finally:
        kl.stop()
    return 0


if __name__ == "__main__":
    sys.exit(main())
