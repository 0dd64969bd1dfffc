"""How much of a kubelet-side Allocate round trip is the transport waking up after idle.

Measures, against the real plugin process (fake kubelet's channel, ``SimCluster``):
* a raw UDS ping-pong between two processes (the OS's own wake-up cost);
* an empty gRPC call (``GetDevicePluginOptions``) — the same client/server path as Allocate,
  with no plugin work;
* ``Allocate`` itself is in the bench's A/B (``allocate_by_mode``);
each back to back and after idle gaps of 1 / 5 / 20 / 50 ms (admissions arrive sporadically:
one per pod start). Prints one JSON object.
"""
from __future__ import annotations

import json
import os
import socket
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

GAPS = (0.0, 0.001, 0.005, 0.02, 0.05)


def _p50(xs):
    xs = sorted(xs)
    return round(xs[len(xs) // 2] * 1e3, 3)


def raw_uds(n: int = 60) -> dict:
    a, b = socket.socketpair()
    pid = os.fork()
    if pid == 0:                                   # no GPU in this process: plain fork is fine
        a.close()
        while True:
            d = b.recv(64)
            if not d:
                os._exit(0)
            b.send(d)
    b.close()
    out = {}
    for gap in GAPS:
        ts = []
        for _ in range(n):
            if gap:
                time.sleep(gap)
            t = time.perf_counter()
            a.send(b"x")
            a.recv(64)
            ts.append(time.perf_counter() - t)
        out[f"{gap * 1e3:g}ms"] = _p50(ts)
    a.close()
    os.waitpid(pid, 0)
    return out


def grpc_empty(n: int = 60) -> dict:
    from aliyun_gpushare_device_plugin_amd.api import v1beta1 as api
    from aliyun_gpushare_device_plugin_amd.sim.cluster import SimCluster

    out = {}
    with SimCluster([("n", "fake:1x288G")], plugin_mode="process", apiserver="process") as c:
        stub = c.nodes["n"].kubelet._stub
        for gap in GAPS:
            ts = []
            for _ in range(n):
                if gap:
                    time.sleep(gap)
                t = time.perf_counter()
                stub.GetDevicePluginOptions(api.Empty(), timeout=5)
                ts.append(time.perf_counter() - t)
            out[f"{gap * 1e3:g}ms"] = _p50(ts)
    return out


def main() -> int:
    res = {"probe": "transport wake-up after idle (p50 round trip, ms, by idle gap)",
           "raw_uds_pingpong": raw_uds(), "grpc_empty_call": grpc_empty()}
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())
