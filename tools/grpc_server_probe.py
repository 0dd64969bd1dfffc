"""Which grpcio server model answers a sporadic unary RPC fastest: the thread-pool server the
plugin uses, or the asyncio (grpc.aio) server. Both serve the same prepared Allocate answer
(wire bytes, ~1 KB) over a Unix socket; a client in another process calls every ``--gap-ms``
(the kubelet admits pods sporadically) and reports round-trip quantiles.

    python tools/grpc_server_probe.py [--calls 400] [--gap-ms 20]
"""
from __future__ import annotations

import argparse
import asyncio
import concurrent.futures as cf
import json
import multiprocessing as mp
import os
import sys
import tempfile
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from aliyun_gpushare_device_plugin_amd.api import v1beta1 as api  # noqa: E402

RESP = api.AllocateResponse()
_c = RESP.container_responses.add(envs={f"K{i}": "v" * 40 for i in range(8)})
_c.devices.add(container_path="/dev/kfd", host_path="/dev/kfd", permissions="rw")
BODY = RESP.SerializeToString()


class Impl:
    def Allocate(self, request, context):
        return BODY


def serve_sync(path, ready):
    import grpc

    srv = grpc.server(cf.ThreadPoolExecutor(max_workers=16))
    h = grpc.unary_unary_rpc_method_handler(Impl().Allocate, request_deserializer=api.AllocateRequest.FromString,
                                            response_serializer=lambda b: b)
    srv.add_generic_rpc_handlers((grpc.method_handlers_generic_handler("v1beta1.DevicePlugin", {"Allocate": h}),))
    srv.add_insecure_port("unix://" + path)
    srv.start()
    ready.set()
    srv.wait_for_termination()


def serve_aio(path, ready):
    import grpc

    async def main():
        srv = grpc.aio.server()

        async def alloc(request, context):
            return BODY
        h = grpc.unary_unary_rpc_method_handler(alloc, request_deserializer=api.AllocateRequest.FromString,
                                                response_serializer=lambda b: b)
        srv.add_generic_rpc_handlers((grpc.method_handlers_generic_handler("v1beta1.DevicePlugin", {"Allocate": h}),))
        srv.add_insecure_port("unix://" + path)
        await srv.start()
        ready.set()
        await srv.wait_for_termination()
    asyncio.run(main())


def client(path, calls, gap, q):
    import grpc

    ch = grpc.insecure_channel("unix://" + path)
    grpc.channel_ready_future(ch).result(timeout=10)
    stub = ch.unary_unary("/v1beta1.DevicePlugin/Allocate", request_serializer=api.AllocateRequest.SerializeToString,
                          response_deserializer=api.AllocateResponse.FromString)
    req = api.AllocateRequest(container_requests=[api.ContainerAllocateRequest(
        devices_ids=[f"GPU-0123456789abcdef-_-{i}" for i in range(64)])])
    for _ in range(20):
        stub(req)
    lat = []
    for _ in range(calls):
        time.sleep(gap)
        t = time.perf_counter()
        stub(req)
        lat.append(time.perf_counter() - t)
    lat.sort()
    q.put({"p50_ms": round(lat[len(lat) // 2] * 1e3, 3), "p90_ms": round(lat[int(len(lat) * 0.9)] * 1e3, 3)})


def burner(stop):
    while not stop.is_set():
        sum(i * i for i in range(2000))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=400)
    ap.add_argument("--gap-ms", type=float, default=20.0)
    ap.add_argument("--busy-threads", type=int, default=1, help="CPU-bound threads inside the server process")
    ap.add_argument("--models", default="sync,aio", help="server models to measure")
    ap.add_argument("--switch-interval", type=float, default=0.00025,
                    help="server process GIL switch interval (the plugin's default)")
    a = ap.parse_args()
    out = {}
    models = {"sync": serve_sync, "aio": serve_aio}
    for name, fn in ((m, models[m]) for m in a.models.split(",")):
        path = os.path.join(tempfile.mkdtemp(prefix="gsp-"), "s.sock")
        ready = mp.Event()
        srv = mp.Process(target=_with_burners, args=(fn, path, ready, a.busy_threads, a.switch_interval), daemon=True)
        srv.start()
        ready.wait(20)
        q = mp.Queue()
        c = mp.Process(target=client, args=(path, a.calls, a.gap_ms / 1e3, q))
        c.start()
        out[name] = q.get(timeout=300)
        c.join()
        srv.terminate()
    print(json.dumps({"gap_ms": a.gap_ms, "busy_threads": a.busy_threads, **out}))


def _with_burners(fn, path, ready, n, switch_interval):
    sys.setswitchinterval(switch_interval)
    stop = threading.Event()
    for _ in range(n):
        threading.Thread(target=burner, args=(stop,), daemon=True).start()
    fn(path, ready)


if __name__ == "__main__":
    main()
