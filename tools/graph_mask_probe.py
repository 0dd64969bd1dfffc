#!/usr/bin/env python3
"""Does hipGraph replay stall in a CU-masked process next to a busy neighbour? (profiles/cu_mask)

Run as: graph_mask_probe.py victim|aggressor. The victim times steps of 256 small kernels (a chain
of in-place adds on a 1 MiB tensor), launched eagerly or replayed from one hipGraph; the aggressor
keeps 8192^3 bf16 GEMMs running. The caller sets HSA_CU_MASK per process."""
import json
import os
import sys
import time

import torch

role = sys.argv[1]
seconds = float(os.environ.get("PROBE_SECONDS", "6"))
if role == "aggressor":
    a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    print(json.dumps({"role": role, "ready": True}), flush=True)
    t0 = time.time()
    n = 0
    while time.time() - t0 < seconds + 4:
        for _ in range(4):
            a @ b
        torch.cuda.synchronize()
        n += 4
    print(json.dumps({"role": role, "gemms": n}), flush=True)
    sys.exit(0)

x = torch.zeros(1 << 18, device="cuda")


def body():
    for _ in range(256):
        x.add_(1.0)


body()
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    body()
torch.cuda.current_stream().wait_stream(s)
with torch.cuda.graph(g):
    body()
res = {"role": role, "mask": os.environ.get("HSA_CU_MASK")}
time.sleep(float(os.environ.get("PROBE_DELAY", "0")))
for mode in ("eager", "graph"):
    lat = []
    t0 = time.time()
    while time.time() - t0 < seconds / 2:
        t = time.perf_counter()
        g.replay() if mode == "graph" else body()
        torch.cuda.synchronize()
        lat.append((time.perf_counter() - t) * 1e3)
    lat.sort()
    res[mode + "_ms_p50"] = round(lat[len(lat) // 2], 3)
    res[mode + "_ms_p99"] = round(lat[int(len(lat) * 0.99)], 3)
print(json.dumps(res), flush=True)
