#!/usr/bin/env python3
"""Where does a GEMM lose time at kernel boundaries? Event-timed, 20 GEMMs per measurement:

* ``same``: 20 launches on one stream (each dispatch waits for the previous one to finish);
* ``two_streams``: the same 20 launches alternating between two streams joined by events at the
  ends, so a dispatch may start while its predecessor drains (writes to separate outputs);
* ``one_dispatch``: ours only, the 20 GEMMs as grid.y = 20 of one dispatch (gemm_nt_repeat).

If ``two_streams`` or ``one_dispatch`` is much faster than ``same``, the per-launch fixed cost is
the drain/fill at the kernel boundary, not time inside the kernel
(profiles/gemm_kernel_trace_4096.md). Prints one JSON line per shape.
"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from aliyun_gpushare_device_plugin_amd.ops import gemm_nt  # noqa: E402
from aliyun_gpushare_device_plugin_amd.ops.gemm import gemm_nt_repeat  # noqa: E402

N_GEMM = 20


def timed(fn):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / N_GEMM


def main():
    shapes = sys.argv[1] if len(sys.argv) > 1 else "4096x4096x4096,4096x4096x1024,8192x8192x8192"
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for shape in shapes.split(","):
        M, N, K = map(int, shape.split("x"))
        a = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        b = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        c = [torch.empty(M, N, device="cuda", dtype=torch.bfloat16) for _ in range(2)]
        kern = {"ours": lambda o: gemm_nt(a, b, out=o), "torch": lambda o: torch.matmul(a, b.t(), out=o)}

        def same(k):
            return lambda: [kern[k](c[i & 1]) for i in range(N_GEMM)]

        def two(k):
            def f():
                cur = torch.cuda.current_stream()
                s1.wait_stream(cur)
                s2.wait_stream(cur)
                for i in range(N_GEMM):
                    with torch.cuda.stream(s1 if i & 1 else s2):
                        kern[k](c[i & 1])
                cur.wait_stream(s1)
                cur.wait_stream(s2)
            return f

        fns = {"ours_same": same("ours"), "ours_two_streams": two("ours"),
               "ours_one_dispatch": lambda: gemm_nt_repeat(a, b, c[0], N_GEMM),
               "torch_same": same("torch"), "torch_two_streams": two("torch")}
        for f in fns.values():
            f()
        row = {"shape": [M, N, K]}
        res = {k: [] for k in fns}
        for _ in range(5):
            for k, f in fns.items():
                res[k].append(timed(f))
        flop = 2.0 * M * N * K
        for k, v in res.items():
            us = statistics.median(v)
            row[k + "_us"] = round(us, 1)
            row[k + "_tflops"] = round(flop / us / 1e6, 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
