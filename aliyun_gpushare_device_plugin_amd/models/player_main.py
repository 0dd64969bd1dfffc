"""Container entry point of the MI355X ``gpu-player`` (bin-pack demo pod).

Reads its share from the Allocate env contract (``ALIYUN_COM_GPU_MEM_CONTAINER`` /
``_DEV``; the quota shim enforces the same numbers), allocates it and drives MFMA GEMMs,
printing achieved TFLOP/s periodically.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gemm", type=int, default=4096)
    ap.add_argument("--burst", type=int, default=50)
    ap.add_argument("--seconds", type=float, default=0.0, help="0 = run forever")
    ap.add_argument("--touch-fraction", type=float, default=0.8)
    a = ap.parse_args(argv)

    import torch

    from .gemm_player import GemmPlayer

    free, total = torch.cuda.mem_get_info()      # = the quota under the shim
    ctr = int(os.environ.get("ALIYUN_COM_GPU_MEM_CONTAINER", "0") or 0)
    dev = int(os.environ.get("ALIYUN_COM_GPU_MEM_DEV", "0") or 0)
    share = total * ctr // dev if ctr and dev else total
    share = min(share, free)
    p = GemmPlayer(share, 0, a.gemm, a.gemm, a.gemm, touch_fraction=a.touch_fraction)
    print(json.dumps({"event": "start", "share_bytes": p.share_bytes, "device_total_seen": total}), flush=True)
    t0 = last = time.perf_counter()
    flops = 0.0
    while a.seconds <= 0 or time.perf_counter() - t0 < a.seconds:
        p.run(a.burst)
        p.synchronize()
        flops += 2.0 * a.gemm ** 3 * a.burst
        now = time.perf_counter()
        if now - last >= 10:
            print(json.dumps({"event": "progress", "tflops": flops / (now - t0) / 1e12}), flush=True)
            last = now
    print(json.dumps({"event": "done", "tflops": flops / (time.perf_counter() - t0) / 1e12}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
