"""Run tools/diag/vmm_semantics_probe.cpp inside a process that imported torch, so the probe's
HIP calls go to PyTorch's bundled runtime (the one torch pods use); prints one JSON line.

    python tools/diag/vmm_semantics_probe.py [granule MiB]
"""
from __future__ import annotations

import ctypes
import json
import os
import sys

import torch

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "build", "libvmm_semantics_probe.so")


def main() -> int:
    torch.zeros(1, device="cuda")              # the runtime is loaded and the device is up
    lib = ctypes.CDLL(LIB, mode=ctypes.RTLD_GLOBAL)
    lib.vmm_semantics_probe.restype = ctypes.c_char_p
    r = json.loads(lib.vmm_semantics_probe(ctypes.c_ulonglong(int(sys.argv[1]) if len(sys.argv) > 1 else 1024)))
    r["torch"] = torch.__version__
    r["hip"] = torch.version.hip
    print(json.dumps(r), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
