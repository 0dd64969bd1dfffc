"""Run tools/diag/dmabuf_ref_probe.cpp inside a process that imported torch (not yet using the
GPU), so the tenant's HIP calls go to PyTorch's bundled runtime, the one torch pods use; prints
one JSON line.

    python tools/diag/dmabuf_ref_probe.py [warm: 0|1]
"""
from __future__ import annotations

import ctypes
import json
import os
import sys

import torch

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "build", "libdmabuf_ref_probe.so")


def main() -> int:
    # the runtime library is loaded with torch; the probe forks before either process uses it
    ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"), mode=ctypes.RTLD_GLOBAL)
    lib = ctypes.CDLL(LIB, mode=ctypes.RTLD_GLOBAL)
    lib.dmabuf_ref_probe.restype = ctypes.c_char_p
    lib.dmabuf_ref_probe.argtypes = [ctypes.c_int]
    r = json.loads(lib.dmabuf_ref_probe(int(sys.argv[1]) if len(sys.argv) > 1 else 0))
    r["torch"] = torch.__version__
    r["hip"] = torch.version.hip
    print(json.dumps(r), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
