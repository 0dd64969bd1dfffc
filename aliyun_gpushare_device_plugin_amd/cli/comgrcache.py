"""``gpushare-comgr-cache``: fill and seal the node's comgr cache (the DaemonSet's init container;
``quota/comgr_cache.py``).

    gpushare-comgr-cache --dir /var/lib/gpushare/comgr-cache [--runtimes system,torch] [--device 0]

Prints one JSON line. The cache only saves start-up time, so a runtime that cannot be warmed
(no PyTorch in the image, no GPU free) does not fail the DaemonSet: the cache is sealed with what
the others left, and the pods of that runtime compile as they would without it. ``--strict``
exits 1 when no runtime filled it.
"""
from __future__ import annotations

import argparse
import json
import sys

from ..quota import comgr_cache


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="gpushare-comgr-cache", description=__doc__.splitlines()[0])
    ap.add_argument("--dir", required=True, help="the cache directory on the host (the plugin's --comgr-cache-dir)")
    ap.add_argument("--runtimes", default=",".join(comgr_cache.RUNTIMES),
                    help="HIP runtimes whose first-stream kernels to cache (system = /opt/rocm, torch = PyTorch's)")
    ap.add_argument("--device", type=int, default=0, help="the GPU the warm-up runs on (any of the node's)")
    ap.add_argument("--keep", action="store_true", help="add to the existing cache instead of starting empty")
    ap.add_argument("--strict", action="store_true", help="exit 1 when no runtime filled the cache")
    a = ap.parse_args(argv)
    rts = tuple(r for r in a.runtimes.split(",") if r)
    res = comgr_cache.warm(a.dir, rts, device=a.device, fresh=not a.keep)
    comgr_cache.seal(a.dir)
    res["sealed"] = True
    print(json.dumps(res), flush=True)
    return 1 if a.strict and not any(r.get("ok") for r in res["runtimes"].values()) else 0


if __name__ == "__main__":
    sys.exit(main())
