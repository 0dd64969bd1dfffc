"""Which XCDs / CUs does this process's queue actually run on? (``native/kernels/census.hip``)

Used to check compute isolation on hardware: a container admitted with a CU-slot run
(``alloc/cuslots.py``) must see exactly ``slots x 8`` distinct CUs, the same number on every XCD.
"""
from __future__ import annotations

import torch

from . import _lib


def cu_census(nblocks: int = 4096, spin: int = 4, device=None) -> dict:
    """Launch ``nblocks`` sleeping workgroups on the current stream and report where they ran:
    ``{"distinct_cus": n, "per_xcc": {xcc: n_cus}, "cus": sorted [(xcc, se, cu)]}``."""
    out = torch.empty(nblocks, dtype=torch.int32, device=device or "cuda")
    _lib.check(_lib.lib().gs_cu_census(out.data_ptr(), nblocks, spin, _lib.stream_ptr(out.device)), "gs_cu_census")
    vals = out.cpu().tolist()
    cus = set()
    for v in vals:
        v &= 0xffffffff
        xcc, se, sh, cu = v >> 16, (v >> 13) & 3, (v >> 12) & 1, (v >> 8) & 15
        cus.add((xcc, se * 2 + sh, cu))
    per: dict[int, int] = {}
    for x, _, _ in cus:
        per[x] = per.get(x, 0) + 1
    return {"distinct_cus": len(cus), "per_xcc": dict(sorted(per.items())), "cus": sorted(cus)}
