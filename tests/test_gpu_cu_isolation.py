"""Compute isolation on a real MI355X: the plugin's CU-slot masks confine a pod's queues.

A pod admitted with ``--compute-isolation=cu`` is run as a child process with exactly its
Allocate environment; the CU census kernel (``native/kernels/census.hip``) then sees
``slots x 8`` distinct CUs, the same count on every XCD, HIP reports that many compute units,
and the MFMA GEMM is still correct on the slice.
"""
import json
import os
import subprocess
import sys

import pytest

from aliyun_gpushare_device_plugin_amd import const

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, torch
from aliyun_gpushare_device_plugin_amd.ops import cu_census, gemm_nt
c = cu_census()
a = torch.randn(512, 256, device="cuda", dtype=torch.bfloat16)
b = torch.randn(768, 256, device="cuda", dtype=torch.bfloat16)
err = (gemm_nt(a, b).float() - a.float() @ b.float().t()).abs().max().item()
print(json.dumps({"mp": torch.cuda.get_device_properties(0).multi_processor_count,
                  "distinct": c["distinct_cus"], "per_xcc": c["per_xcc"], "gemm_err": err}))
"""


def _run(envs: dict) -> dict:
    env = dict(os.environ)
    env.update(envs)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_census_without_mask_sees_every_cu():
    import torch

    from aliyun_gpushare_device_plugin_amd.ops import cu_census

    c = cu_census()
    n = torch.cuda.get_device_properties(0).multi_processor_count
    assert c["distinct_cus"] == n
    assert len(set(c["per_xcc"].values())) == 1          # symmetric over the XCDs


def test_cu_slot_masks_confine_pods_on_mi355x():
    from aliyun_gpushare_device_plugin_amd.sim.cluster import SimCluster

    with SimCluster([("g", "auto")], compute_isolation="cu") as c:
        _, wa, adm_a = c.run_pod(64)                                            # floor(32*64/288) = 7 slots
        _, wb, adm_b = c.run_pod(64, annotations={const.POD_ANNOTATION_CU_SLOTS_REQUEST: "16"})
        assert adm_a.error is None and adm_b.error is None
        envs = [dict(adm_a.responses[0].envs), dict(adm_b.responses[0].envs)]
    assert envs[0][const.ENV_CU_SLOTS] == "0-6" and envs[1][const.ENV_CU_SLOTS] == "7-22"
    for e, slots in zip(envs, (7, 16)):
        got = _run({k: v for k, v in e.items() if k in (const.ENV_HSA_CU_MASK, const.ENV_ROC_CU_MASK)})
        ncu = slots * 8
        assert got["distinct"] == ncu, got
        assert set(got["per_xcc"].values()) == {slots} and len(got["per_xcc"]) == 8, got
        assert got["mp"] == ncu
        assert got["gemm_err"] < 0.5
