"""One tiny end-to-end slice (SURVEY §7.3 minimum slice), used by ``__graft_entry__.smoke``:

1. the real plugin enumerates the MI355X through libgpushare_gpuinfo and registers with the
   fake kubelet; the node advertises its ``aliyun.com/gpu-mem`` units and ``gpu-count``;
2. the extender stand-in assumes an 8 GiB pod, the kubelet calls ``Allocate`` over gRPC/UDS,
   the plugin answers with the env contract + ``/dev/kfd`` + render node and patches
   ``ASSIGNED=true``;
3. the pod's workload runs on ``cuda:0``: one forward + backward of a bf16 linear layer on the
   hand-written MFMA GEMM, checked against an fp32 PyTorch reference.
"""
from __future__ import annotations

import json
import time


def run_smoke(verbose: bool = True) -> dict:
    import torch

    from . import const
    from .cluster import objects as O
    from .ops import linear_autograd, rmsnorm
    from .ops import _lib
    from .sim.cluster import SimCluster

    t0 = time.time()
    out = {}
    with SimCluster([("smoke-node", "auto")]) as c:
        node = c.client.get_node("smoke-node")
        out["gpu_count"] = O.node_allocatable(node, const.RESOURCE_COUNT)
        out["gpu_mem_units"] = O.node_allocatable(node, const.RESOURCE_NAME)
        pod, where, adm = c.run_pod(8)
        assert adm is not None and adm.error is None, adm and adm.error
        envs = dict(adm.responses[0].envs)
        out["allocate_ms"] = round(adm.latencies[0] * 1e3, 3)
        out["envs"] = {k: v for k, v in envs.items() if k.startswith("ALIYUN")}
        out["devices"] = [d.host_path for d in adm.responses[0].devices]
        assert O.annotations(c.wait_assigned(pod))[const.ENV_ASSIGNED_FLAG] == "true"

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    x = torch.randn(128, 256, device=dev, dtype=torch.bfloat16, requires_grad=True)
    w = (torch.randn(512, 256, device=dev, dtype=torch.bfloat16) * 0.05).requires_grad_()
    y = linear_autograd(x, w)
    loss = y.float().pow(2).mean()
    loss.backward()
    torch.cuda.synchronize()
    xr, wr = x.detach().float().requires_grad_(), w.detach().float().requires_grad_()
    (xr @ wr.t()).pow(2).mean().backward()
    fwd_err = (y.float() - (xr @ wr.t())).abs().max().item()
    gx_err = (x.grad.float() - xr.grad).abs().max().item() / (xr.grad.abs().max().item() + 1e-12)
    gw_err = (w.grad.float() - wr.grad).abs().max().item() / (wr.grad.abs().max().item() + 1e-12)
    assert fwd_err < 0.1 and gx_err < 0.05 and gw_err < 0.05, (fwd_err, gx_err, gw_err)
    gain = torch.rand(512, device=dev, dtype=torch.bfloat16) + 0.5
    z = rmsnorm(y.detach().contiguous(), gain)
    yf = y.detach().float()
    zr = yf * torch.rsqrt(yf.pow(2).mean(-1, keepdim=True) + 1e-5) * gain.float()
    norm_err = (z.float() - zr).abs().max().item()
    assert norm_err < 0.1, norm_err
    out["rmsnorm_max_abs_err"] = norm_err
    out.update(fwd_max_abs_err=fwd_err, grad_x_rel_err=gx_err, grad_w_rel_err=gw_err,
               kernels_lib=_lib.lib()._name, seconds=round(time.time() - t0, 2))
    if verbose:
        print(json.dumps(out))
    return out


if __name__ == "__main__":
    run_smoke()
