"""Run one flash-attention variant on one shape a few times (for rocprofv3 --pmc passes).
    python tools/diag/attn_pmc_probe.py VARIANT [B S Hq Hkv causal]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from aliyun_gpushare_device_plugin_amd.ops import attention  # noqa: E402
from aliyun_gpushare_device_plugin_amd.ops.attention import set_attention_variant  # noqa: E402


def main():
    a = sys.argv[1:]
    var = int(a[0]) if a else 14
    B, S, Hq, Hkv, causal = (int(x) for x in a[1:6]) if len(a) >= 6 else (16, 2048, 64, 8, 0)
    torch.manual_seed(0)
    q = torch.randn(B, S, Hq, 128, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(B, S, Hkv, 128, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(B, S, Hkv, 128, device="cuda", dtype=torch.bfloat16)
    set_attention_variant(var)
    for _ in range(5):
        attention(q, k, v, causal=bool(causal))
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
