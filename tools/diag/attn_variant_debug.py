"""Where a flash-attention kernel variant disagrees with the fp32 reference: per shape, the max
error, the first bad query rows and head dims, and whether rows with only a few visible keys
differ. python tools/diag/attn_variant_debug.py VARIANT"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from aliyun_gpushare_device_plugin_amd.ops import attention, reference_attention  # noqa: E402
from aliyun_gpushare_device_plugin_amd.ops.attention import ATTN_AUTO, set_attention_variant  # noqa: E402


def main():
    var = int(sys.argv[1]) if len(sys.argv) > 1 else 14
    for (B, S, Hq, Hkv, causal, kind) in [(1, 32, 1, 1, False, "randn"), (1, 64, 1, 1, False, "randn"),
                                           (1, 32, 1, 1, False, "vconst"), (1, 64, 1, 1, False, "vconst"),
                                           (1, 64, 1, 1, False, "qzero"), (1, 256, 1, 1, False, "randn"),
                                           (1, 64, 1, 1, True, "randn"), (1, 300, 2, 1, True, "randn")]:
        torch.manual_seed(0)
        q = torch.randn(B, S, Hq, 128, device="cuda", dtype=torch.bfloat16)
        k = torch.randn(B, S, Hkv, 128, device="cuda", dtype=torch.bfloat16)
        v = torch.randn(B, S, Hkv, 128, device="cuda", dtype=torch.bfloat16)
        if kind == "vconst":        # V[key][d] = key index: the output row is the softmax-weighted key
            v = torch.arange(S, device="cuda", dtype=torch.float32)[None, :, None, None].expand(B, S, Hkv, 128)
            v = v.to(torch.bfloat16).contiguous() / S
        if kind == "qzero":         # uniform attention: output = mean of visible V rows
            q = torch.zeros_like(q)
        ref = reference_attention(q, k, v, causal=causal)
        set_attention_variant(var)
        out = attention(q, k, v, causal=causal).float()
        set_attention_variant(ATTN_AUTO)
        err = (out - ref).abs()
        row_err = err.amax(dim=(0, 2, 3))
        col_err = err.amax(dim=(0, 1, 2))
        bad_rows = (row_err > 3e-2).nonzero().flatten().tolist()
        bad_cols = (col_err > 3e-2).nonzero().flatten().tolist()
        print(json.dumps({"shape": [B, S, Hq, Hkv], "causal": causal, "kind": kind,
                          "max_err": round(err.max().item(), 4), "bad_rows": bad_rows[:16], "n_bad_rows": len(bad_rows),
                          "bad_cols": bad_cols[:16], "n_bad_cols": len(bad_cols),
                          "row0_out": [round(x, 3) for x in out[0, 0, 0, :6].tolist()],
                          "row0_ref": [round(x, 3) for x in ref[0, 0, 0, :6].tolist()],
                          "nan": bool(torch.isnan(out).any())}), flush=True)


if __name__ == "__main__":
    main()
