"""Attention diagnosis: tr-read path vs gather path vs fp32 reference, plus structured inputs."""
import torch, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from aliyun_gpushare_device_plugin_amd.ops import attention, reference_attention
torch.manual_seed(0)
for (B,S,H,D) in [(1,64,1,128),(1,64,4,128),(1,256,2,128),(1,64,1,64)]:
    q=torch.randn(B,S,H,D,device="cuda",dtype=torch.bfloat16)
    k=torch.randn(B,S,H,D,device="cuda",dtype=torch.bfloat16)
    v=torch.randn(B,S,H,D,device="cuda",dtype=torch.bfloat16)
    ref=reference_attention(q,k,v,True)
    for dbg in (False, True):
        o=attention(q,k,v,True,_debug_gather=dbg)
        print((B,S,H,D),"gather" if dbg else "tr", "maxerr", (o.float()-ref).abs().max().item(), flush=True)
# uniform attention (q=k=0): row i -> mean(V[0..i]); V[j][d] = j (row id) to read the mixing
S,D=64,128
q=torch.zeros(1,S,1,D,device="cuda",dtype=torch.bfloat16); k=torch.zeros_like(q)
v=torch.arange(S,device="cuda",dtype=torch.float32)[None,:,None,None].expand(1,S,1,D).to(torch.bfloat16).contiguous()
o=attention(q,k,v,True)
print("uniform rows 0..7 col0:", o[0,:8,0,0].float().tolist(), "expect", [i/2 for i in range(8)])
v2=torch.arange(D,device="cuda",dtype=torch.float32)[None,None,None,:].expand(1,S,1,D).to(torch.bfloat16).contiguous()
o2=attention(q,k,v2,True)
print("uniform row 5 cols 0..20:", o2[0,5,:20,0].float().tolist() if False else o2[0,5,0,:20].float().tolist())
