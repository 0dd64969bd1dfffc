set -o pipefail
# a pod's first stream with comgr's whole pipeline cached (libgpushare_comgrcache.so preloaded)
O=gpurun_out/r6ac; mkdir -p $O/cache $O/xdg
L=$PWD/aliyun_gpushare_device_plugin_amd/_native/libgpushare_comgrcache.so
export AMD_COMGR_CACHE=1 AMD_COMGR_CACHE_DIR=$PWD/$O/cache XDG_CACHE_HOME=$PWD/$O/xdg
export GPUSHARE_COMGR_ACTION_CACHE=$PWD/$O/cache GPUSHARE_COMGR_ACTION_CACHE_LOG=1
GPUSHARE_COMGR_ACTION_CACHE_WRITE=1 LD_PRELOAD=$L timeout -k 10 120 python -u tools/diag/first_kernel_split.py > $O/fill.json 2> $O/fill.err &&
LD_PRELOAD=$L timeout -k 10 120 python -u tools/diag/first_kernel_split.py > $O/hit.json 2> $O/hit.err &&
LD_PRELOAD=$L timeout -k 10 120 python -u tools/diag/first_kernel_split.py > $O/hit2.json 2> $O/hit2.err &&
timeout -k 10 120 python -u tools/diag/first_kernel_split.py > $O/comgr_only.json 2> $O/comgr_only.err &&
LD_PRELOAD=$L timeout -k 10 120 python -u -c "
import torch
x = torch.empty(1 << 24, dtype=torch.int32, device='cuda'); x.fill_(7)
y = torch.empty_like(x); y.copy_(x); h = y.cpu()
assert int((h == 7).sum()) == h.numel(), 'blit result'
z = torch.zeros(1 << 20, device='cuda'); assert float(z.abs().sum().item()) == 0.0
print('blit kernels from the cache: results ok')" > $O/check.log 2>&1 &&
ls -la $O/cache > $O/cache_ls.txt
