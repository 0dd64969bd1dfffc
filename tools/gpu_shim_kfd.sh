#!/bin/bash
# Quota shim at the KFD boundary on MI355X (exploration, round 2): scratch alloc/free trace,
# hipMalloc denial at a small quota, PyTorch under the shim, the shim GPU tests; last, the
# pool-allocation OOM path under the shim and under a real HBM exhaustion (no shim).
set -o pipefail
mkdir -p gpurun_out/shim
export TMPDIR=/tmp
S=$PWD/aliyun_gpushare_device_plugin_amd/_native
SHIM=$S/libgpushare_hipquota.so
timeout -k 10 90 env LD_PRELOAD=$SHIM GPUSHARE_QUOTA_BYTES=$((64<<30)) GPUSHARE_SHIM_LOG=2 \
    $S/shim_probe scratch 4 scratch 16 scratch 4 > gpurun_out/shim/probe_scratch.log 2>&1 \
 && timeout -k 10 90 env LD_PRELOAD=$SHIM GPUSHARE_QUOTA_BYTES=$((768<<20)) GPUSHARE_SHIM_LOG=1 \
    $S/shim_probe alloc 268435456 alloc 1073741824 alloc 268435456 > gpurun_out/shim/probe_small.log 2>&1 \
 && timeout -k 10 120 env GPUSHARE_SHIM_LOG=1 ALIYUN_COM_GPU_MEM_CONTAINER=64 ALIYUN_COM_GPU_MEM_DEV=288 LD_PRELOAD=$SHIM \
    python -c "
import torch, json
f, t = torch.cuda.mem_get_info()
x = torch.empty(int(t * 0.8) // 2, dtype=torch.bfloat16, device='cuda')
try:
    y = torch.empty(int(t * 0.5) // 2, dtype=torch.bfloat16, device='cuda'); r = 'allowed'
except torch.OutOfMemoryError as e:
    r = 'denied'
del x; torch.cuda.empty_cache()
z = torch.empty(int(t * 0.9) // 2, dtype=torch.bfloat16, device='cuda')
print(json.dumps({'free': f, 'total': t, 'over': r, 'after_free': True}))
" > gpurun_out/shim/torch.log 2>&1 \
 && timeout -k 10 300 python -u -m pytest tests/test_gpu_native.py -x -v -m gpu --timeout 120 --timeout-method thread -k shim > gpurun_out/shim/pytest.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
