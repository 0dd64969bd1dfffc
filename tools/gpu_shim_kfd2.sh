#!/bin/bash
# Quota shim exploration, part 2: where small allocations' HBM comes from (KFD trace), and the
# stream-ordered pool's out-of-memory path under a real HBM exhaustion (no shim) vs the shim.
set -o pipefail
mkdir -p gpurun_out/shim
export TMPDIR=/tmp
S=$PWD/aliyun_gpushare_device_plugin_amd/_native
SHIM=$S/libgpushare_hipquota.so
timeout -k 10 90 env LD_PRELOAD=$SHIM GPUSHARE_QUOTA_BYTES=$((64<<30)) GPUSHARE_SHIM_LOG=2 \
    $S/shim_probe granule smalls 100 4096 smalls 10 65536 smalls 20 3145728 > gpurun_out/shim/probe_granule.log 2>&1 \
 && timeout -k 10 120 $S/shim_probe fill 536870912 pool 1073741824 alloc 268435456 > gpurun_out/shim/probe_realoom.log 2>&1 \
 && timeout -k 10 90 env LD_PRELOAD=$SHIM GPUSHARE_QUOTA_BYTES=$((768<<20)) GPUSHARE_SHIM_LOG=2 \
    $S/shim_probe alloc 268435456 pool 1073741824 alloc 268435456 > gpurun_out/shim/probe_pool_quota.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
