#!/bin/bash
# Quota shim at the KFD boundary, validation: shim GPU tests, a rocprofv3 memory-allocation
# trace of the probe under the shim (the profiler's view of every allocation next to the shim
# ledger's), then (last, exploratory) a scratch-heavy kernel whose scratch exceeds the quota.
set -o pipefail
mkdir -p gpurun_out/shim/rocprof
export TMPDIR=/tmp
S=$PWD/aliyun_gpushare_device_plugin_amd/_native
SHIM=$S/libgpushare_hipquota.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_native.py -x -v -m gpu --timeout 120 --timeout-method thread -k shim > gpurun_out/shim/pytest.log 2>&1 \
 && (export LD_PRELOAD=$SHIM GPUSHARE_QUOTA_BYTES=$((64<<30)) GPUSHARE_SHIM_LOG=2; cd /tmp && timeout -k 10 120 rocprofv3 --memory-allocation-trace --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/shim/rocprof -o shim -- $S/shim_probe pool 1073741824 scratch 4 alloc 67108864 > $GRAFT_REPO_ROOT/gpurun_out/shim/rocprof/probe.log 2>&1) \
 && timeout -k 10 60 env LD_PRELOAD=$SHIM GPUSHARE_QUOTA_BYTES=$((1<<30)) GPUSHARE_SHIM_LOG=1 $S/shim_probe scratch 16 alloc 67108864 > gpurun_out/shim/probe_scratch_over.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
