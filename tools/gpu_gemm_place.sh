#!/bin/bash
# 4-wave GEMM: MFMA-slot placement of the DMA and fragment reads (schedules 13-15 vs 0), bitwise
# tests, then an order-rotated sweep against hipBLASLt.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu -k "w4_schedules" --timeout 120 --timeout-method thread > gpurun_out/gemm_place_tests.log 2>&1 \
 && timeout -k 10 600 python -u tools/gemm_sched_sweep.py --scheds 0,13,14,15 --rounds 12 --shapes 4096x4096x4096,4096x4096x1024,8192x8192x8192,4096x4096x14336 --out gpurun_out/gemm_place_sweep.json > gpurun_out/gemm_place_sweep.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
