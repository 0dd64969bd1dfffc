#!/bin/bash
# 4-wave GEMM with the K offset in the VGPR offset as the default: GEMM + model tests, then the
# sweep against the scalar-offset schedule (12) and hipBLASLt.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
true \
 && timeout -k 10 500 python -u tools/gemm_sched_sweep.py --scheds 0,12,9 --rounds 12 --shapes 4096x4096x4096,4096x4096x1024,8192x8192x8192,4096x4096x14336,4096x14336x4096 --out gpurun_out/gemm_kv_sweep3.json > gpurun_out/gemm_kv_sweep3.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
