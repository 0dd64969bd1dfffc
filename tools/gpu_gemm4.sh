#!/bin/bash
# GEMM variant-4 check: numerics tests, then interleaved A/B timing vs v2 and hipBLASLt.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -v -m gpu -k gemm --timeout 120 --timeout-method thread > gpurun_out/gemm4_tests.log 2>&1 \
 && timeout -k 10 300 python -u tools/bench_gemm.py --variants ${VARIANTS:-2,4} --rounds 5 --iters 20 --out gpurun_out/gemm4_bench.json > gpurun_out/gemm4_bench.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
