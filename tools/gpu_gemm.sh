#!/bin/bash
# GEMM session: numerics of both kernels, then v2 (ping-pong) vs v1 vs hipBLASLt.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_ops.py -x -q > gpurun_out/gpu_ops.log 2>&1 \
 && timeout -k 10 300 python tools/bench_gemm.py --rounds 5 --iters 20 --out gpurun_out/gemm_bench.json > gpurun_out/gemm_bench.log 2>&1
rc=$?
echo "rc=$rc"
tail -n 5 gpurun_out/gpu_ops.log
cat gpurun_out/gemm_bench.log 2>/dev/null | tail -n 8
exit $rc
