#!/bin/bash
# Skinny GEMM default schedule (auto: non-temporal W in unsplit grids): agreement tests, the GEMM
# micro-benchmark with HBM-resident weights, and the batch-32 decode step auto / 1 / 4 rotated.
set -o pipefail
mkdir -p gpurun_out/auto2
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/auto2/tests.log 2>&1 \
 && timeout -k 10 400 python -u tools/bench_decode.py --micro-only --no-attn-micro > gpurun_out/auto2/micro.log 2>&1 \
 && timeout -k 10 300 python -u tools/bench_decode.py --no-attn-micro --no-gemm-micro --gemms skinny_rope --prefetch 0 > gpurun_out/auto2/step.log 2>&1 \
 && timeout -k 10 300 python -u tools/bench_decode.py --no-attn-micro --no-gemm-micro --gemms skinny_rope --prefetch 1 >> gpurun_out/auto2/step.log 2>&1 \
 && timeout -k 10 300 python -u tools/bench_decode.py --no-attn-micro --no-gemm-micro --gemms skinny_rope --prefetch 4 >> gpurun_out/auto2/step.log 2>&1 \
 && timeout -k 10 300 python -u tools/bench_decode.py --no-attn-micro --no-gemm-micro --gemms hipblaslt,skinny_rope --prefetch 0 >> gpurun_out/auto2/step.log 2>&1 \
 && timeout -k 10 300 python -u tools/bench_decode.py --no-attn-micro --no-gemm-micro --gemms skinny_rope --prefetch 4 >> gpurun_out/auto2/step.log 2>&1 \
 && timeout -k 10 300 python -u tools/bench_decode.py --no-attn-micro --no-gemm-micro --gemms skinny_rope --prefetch 1 >> gpurun_out/auto2/step.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
