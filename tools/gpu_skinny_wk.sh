#!/bin/bash
# Skinny GEMM schedules (1 = one k-slice in flight, 2 = two, 3 = wave-level K split, 4 = 1 with nt W loads):
# the GEMM micro-benchmark order-rotated, and the Llama-3-8B batch-32 decode step per schedule.
set -o pipefail
mkdir -p gpurun_out/nt2
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/nt2/tests.log 2>&1 \
 && timeout -k 10 400 python -u tools/bench_decode.py --micro-only --no-attn-micro > gpurun_out/nt2/micro.log 2>&1 \
 && timeout -k 10 300 python -u tools/bench_decode.py --no-attn-micro --no-gemm-micro --gemms skinny_rope --prefetch 1 > gpurun_out/nt2/step.log 2>&1 \
 && timeout -k 10 300 python -u tools/bench_decode.py --no-attn-micro --no-gemm-micro --gemms skinny_rope --prefetch 4 >> gpurun_out/nt2/step.log 2>&1 \
 && timeout -k 10 300 python -u tools/bench_decode.py --no-attn-micro --no-gemm-micro --gemms skinny_rope --prefetch 1 >> gpurun_out/nt2/step.log 2>&1 \
 && timeout -k 10 300 python -u tools/bench_decode.py --no-attn-micro --no-gemm-micro --gemms skinny_rope --prefetch 4 >> gpurun_out/nt2/step.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
