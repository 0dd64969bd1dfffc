#!/bin/bash
# Skinny GEMM k-slices in flight (1 vs 2): bitwise agreement tests, the GEMM micro-benchmark with
# both depths order-rotated, and the Llama-3-8B batch-32 decode step at each depth (pf 1, 2, 1).
set -o pipefail
mkdir -p gpurun_out/pf
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pf/tests.log 2>&1 \
 && timeout -k 10 400 python -u tools/bench_decode.py --micro-only --no-attn-micro --out gpurun_out/pf/micro.jsonl > gpurun_out/pf/micro.log 2>&1 \
 && timeout -k 10 300 python -u tools/bench_decode.py --no-attn-micro --no-gemm-micro --gemms skinny_rope --prefetch 1 --out gpurun_out/pf/step_pf1a.jsonl > gpurun_out/pf/step.log 2>&1 \
 && timeout -k 10 300 python -u tools/bench_decode.py --no-attn-micro --no-gemm-micro --gemms skinny_rope --prefetch 2 --out gpurun_out/pf/step_pf2.jsonl >> gpurun_out/pf/step.log 2>&1 \
 && timeout -k 10 300 python -u tools/bench_decode.py --no-attn-micro --no-gemm-micro --gemms skinny_rope --prefetch 1 --out gpurun_out/pf/step_pf1b.jsonl >> gpurun_out/pf/step.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
