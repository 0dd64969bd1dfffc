#!/bin/bash
# (Historical: schedule 5 was measured slower and removed, profiles/decode/skinny_pf5_r3_*.jsonl; the
# library now refuses --prefetch 5.)
# Skinny schedule 5 (two k-slices in flight, W non-temporal) vs auto / 4: agreement tests, the GEMM
# micro-benchmark with HBM-streamed weights, and the batch-32 decode step (auto / 5 / 5 / auto).
set -o pipefail
O=gpurun_out/pf5
mkdir -p $O
export TMPDIR=/tmp
S="timeout -k 10 300 python -u tools/bench_decode.py --no-attn-micro --no-gemm-micro --gemms skinny_rope"
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 \
 && timeout -k 10 600 python -u tools/bench_decode.py --micro-only --no-attn-micro > $O/micro.log 2>&1 \
 && $S --prefetch 0 > $O/step.log 2>&1 \
 && $S --prefetch 5 >> $O/step.log 2>&1 \
 && $S --prefetch 5 >> $O/step.log 2>&1 \
 && $S --prefetch 0 >> $O/step.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
