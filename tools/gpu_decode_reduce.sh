#!/bin/bash
# Split reductions with compile-time split counts and the latency-shaped decode merge: decode tests
# (bitwise static-vs-loop reductions), attention micro-benchmark, and the batch-32 decode step with
# static / loop reductions, order rotated.
set -o pipefail
O=gpurun_out/red
mkdir -p $O
export TMPDIR=/tmp
S="timeout -k 10 300 python -u tools/bench_decode.py --no-attn-micro --no-gemm-micro --gemms skinny_rope"
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 \
 && timeout -k 10 400 python -u tools/bench_decode.py --micro-only --no-gemm-micro > $O/micro.log 2>&1 \
 && $S --reduce-static 1 > $O/step.log 2>&1 \
 && $S --reduce-static 0 >> $O/step.log 2>&1 \
 && $S --reduce-static 0 >> $O/step.log 2>&1 \
 && $S --reduce-static 1 >> $O/step.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
