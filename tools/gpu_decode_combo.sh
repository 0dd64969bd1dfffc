#!/bin/bash
# Decode path load policies in one box session: agreement tests; micro-benchmarks (attention caches and
# GEMM weights > 1 GB, rotated, so both stream from HBM); the batch-32 Llama-3-8B decode step with the
# skinny schedule (auto / 1) and the attention K/V policy (plain / nt), order rotated.
set -o pipefail
O=gpurun_out/combo
mkdir -p $O
export TMPDIR=/tmp
S="timeout -k 10 300 python -u tools/bench_decode.py --no-attn-micro --no-gemm-micro --gemms skinny_rope"
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 \
 && timeout -k 10 600 python -u tools/bench_decode.py --micro-only > $O/micro.log 2>&1 \
 && $S --prefetch 0 --attn-nt 0 > $O/step.log 2>&1 \
 && $S --prefetch 0 --attn-nt 1 >> $O/step.log 2>&1 \
 && $S --prefetch 1 --attn-nt 0 >> $O/step.log 2>&1 \
 && $S --prefetch 1 --attn-nt 0 >> $O/step.log 2>&1 \
 && $S --prefetch 0 --attn-nt 1 >> $O/step.log 2>&1 \
 && $S --prefetch 0 --attn-nt 0 >> $O/step.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
