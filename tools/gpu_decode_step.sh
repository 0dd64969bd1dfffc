#!/bin/bash
# Decode tests, then the batch-32 decode step twice (skinny) and once with hipBLASLt projections.
set -o pipefail
O=gpurun_out/${1:-step}
mkdir -p $O
export TMPDIR=/tmp
S="timeout -k 10 300 python -u tools/bench_decode.py --no-attn-micro --no-gemm-micro"
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 \
 && $S --gemms skinny_rope,hipblaslt > $O/step.log 2>&1 \
 && $S --gemms skinny_rope >> $O/step.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
