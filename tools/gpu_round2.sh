#!/bin/bash
# GPU round: new GPU tests (attention/llama), GEMM bench, config-4 co-location bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_attention_llama.py -x -q -m gpu > gpurun_out/gpu_attn.log 2>&1 \
 && timeout -k 10 900 python tools/bench_colocate.py --seconds 20 --out gpurun_out/colocate.json > gpurun_out/colocate.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
