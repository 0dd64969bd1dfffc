#!/bin/bash
# Attention kernel A/B: the GPU numerics tests, then the sweep in two variant orders.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${1:-7 11 12}"
timeout -k 10 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_attention_llama.py -m gpu > gpurun_out/attn_tests.log 2>&1 \
 && timeout -k 10 300 python tools/attn_sweep.py $V > gpurun_out/attn_sweep_a.jsonl 2>&1 \
 && timeout -k 10 300 python tools/attn_sweep.py $(echo $V | tr ' ' '\n' | tac | tr '\n' ' ') > gpurun_out/attn_sweep_b.jsonl 2>&1
rc=$?
echo "rc=$rc"
exit $rc
