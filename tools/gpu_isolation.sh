#!/bin/bash
# Compute isolation on MI355X: GPU tests for CU-slot masks, then config 4 (2 x Llama-3-8B) under
# time-slicing vs CU slots, equal pods and a latency-sensitive pod A next to a heavy pod B.
set -o pipefail
mkdir -p gpurun_out/iso
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_cu_isolation.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/iso/tests.log 2>&1 \
 && timeout -k 10 900 python -u tools/bench_colocate.py --isolation both --seconds 15 --out gpurun_out/iso/coloc_equal.json > gpurun_out/iso/coloc_equal.log 2>&1 \
 && timeout -k 10 900 python -u tools/bench_colocate.py --isolation both --seconds 15 --batch 1 --batch-b 8 --out gpurun_out/iso/coloc_victim.json > gpurun_out/iso/coloc_victim.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
