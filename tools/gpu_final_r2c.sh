#!/bin/bash
# Final-build GPU session: GEMM tests + store/schedule sweep vs hipBLASLt, smoke + whole GPU suite,
# 1-GPU headline bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/gemm_sched_sweep.py --scheds 0,9 --out gpurun_out/gemm_final_sweep.json > gpurun_out/gemm_final_sweep.log 2>&1 \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
 && timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 \
 && timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --json-out gpurun_out/bench1.json > gpurun_out/bench1.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
