#!/bin/bash
# 4-wave GEMM store policy / schedule variants: GEMM + model tests, the interleaved sweep vs
# hipBLASLt, and the kernel-boundary probe.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_attention_llama.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gemm_sched_tests.log 2>&1 \
 && timeout -k 10 400 python -u tools/gemm_sched_sweep.py ${SWEEP_ARGS} --out gpurun_out/gemm_sched_sweep4.json > gpurun_out/gemm_sched_sweep4.log 2>&1 \
 && timeout -k 10 300 python -u tools/gemm_boundary_probe.py > gpurun_out/gemm_boundary4.jsonl 2> gpurun_out/gemm_boundary4.err
rc=$?
echo "rc=$rc"
exit $rc
