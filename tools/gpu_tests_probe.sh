#!/bin/bash
# GPU validation (smoke + whole GPU suite), then the GEMM kernel-boundary probe and the 4-wave
# GEMM phase-B schedule sweep.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
 && timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 \
 && timeout -k 10 300 python -u tools/gemm_boundary_probe.py > gpurun_out/gemm_boundary.jsonl 2> gpurun_out/gemm_boundary.err \
 && timeout -k 10 400 python -u tools/gemm_sched_sweep.py --out gpurun_out/gemm_sched_sweep.json > gpurun_out/gemm_sched_sweep.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
