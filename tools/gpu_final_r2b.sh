#!/bin/bash
# Final-build GPU session: smoke + whole GPU suite, 1-GPU headline bench with a rocprofv3 kernel
# profile, then BASELINE config 4 (two Llama-3-8B pods) with the round-2 GEMM store policy.
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
 && timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 \
 && timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --json-out gpurun_out/bench1.json > gpurun_out/bench1.log 2>&1 \
 && timeout -k 10 600 python -u tools/bench_colocate.py --seconds 20 --out gpurun_out/colocate.json > gpurun_out/colocate.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
