#!/bin/bash
# One GPU-box session: GPU tests, 1-GPU bench, rocprofv3 kernel profile of the bench.
# Every GPU step has its own time limit; steps are chained so a failure stops the run.
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
STEPS=${STEPS:-20}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
  timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 \
 && timeout -k 10 300 python bench.py --gpus 1 --steps $STEPS --warmup 3 --json-out gpurun_out/bench1.json > gpurun_out/bench1.log 2>&1 \
 && (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 10 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof/bench_prof.log 2>&1)
rc=$?
echo "rc=$rc"
exit $rc
