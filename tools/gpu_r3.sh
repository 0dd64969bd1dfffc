#!/bin/bash
# Round-3 GPU session: the new hardware tests (watchdog, render-node GEM, HBM gauge), then a
# rocprofv3 kernel profile of a short bench run. Every GPU step has its own time limit.
set -o pipefail
mkdir -p gpurun_out/prof_r3
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_native.py -m gpu \
    -k "watchdog or gem or hbm_used or single_rank" > gpurun_out/gpu_watchdog.log 2>&1 \
 && (cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_r3 -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 10 --warmup 2 --compare-rtts "" --fill-orders "" > $GRAFT_REPO_ROOT/gpurun_out/prof_r3/bench_prof.log 2>&1)
rc=$?
echo "rc=$rc"
exit $rc
