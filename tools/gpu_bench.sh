#!/bin/bash
# One GPU-box session for the headline bench: 1-GPU bench (pods as processes under the shim),
# then a rocprofv3 kernel profile of a shorter run. Every GPU step has its own time limit.
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
STEPS=${STEPS:-20}
timeout -k 10 600 python bench.py --gpus 1 --steps $STEPS --warmup 3 --json-out gpurun_out/bench1.json > gpurun_out/bench1.log 2>&1 \
 && (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 10 --warmup 2 --compare-rtts "" > $GRAFT_REPO_ROOT/gpurun_out/prof/bench_prof.log 2>&1)
rc=$?
echo "rc=$rc"
exit $rc
