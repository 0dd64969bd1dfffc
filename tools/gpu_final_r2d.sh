#!/bin/bash
# Last GPU session of round 2: smoke + whole GPU suite, then the 1-GPU headline bench with a
# rocprofv3 kernel-stats run of a shorter bench.
set -o pipefail
mkdir -p gpurun_out/prof_final
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
 && timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 \
 && timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --json-out gpurun_out/bench1.json > gpurun_out/bench1.log 2>&1 \
 && (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_final -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 10 --warmup 2 --compare-rtts "" > $GRAFT_REPO_ROOT/gpurun_out/prof_final/bench_prof.log 2>&1)
rc=$?
echo "rc=$rc"
exit $rc
