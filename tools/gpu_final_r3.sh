#!/bin/bash
# Round-3 validation of the final tree: smoke, the whole GPU suite (one process, per-test limits),
# then the 1-GPU headline bench with the driver's step counts.
set -o pipefail
O=gpurun_out/${1:-final}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
 && timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 \
 && timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --json-out $O/bench1.json > $O/bench1.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
