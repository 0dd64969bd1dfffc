#!/bin/bash
# GPU validation: smoke, then the whole GPU test suite (one process, per-test timeouts).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
 && timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
