#!/bin/bash
# BASELINE config 4 on one MI355X: two Llama-3-8B pods under the plugin + quota shim.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u tools/bench_colocate.py --seconds ${SECONDS_PER_PHASE:-20} --out gpurun_out/colocate.json > gpurun_out/colocate.log 2>&1
rc=$?
echo "rc=$rc"
tail -3 gpurun_out/colocate.log
exit $rc
