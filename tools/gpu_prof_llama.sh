#!/bin/bash
# Per-kernel time of a Llama-3-8B prefill forward (rocprofv3 --kernel-trace --stats).
set -o pipefail
mkdir -p gpurun_out/prof_llama
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/prof_llama.py > gpurun_out/prof_llama/plain.log 2>&1 \
 && (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_llama -o llama -- python3 $R/tools/prof_llama.py --iters 2 > $R/gpurun_out/prof_llama/prof.log 2>&1)
rc=$?
echo "rc=$rc"
cat gpurun_out/prof_llama/plain.log | tail -2
exit $rc
