#!/bin/bash
# Kernel profile of graph-replayed Llama-3-8B decode steps.
set -o pipefail
mkdir -p gpurun_out/decprof
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/decprof -o dec -- python3 $GRAFT_REPO_ROOT/tools/prof_decode.py --steps 20 > $GRAFT_REPO_ROOT/gpurun_out/decprof/log.txt 2>&1
rc=$?
echo "rc=$rc"
exit $rc
