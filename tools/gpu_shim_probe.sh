#!/bin/bash
# Quota-shim granule evidence on MI355X: plain run, then the same run under rocprofv3's
# memory-allocation + HIP API traces (no --pmc in this run).
set -o pipefail
mkdir -p gpurun_out/shimprobe
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 120 python3 tools/shim_granule_probe.py > gpurun_out/shimprobe/probe.json 2> gpurun_out/shimprobe/probe.err \
 && (cd /tmp && timeout -k 10 180 rocprofv3 --memory-allocation-trace --hip-trace --output-format csv -d $R/gpurun_out/shimprobe/trace -o shim -- python3 $R/tools/shim_granule_probe.py > $R/gpurun_out/shimprobe/probe_traced.json 2> $R/gpurun_out/shimprobe/trace.log)
rc=$?
echo "rc=$rc"
cat gpurun_out/shimprobe/probe.json | head -80
find gpurun_out/shimprobe -name "*.csv" | head
exit $rc
