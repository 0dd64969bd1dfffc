#!/bin/bash
# Field diagnosis of the shim's ledger mapping in the bench's pod processes: a plain short bench,
# then the same under rocprofv3 kernel tracing. GPUSHARE_SHIM_DIAG=1 makes a pod process report
# where its ledger is mapped and abort with its memory map if the page disappears.
set -o pipefail
mkdir -p gpurun_out/diag
export TMPDIR=/tmp GPUSHARE_SHIM_DIAG=1
timeout -k 10 400 python3 bench.py --gpus 1 --steps 4 --warmup 1 --compare-rtts "" --fill-orders "" \
    > gpurun_out/diag/bench_plain.log 2>&1 \
 && (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/diag/prof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 4 --warmup 1 --compare-rtts "" --fill-orders "" > $GRAFT_REPO_ROOT/gpurun_out/diag/bench_prof.log 2>&1)
rc=$?
echo "rc=$rc"
exit $rc
