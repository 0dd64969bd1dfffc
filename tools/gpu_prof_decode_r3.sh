#!/bin/bash
# rocprofv3 kernel stats of the graph-replayed batch-32 Llama-3-8B decode step (final round-3 kernels).
set -o pipefail
mkdir -p gpurun_out/dprof2
export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/dprof2 -o dec -- python3 $GRAFT_REPO_ROOT/tools/bench_decode.py --no-attn-micro --no-gemm-micro --gemms skinny_rope --steps 32 > $GRAFT_REPO_ROOT/gpurun_out/dprof2/prof.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
