#!/bin/bash
# Serving path on MI355X: decode tests, decode bench (attention micro + Llama-3-8B eager vs hipGraph),
# kernel profile of the graph-replayed decode. Each GPU step has its own limit.
set -o pipefail
mkdir -p gpurun_out/dec/prof
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/dec/tests.log 2>&1 \
 && timeout -k 10 400 python -u tools/bench_decode.py --out gpurun_out/dec/bench.jsonl > gpurun_out/dec/bench.log 2>&1 \
 && (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/dec/prof -o dec -- python3 $GRAFT_REPO_ROOT/tools/bench_decode.py --steps 16 > $GRAFT_REPO_ROOT/gpurun_out/dec/prof/prof.log 2>&1)
rc=$?
echo "rc=$rc"
exit $rc
