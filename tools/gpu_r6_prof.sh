set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6prof; mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o bench -- python3 -u bench.py --steps 8 --warmup 1 \
  --comparator-steps 0 --driver-path-steps 0 --compare-rtts "" --fill-orders "" --json-out $O/bench.json > $O/bench.log 2>&1
