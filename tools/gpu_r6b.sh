set -o pipefail
mkdir -p gpurun_out/r6p
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 1000 python -u bench.py --steps 20 --warmup 3 --json-out gpurun_out/r6p/bench.json > gpurun_out/r6p/bench.log 2>&1 \
 && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r6p/prof -o bench -- python -u bench.py --steps 6 --warmup 1 --comparator-steps 0 --driver-path-steps 0 --json-out gpurun_out/r6p/bench_prof.json > gpurun_out/r6p/bench_prof.log 2>&1
