set -o pipefail
mkdir -p gpurun_out/r6y
timeout -k 10 1000 python -u bench.py --steps 20 --warmup 3 --json-out gpurun_out/r6y/bench.json > gpurun_out/r6y/bench.log 2>&1
