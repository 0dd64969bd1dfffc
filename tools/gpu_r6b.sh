set -o pipefail
mkdir -p gpurun_out/r6g
timeout -k 10 900 python -u bench.py --steps 20 --warmup 3 --json-out gpurun_out/r6g/bench.json > gpurun_out/r6g/bench.log 2>&1
