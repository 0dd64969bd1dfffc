set -o pipefail
O=gpurun_out/r6final2; mkdir -p $O
timeout -k 10 1000 python -u bench.py --steps 20 --warmup 3 --json-out $O/bench.json > $O/bench.log 2>&1
