set -o pipefail
# the comgr action cache on hardware: its GPU test, then the bench line
O=gpurun_out/r6d2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_comgr_cache.py -m gpu -x -v -s --timeout 240 --timeout-method thread > $O/test.log 2>&1 &&
timeout -k 10 1000 python -u bench.py --steps 20 --warmup 3 --json-out $O/bench.json > $O/bench.log 2>&1
