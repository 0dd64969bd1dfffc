set -o pipefail
mkdir -p gpurun_out/r6j
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -s tests/test_comgr_cache.py > gpurun_out/r6j/comgr_tests.log 2>&1 \
 && timeout -k 10 1000 python -u bench.py --steps 20 --warmup 3 --json-out gpurun_out/r6j/bench.json > gpurun_out/r6j/bench.log 2>&1
