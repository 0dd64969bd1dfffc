set -o pipefail
mkdir -p gpurun_out/r6c
timeout -k 10 90 tools/diag/release_probe 16 pergran > gpurun_out/r6c/release_probe.jsonl 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s tests/test_hbm_broker.py > gpurun_out/r6c/hbm_broker_tests.log 2>&1
