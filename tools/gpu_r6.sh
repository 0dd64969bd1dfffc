#!/bin/bash
# Round 6 on one MI355X: the broker / shim GPU tests, then the headline bench with its comparators.
# Every GPU step has its own time limit; a failure ends the script (set -e semantics by hand).
mkdir -p gpurun_out/r6
timeout -k 10 900 python -u -m pytest tests/test_hbm_broker.py -v --timeout 300 --timeout-method thread -s -p no:cacheprovider \
  > gpurun_out/r6/hbm_broker_tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> gpurun_out/r6/steps.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi   # 1 = a test failed (read it); anything else: stop here
timeout -k 10 900 python -u bench.py --steps 20 --warmup 3 --json-out gpurun_out/r6/bench.json > gpurun_out/r6/bench.log 2>&1
rc=$?
echo "bench rc=$rc" >> gpurun_out/r6/steps.log
exit $rc
