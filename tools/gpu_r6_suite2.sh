set -o pipefail
mkdir -p gpurun_out/r6s2
# the two tests after every other GPU test (as in the full suite): the GEMM/attention tests first
timeout -k 10 900 python -u -m pytest tests/test_gpu_ops.py tests/test_hbm_broker.py -m gpu -v --timeout 300 --timeout-method thread -k "not sanitizer" > gpurun_out/r6s2/suite.log 2>&1
rc=$?
tail -5 gpurun_out/r6s2/suite.log
exit $rc
