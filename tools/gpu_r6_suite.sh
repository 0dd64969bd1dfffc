set -o pipefail
mkdir -p gpurun_out/r6s
timeout -k 10 1150 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r6s/gpu_suite.log 2>&1
rc=$?
tail -5 gpurun_out/r6s/gpu_suite.log
exit $rc
