set -o pipefail
mkdir -p gpurun_out/r6s6
timeout -k 10 1150 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r6s6/gpu_suite.log 2>&1 \
 && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6s6/smoke.log 2>&1
rc=$?
tail -3 gpurun_out/r6s6/gpu_suite.log
exit $rc
