# the whole GPU suite into gpurun_out/$1/gpu_tests.log
set -o pipefail
D=gpurun_out/$1
mkdir -p $D
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $D/gpu_tests.log 2>&1
echo "suite rc=$?" >> $D/steps.log
