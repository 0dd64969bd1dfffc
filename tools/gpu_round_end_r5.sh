# what the driver runs at round end, on the current tree: the GPU suite, then smoke()
set -o pipefail
D=gpurun_out/${1:-round_end}
mkdir -p $D
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $D/gpu_tests.log 2>&1
rc=$?; echo "suite rc=$rc" >> $D/steps.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1
echo "smoke rc=$?" >> $D/steps.log
