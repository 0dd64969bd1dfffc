set -o pipefail
mkdir -p gpurun_out/r5f
# each step bounded; a crash, abort or time limit ends the script (no later GPU step);
# "soft" steps go on after ordinary test failures (exit 1)
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
soft() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
soft spill timeout -k 10 90 ./tools/diag/build/vmm_spill_probe > gpurun_out/r5f/vmm_spill.json 2> gpurun_out/r5f/vmm_spill.err
soft broker_tests timeout -k 10 600 python -u -m pytest tests/test_hbm_broker.py -v -s --timeout 200 --timeout-method thread > gpurun_out/r5f/hbm_broker_tests.log 2>&1
step bench timeout -k 10 420 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5f/bench_n1.json 2> gpurun_out/r5f/bench_n1.err
