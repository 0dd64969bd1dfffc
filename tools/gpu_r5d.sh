set -o pipefail
mkdir -p gpurun_out/r5d
# each step bounded; a step that fails, faults or times out ends the script (no later GPU step)
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step broker_tests timeout -k 10 700 python -u -m pytest tests/test_hbm_broker.py -v -s --timeout 200 --timeout-method thread > gpurun_out/r5d/hbm_broker_tests.log 2>&1
step bench timeout -k 10 420 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5d/bench_n1.json 2> gpurun_out/r5d/bench_n1.err
