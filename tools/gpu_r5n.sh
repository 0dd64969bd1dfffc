set -o pipefail
D=gpurun_out/r5n
mkdir -p $D
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc" >> $D/steps.log; [ $rc -eq 0 ] || exit $rc; }
soft() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc" >> $D/steps.log; [ $rc -le 1 ] || exit $rc; }
soft broker_tests timeout -k 10 600 python -u -m pytest tests/test_hbm_broker.py -v -s --timeout 200 --timeout-method thread > $D/hbm_broker_tests.log 2>&1
step bench timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_n1.json 2> $D/bench_n1.err
