set -o pipefail
D=gpurun_out/$1
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_hbm_broker.py -v -s --timeout 200 --timeout-method thread > $D/hbm_broker_tests.log 2>&1
rc=$?; echo "broker_tests rc=$rc" >> $D/steps.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 420 python bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench.json 2> $D/bench.err
echo "bench rc=$?" >> $D/steps.log
