set -o pipefail
D=gpurun_out/r5i
mkdir -p $D
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc" >> $D/steps.log; [ $rc -eq 0 ] || exit $rc; }
soft() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc" >> $D/steps.log; [ $rc -le 1 ] || exit $rc; }
step dmabuf timeout -k 10 90 ./tools/diag/build/dmabuf_ref_probe > $D/dmabuf_ref.json 2> $D/dmabuf_ref.err
soft broker_tests timeout -k 10 300 python -u -m pytest tests/test_hbm_broker.py -v -s --timeout 200 --timeout-method thread -k "released_arena or exporter_death" > $D/hbm_broker_tests.log 2>&1
