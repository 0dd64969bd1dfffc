set -o pipefail
mkdir -p gpurun_out/r5c
# each step bounded; a step that faults, aborts or times out ends the script (no later GPU step)
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step sys timeout -k 10 120 ./tools/diag/build/vmm_semantics_probe 1024 > gpurun_out/r5c/vmm_semantics_sys.json 2> gpurun_out/r5c/vmm_semantics_sys.err
step torch timeout -k 10 180 python tools/diag/vmm_semantics_probe.py 1024 > gpurun_out/r5c/vmm_semantics_torch.json 2> gpurun_out/r5c/vmm_semantics_torch.err
step tests timeout -k 10 600 python -u -m pytest tests/test_hbm_broker.py -v -s --timeout 170 --timeout-method thread > gpurun_out/r5c/hbm_broker_tests.log 2>&1
