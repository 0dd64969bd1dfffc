set -o pipefail
mkdir -p gpurun_out/r5c
timeout -k 10 120 ./tools/diag/build/vmm_semantics_probe 1024 > gpurun_out/r5c/vmm_semantics_sys.json 2> gpurun_out/r5c/vmm_semantics_sys.err
echo "sys rc=$?"
timeout -k 10 180 python tools/diag/vmm_semantics_probe.py 1024 > gpurun_out/r5c/vmm_semantics_torch.json 2> gpurun_out/r5c/vmm_semantics_torch.err
echo "torch rc=$?"
timeout -k 10 600 python -u -m pytest tests/test_hbm_broker.py -v -s --timeout 170 --timeout-method thread > gpurun_out/r5c/hbm_broker_tests.log 2>&1
echo "tests rc=$?"
