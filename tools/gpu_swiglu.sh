set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_attention_llama.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/swiglu_tests.log 2>&1 \
 && timeout -k 10 300 python -u tools/prof_llama.py > gpurun_out/llama_fwd.log 2>&1
rc=$?; echo rc=$rc; tail -3 gpurun_out/swiglu_tests.log; tail -1 gpurun_out/llama_fwd.log; exit $rc
