#!/bin/bash
# Serving pod (Llama-3-8B decode, batch 16, 1024-token prompt, hipGraph per step) next to a heavy
# prefill pod (batch 8 x 2048): time-sliced vs CU slots 16 + 16.
set -o pipefail
mkdir -p gpurun_out/serve
export TMPDIR=/tmp
timeout -k 10 1000 python -u tools/bench_colocate.py --isolation both --mode-a decode --seq-a 1024 --batch 16 \
  --batch-b 8 --seconds 15 --out gpurun_out/serve/coloc_decode.json > gpurun_out/serve/coloc_decode.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
