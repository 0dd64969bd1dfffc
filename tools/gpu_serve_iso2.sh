#!/bin/bash
# Same as gpu_serve_iso.sh with the decode pod launching kernel by kernel (no hipGraph), to see
# whether graph replay is what CU slots interact badly with.
set -o pipefail
mkdir -p gpurun_out/serve
export TMPDIR=/tmp
timeout -k 10 1000 python -u tools/bench_colocate.py --isolation both --mode-a decode --seq-a 1024 --batch 16 \
  --batch-b 8 --seconds 15 --decode-eager --out gpurun_out/serve/coloc_decode_eager.json > gpurun_out/serve/coloc_decode_eager.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
