#!/bin/bash
# Config 4, decode server next to a prefill neighbour, time-sliced vs CU slots (the server launches
# eagerly under CU slots: graph replay stalls there, profiles/cu_mask/README.md).
set -o pipefail
O=gpurun_out/coloc
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/bench_colocate.py --mode-a decode --decode-eager --batch 32 --seq-a 1024 --batch-b 4 --seconds 15 --isolation both --out $O/decode_vs_prefill_cu.json > $O/decode_vs_prefill_cu.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
