#!/bin/bash
# config 4 on the broker path with the plugin's answer as shipped (host kernel arguments for pods on broker memory)
set -o pipefail
O=gpurun_out/coloc6final
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/bench_colocate.py --seconds 15 --out $O/prefill_x2.json > $O/prefill_x2.log 2>&1 \
 && timeout -k 10 600 python -u tools/bench_colocate.py --mode-a decode --batch 32 --seq-a 1024 --batch-b 4 --seconds 15 --out $O/decode_vs_prefill.json > $O/decode_vs_prefill.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
