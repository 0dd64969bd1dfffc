#!/bin/bash
# config 4(b) under the broker, pod A decoding eagerly (no hipGraph)
set -o pipefail
O=gpurun_out/coloc6g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/bench_colocate.py --mode-a decode --batch 32 --seq-a 1024 --batch-b 4 --seconds 8 --decode-eager --out $O/broker_eager.json > $O/eager.log 2>&1 \
 && timeout -k 10 600 python -u tools/bench_colocate.py --mode-a decode --batch 32 --seq-a 1024 --batch-b 4 --seconds 8 --decode-eager --no-hbm-broker --out $O/nobroker_eager.json > $O/nobroker_eager.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
