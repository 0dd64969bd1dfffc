#!/bin/bash
# BASELINE config 4 on the shipped default: two Llama-3-8B pods admitted by the
# plugin with --hbm-broker-dir, their HBM from the GPU's broker (started as the DS starts it), under
# the quota shim: (a) both prefill, (b) pod A a batch-32 decode server (KV cache, hipGraph per step)
# next to a prefill neighbour. Same shapes as tools/gpu_colocate_r3.sh.
set -o pipefail
O=gpurun_out/coloc6
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/bench_colocate.py --seconds 15 --out $O/prefill_x2.json > $O/prefill_x2.log 2>&1 \
 && timeout -k 10 600 python -u tools/bench_colocate.py --mode-a decode --batch 32 --seq-a 1024 --batch-b 4 --seconds 15 --out $O/decode_vs_prefill.json > $O/decode_vs_prefill.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
