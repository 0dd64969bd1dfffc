#!/bin/bash
# Per-XCD CU masks: does "bit b -> XCC b % 8" select whole XCDs, via both env forms?
set -o pipefail
mkdir -p gpurun_out/cumask2
O=gpurun_out/cumask2
P="tools/bin/cu_mask_probe env"
X0=$(python3 -c "print(','.join(str(b) for b in range(0,256,8)))")
X01=$(python3 -c "print(','.join(str(b) for b in range(256) if b % 8 in (0,1)))")
X4567=$(python3 -c "print(','.join(str(b) for b in range(256) if b % 8 >= 4))")
R0=0x$(python3 -c "print('%064x' % sum(1<<b for b in range(0,256,8)))")
R4567=0x$(python3 -c "print('%064x' % sum(1<<b for b in range(256) if b % 8 >= 4))")
HSA_CU_MASK="0:$X0" timeout -k 5 45 $P > $O/hsa_xcd0.jsonl 2> $O/hsa_xcd0.err \
 && HSA_CU_MASK="0:$X01" timeout -k 5 45 $P > $O/hsa_xcd01.jsonl 2> $O/hsa_xcd01.err \
 && HSA_CU_MASK="0:$X4567" timeout -k 5 45 $P > $O/hsa_xcd4567.jsonl 2> $O/hsa_xcd4567.err \
 && ROC_GLOBAL_CU_MASK=$R0 timeout -k 5 45 $P > $O/roc_xcd0.jsonl 2> $O/roc_xcd0.err \
 && ROC_GLOBAL_CU_MASK=$R4567 timeout -k 5 45 $P > $O/roc_xcd4567.jsonl 2> $O/roc_xcd4567.err \
 && HSA_CU_MASK="0:$X4567" ROC_GLOBAL_CU_MASK=$R4567 timeout -k 5 45 $P > $O/both_xcd4567.jsonl 2> $O/both_xcd4567.err \
 && HSA_CU_MASK="0:$X4567" ROC_GLOBAL_CU_MASK=$R4567 timeout -k 10 120 python tools/cu_mask_gemm.py > $O/gemm_xcd4567.jsonl 2> $O/gemm.err
rc=$?
echo "rc=$rc"
exit $rc
