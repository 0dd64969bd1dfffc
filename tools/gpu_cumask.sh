#!/bin/bash
# Probe process-wide CU masks on an MI355X (HSA_CU_MASK read by ROCr at queue creation,
# ROC_GLOBAL_CU_MASK read by HIP): which XCD/SE/CUs the default stream's workgroups land on, FMA
# throughput, and the GEMM rate on a subset of CUs. Each GPU step has its own limit.
set -o pipefail
mkdir -p gpurun_out/cumask
O=gpurun_out/cumask
P="tools/bin/cu_mask_probe env"
timeout -k 5 45 $P > $O/env_none.jsonl 2> $O/env_none.err \
 && HSA_CU_MASK="0:0-127" timeout -k 5 45 $P > $O/env_hsa_0-127.jsonl 2> $O/env_hsa_0-127.err \
 && HSA_CU_MASK="0:0-31" timeout -k 5 45 $P > $O/env_hsa_0-31.jsonl 2> $O/env_hsa_0-31.err \
 && HSA_CU_MASK="0:0-7" timeout -k 5 45 $P > $O/env_hsa_0-7.jsonl 2> $O/env_hsa_0-7.err \
 && ROC_GLOBAL_CU_MASK=0xffffffffffffffffffffffffffffffff timeout -k 5 45 $P > $O/env_roc_lo128.jsonl 2> $O/env_roc_lo128.err \
 && timeout -k 10 120 python tools/cu_mask_gemm.py > $O/gemm.jsonl 2> $O/gemm.err \
 && HSA_CU_MASK="0:0-127" timeout -k 10 120 python tools/cu_mask_gemm.py >> $O/gemm.jsonl 2>> $O/gemm.err
rc=$?
echo "rc=$rc"
exit $rc
