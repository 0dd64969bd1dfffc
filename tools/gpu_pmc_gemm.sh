#!/bin/bash
# PMC passes over the GEMM kernels (one counter group per rocprofv3 run, --pmc only).
# PROF_VARIANTS selects our kernel variants (see tools/prof_gemm.py); hipBLASLt always runs.
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $R/gpurun_out/pmc/p1 -o p1 -- python3 $R/tools/prof_gemm.py > $R/gpurun_out/pmc/p1.log 2>&1 \
 && timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU_MFMA_MOPS_BF16 --output-format csv -d $R/gpurun_out/pmc/p2 -o p2 -- python3 $R/tools/prof_gemm.py > $R/gpurun_out/pmc/p2.log 2>&1 \
 && timeout -k 10 -s KILL 120 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --output-format csv -d $R/gpurun_out/pmc/p3 -o p3 -- python3 $R/tools/prof_gemm.py > $R/gpurun_out/pmc/p3.log 2>&1
rc=$?
echo "rc=$rc"
tail -n 3 $R/gpurun_out/pmc/p1.log $R/gpurun_out/pmc/p2.log $R/gpurun_out/pmc/p3.log
find $R/gpurun_out/pmc -name "*.csv" | head
exit $rc
