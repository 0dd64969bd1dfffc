#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --pmc only): 4-wave GEMM with streamed
# device-scope C stores (schedule 0) vs write-back stores (schedule 9) vs hipBLASLt.
set -o pipefail
mkdir -p gpurun_out/pmc_st
export TMPDIR=/tmp
export PROF_VARIANTS= PROF_SCHEDS=0,9
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $R/gpurun_out/pmc_st/p1 -o p1 -- python3 $R/tools/prof_gemm.py 4096x4096x4096,8192x8192x8192 > $R/gpurun_out/pmc_st/p1.log 2>&1 \
 && timeout -k 10 -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d $R/gpurun_out/pmc_st/p2 -o p2 -- python3 $R/tools/prof_gemm.py 4096x4096x4096,8192x8192x8192 > $R/gpurun_out/pmc_st/p2.log 2>&1 \
 && timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pmc_st/kt -o kt -- python3 $R/tools/prof_gemm.py 4096x4096x4096,8192x8192x8192 > $R/gpurun_out/pmc_st/kt.log 2>&1
rc=$?
echo "rc=$rc"
find $R/gpurun_out/pmc_st -name "*.csv" | head -20
exit $rc
