#!/bin/bash
# PMC passes (one counter set per run, kernel trace only) for the attention variants 11 and 14.
set -o pipefail
mkdir -p gpurun_out/pmc_w64
cd /tmp
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in 11 14; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace --output-format csv -d $R/gpurun_out/pmc_w64/a_$v -o p -- python3 $R/tools/diag/attn_pmc_probe.py $v > $R/gpurun_out/pmc_w64/a_$v.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_w64/b_$v -o p -- python3 $R/tools/diag/attn_pmc_probe.py $v > $R/gpurun_out/pmc_w64/b_$v.log 2>&1 || exit 1
done
echo done
