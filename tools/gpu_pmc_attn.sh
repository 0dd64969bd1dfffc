#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/pmca
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $R/gpurun_out/pmca/p1 -o p1 -- python3 $R/tools/prof_attn.py > $R/gpurun_out/pmca/p1.log 2>&1 \
 && timeout -k 10 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $R/gpurun_out/pmca/p2 -o p2 -- python3 $R/tools/prof_attn.py > $R/gpurun_out/pmca/p2.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
