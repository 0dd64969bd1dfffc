#!/bin/bash
# hipGraph replay vs eager launches in a CU-masked victim, alone and next to a GEMM aggressor.
set -o pipefail
O=gpurun_out/graphmask
mkdir -p $O
P=tools/graph_mask_probe.py
run_pair() {   # $1 = label, $2 = victim mask, $3 = aggressor mask ("" = none)
  if [ -n "$3" ]; then HSA_CU_MASK="$3" timeout -k 5 60 python $P aggressor > $O/$1.aggr.log 2>&1 & else timeout -k 5 60 python $P aggressor > $O/$1.aggr.log 2>&1 & fi
  AP=$!
  sleep 8
  if [ -n "$2" ]; then HSA_CU_MASK="$2" PROBE_DELAY=0 timeout -k 5 60 python $P victim > $O/$1.victim.json 2> $O/$1.victim.err; else timeout -k 5 60 python $P victim > $O/$1.victim.json 2> $O/$1.victim.err; fi
  RC=$?
  wait $AP
  return $RC
}
HSA_CU_MASK="0:0-127" timeout -k 5 60 python $P victim > $O/solo_masked.victim.json 2> $O/solo_masked.err \
 && timeout -k 5 60 python $P victim > $O/solo_full.victim.json 2> $O/solo_full.err \
 && run_pair timesliced "" "" \
 && run_pair both_masked "0:0-127" "0:128-255" \
 && run_pair victim_masked_only "0:0-127" "" \
 && run_pair aggressor_masked_only "" "0:128-255"
rc=$?
echo "rc=$rc"
exit $rc
