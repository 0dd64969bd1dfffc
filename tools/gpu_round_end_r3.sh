#!/bin/bash
# Round-3 session end: smoke, GPU suite, 1-GPU bench, then BASELINE config 4 co-location on the round-3
# kernels (two prefill pods; a batch-32 decode server next to a prefill neighbour).
set -o pipefail
bash tools/gpu_final_r3.sh final3 && bash tools/gpu_colocate_r3.sh
rc=$?
echo "rc=$rc"
exit $rc
