# what the first GPU work of a process pays for; variants of runtime settings; one log-level run
set -o pipefail
D=gpurun_out/first_kernel
mkdir -p $D
run() { local name=$1; shift; timeout -k 10 120 env "$@" python tools/diag/first_kernel_split.py > $D/$name.json 2> $D/$name.err; local rc=$?; echo "$name rc=$rc" >> $D/steps.log; [ $rc -eq 0 ] || exit $rc; }
run base X=1
run base2 X=2
run log AMD_LOG_LEVEL=4
run deferred0 HIP_ENABLE_DEFERRED_LOADING=0
run hwq1 GPU_MAX_HW_QUEUES=1
run intr0 HSA_ENABLE_INTERRUPT=0
run base3 X=3
