set -o pipefail
O=gpurun_out/r6is; mkdir -p $O
for i in 1 2 3; do timeout -k 10 120 python -u tools/diag/hip_init_split.py >> $O/split.jsonl 2>> $O/split.err || exit $?; done
timeout -k 10 120 python -u tools/diag/hip_init_split.py HSA_ENABLE_SDMA=0 >> $O/split.jsonl 2>> $O/split.err &&
timeout -k 10 120 python -u tools/diag/hip_init_split.py HSA_ENABLE_INTERRUPT=0 >> $O/split.jsonl 2>> $O/split.err &&
timeout -k 10 120 python -u tools/diag/hip_init_split.py HSA_ENABLE_SCRATCH_ASYNC_RECLAIM=0 >> $O/split.jsonl 2>> $O/split.err &&
timeout -k 10 120 python -u tools/diag/hip_init_split.py HSA_ENABLE_IPC_MODE_LEGACY=1 >> $O/split.jsonl 2>> $O/split.err &&
AMD_LOG_LEVEL=4 timeout -k 10 120 python -u tools/diag/hip_init_split.py > $O/log4.json 2> $O/log4.err
