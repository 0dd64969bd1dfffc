set -o pipefail
O=gpurun_out/r6ip; mkdir -p $O
for i in 1 2; do timeout -k 10 120 python -u tools/diag/hip_init_split.py >> $O/split2.jsonl 2>> $O/split.err || exit $?; done
timeout -k 10 120 python -u tools/diag/hip_init_split.py ROCR_VISIBLE_DEVICES=0 >> $O/split2.jsonl 2>> $O/split.err
