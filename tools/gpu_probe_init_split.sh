# split a fresh process's GPU start-up: runtime init, the rest of torch.cuda.init, first memory op
set -o pipefail
D=gpurun_out/init_split
mkdir -p $D
for op in malloc memset ctx malloc; do
  timeout -k 10 120 python tools/diag/cuda_init_split.py $op >> $D/split.jsonl 2>> $D/split.err || exit $?
done
