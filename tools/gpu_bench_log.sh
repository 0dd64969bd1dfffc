# a 1-GPU bench with the shim's log at level 1 (the pods' stderr lands in bench.err)
set -o pipefail
D=gpurun_out/$1
mkdir -p $D
GPUSHARE_SHIM_LOG=1 timeout -k 10 400 python bench.py --gpus 1 --steps 10 --warmup 3 --driver-path-steps 0 > $D/bench.json 2> $D/bench.err
echo "bench rc=$?" >> $D/steps.log
