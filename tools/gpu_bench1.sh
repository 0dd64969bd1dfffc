# one 1-GPU bench run into gpurun_out/$1 (bench.json / bench.err / steps.log); extra args after $1
set -o pipefail
D=gpurun_out/$1
shift
mkdir -p $D
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 "$@" > $D/bench.json 2> $D/bench.err
echo "bench rc=$?" >> $D/steps.log
