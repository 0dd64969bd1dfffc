# two 1-GPU bench runs on one box: the defaults, then with extra args (an A/B on the same box)
#   bash tools/gpu_bench_ab.sh <gpurun_out subdir> <extra args...>
set -o pipefail
D=gpurun_out/$1
shift
mkdir -p $D
timeout -k 10 420 python bench.py --gpus 1 --steps 20 --warmup 5 --driver-path-steps 0 > $D/a.json 2> $D/a.err
rc=$?; echo "a rc=$rc" >> $D/steps.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python bench.py --gpus 1 --steps 20 --warmup 5 --driver-path-steps 0 "$@" > $D/b.json 2> $D/b.err
echo "b rc=$?" >> $D/steps.log
