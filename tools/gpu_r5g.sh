set -o pipefail
mkdir -p gpurun_out/r5g
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step dmabuf timeout -k 10 90 ./tools/diag/build/dmabuf_ref_probe > gpurun_out/r5g/dmabuf_ref.json 2> gpurun_out/r5g/dmabuf_ref.err
step bench timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5g/bench_n1.json 2> gpurun_out/r5g/bench_n1.err
GPUSHARE_HBM_MAP_THREADS=4 step bench_mt4 timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --driver-path-steps 0 > gpurun_out/r5g/bench_n1_mt4.json 2> gpurun_out/r5g/bench_n1_mt4.err
