set -o pipefail
D=gpurun_out/r5j
mkdir -p $D
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc" >> $D/steps.log; [ $rc -eq 0 ] || exit $rc; }
step sys_cold timeout -k 10 90 ./tools/diag/build/dmabuf_ref_probe 0 > $D/sys_cold.json 2> $D/sys_cold.err
step sys_warm timeout -k 10 90 ./tools/diag/build/dmabuf_ref_probe 1 > $D/sys_warm.json 2> $D/sys_warm.err
step torch_cold timeout -k 10 120 python tools/diag/dmabuf_ref_probe.py 0 > $D/torch_cold.json 2> $D/torch_cold.err
step torch_warm timeout -k 10 120 python tools/diag/dmabuf_ref_probe.py 1 > $D/torch_warm.json 2> $D/torch_warm.err
