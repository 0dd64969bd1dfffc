set -o pipefail
D=gpurun_out/r5m
mkdir -p $D
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc" >> $D/steps.log; [ $rc -eq 0 ] || exit $rc; }
step sys timeout -k 10 90 ./tools/diag/build/dmabuf_ref_probe 1 > $D/sys.json 2> $D/sys.err
step torch timeout -k 10 120 env LD_PRELOAD=$PWD/tools/diag/build/libdmabuf_ref_probe.so python tools/diag/dmabuf_ref_probe.py 1 > $D/torch.json 2> $D/torch.err
