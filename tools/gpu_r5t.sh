set -o pipefail
D=gpurun_out/r5t
mkdir -p $D
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc" >> $D/steps.log; [ $rc -eq 0 ] || exit $rc; }
for w in 0 1 3; do
  step torch_w$w timeout -k 10 120 env LD_PRELOAD=$PWD/tools/diag/build/libdmabuf_ref_probe.so python tools/diag/dmabuf_ref_probe.py $w > $D/torch_w$w.json 2> $D/torch_w$w.err
done
