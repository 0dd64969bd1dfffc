set -o pipefail
D=gpurun_out/r5z
mkdir -p $D
run() { local name=$1; shift; timeout -k 10 120 env "$@" LD_PRELOAD=$PWD/tools/diag/build/libdmabuf_ref_probe.so python tools/diag/dmabuf_ref_probe.py 0 > $D/$name.json 2> $D/$name.err; local rc=$?; echo "$name rc=$rc" >> $D/steps.log; [ $rc -eq 0 ] || exit $rc; }
run base X=1
run sdma0 HSA_ENABLE_SDMA=0
run kernarg HIP_FORCE_DEV_KERNARG=0
run base2 X=2
