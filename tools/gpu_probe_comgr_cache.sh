# the runtime compiles its blit kernels with comgr at the first stream of every process: does
# comgr's compilation cache take that off the second and later processes?
set -o pipefail
D=gpurun_out/comgr_cache
mkdir -p $D
run() { local name=$1; shift; timeout -k 10 120 env "$@" python tools/diag/first_kernel_split.py > $D/$name.json 2> $D/$name.err; local rc=$?; echo "$name rc=$rc" >> $D/steps.log; [ $rc -eq 0 ] || exit $rc; }
run base X=1
run verbose AMD_COMGR_EMIT_VERBOSE_LOGS=1 AMD_COMGR_REDIRECT_LOGS=stderr AMD_COMGR_TIME_STATISTICS=1
run cache1 AMD_COMGR_CACHE=1 AMD_COMGR_CACHE_DIR=$PWD/$D/cc
run cache2 AMD_COMGR_CACHE=1 AMD_COMGR_CACHE_DIR=$PWD/$D/cc
run cache3 AMD_COMGR_CACHE=1 AMD_COMGR_CACHE_DIR=$PWD/$D/cc
run cache_verbose AMD_COMGR_CACHE=1 AMD_COMGR_CACHE_DIR=$PWD/$D/cc AMD_COMGR_EMIT_VERBOSE_LOGS=1 AMD_COMGR_REDIRECT_LOGS=stderr AMD_COMGR_TIME_STATISTICS=1
find $D/cc -type d -exec chmod a-w {} +
run cache_ro1 AMD_COMGR_CACHE=1 AMD_COMGR_CACHE_DIR=$PWD/$D/cc
run cache_ro2 AMD_COMGR_CACHE=1 AMD_COMGR_CACHE_DIR=$PWD/$D/cc
find $D/cc -type d -exec chmod u+w {} +
ls -laR $D/cc > $D/cc_listing.txt 2>&1 || true
du -sh $D/cc >> $D/cc_listing.txt 2>&1 || true
rm -rf $D/cc
