set -o pipefail
# where a pod's first stream spends its time once comgr's cache holds the runtime's blit kernels
O=gpurun_out/r6fs; mkdir -p $O
export AMD_COMGR_CACHE=1 AMD_COMGR_CACHE_DIR=$PWD/$O/cache XDG_CACHE_HOME=$PWD/$O/xdg
timeout -k 10 120 python -u tools/diag/first_kernel_split.py > $O/fill.json 2> $O/fill.err &&
timeout -k 10 120 python -u tools/diag/first_kernel_split.py > $O/cached.json 2> $O/cached.err &&
AMD_LOG_LEVEL=4 timeout -k 10 120 python -u tools/diag/first_kernel_split.py > $O/cached_log.json 2> $O/cached_log.err &&
AMD_COMGR_EMIT_VERBOSE_LOGS=1 AMD_COMGR_REDIRECT_LOGS=stderr AMD_COMGR_TIME_STATISTICS=1 \
  timeout -k 10 120 python -u tools/diag/first_kernel_split.py > $O/cached_comgr.json 2> $O/cached_comgr.err
