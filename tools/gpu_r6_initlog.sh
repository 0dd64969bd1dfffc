# comgr's own account of the blit build at a process's first stream, with the node's cache warm
set -o pipefail
D=gpurun_out/r6r
mkdir -p $D
timeout -k 10 120 python -c "
from aliyun_gpushare_device_plugin_amd.quota import comgr_cache as c
import json; w=c.warm('/tmp/r6r_cc', ('system','torch')); c.seal('/tmp/r6r_cc'); print(json.dumps({k: v.get('ok') for k, v in w['runtimes'].items()}))
" > $D/warm.json 2>&1 \
 && XDG_CACHE_HOME=/tmp/r6r_home AMD_COMGR_EMIT_VERBOSE_LOGS=1 AMD_COMGR_REDIRECT_LOGS=stderr AMD_COMGR_TIME_STATISTICS=1 AMD_COMGR_CACHE=1 AMD_COMGR_CACHE_DIR=/tmp/r6r_cc timeout -k 10 120 python tools/diag/first_kernel_split.py > $D/split.json 2> $D/split.err \
 && XDG_CACHE_HOME=/tmp/r6r_home2 AMD_COMGR_EMIT_VERBOSE_LOGS=1 AMD_COMGR_REDIRECT_LOGS=stderr AMD_COMGR_TIME_STATISTICS=1 timeout -k 10 120 python tools/diag/first_kernel_split.py > $D/split_nocache.json 2> $D/split_nocache.err \
 && gzip -f $D/split.err $D/split_nocache.err
