#!/bin/bash
# (diagnosis) Round-6 open item: a hipGraph decode pod next to a prefill pod keeps 9-22 % of its
# solo rate. Each run is the decode-vs-prefill pair of tools/gpu_colocate_r6.sh (shorter): the
# answer's settings, kernel arguments in device memory, pods off the broker arena, and the decode
# pod's steps on a high-priority stream. Each pod reports KFD's evicted_ms for its process (found
# by PASID). RUNS = space-separated list of TAG:extra-args (commas for spaces).
set -o pipefail
O=gpurun_out/kernarg_evict
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python -c '
import glob, json, os, torch
torch.zeros(1, device="cuda"); torch.cuda.synchronize()
from aliyun_gpushare_device_plugin_amd.models import llama_pod as m
print(json.dumps({"pid": os.getpid(), "kfd_proc": m._kfd_proc_dir(), "evicted_ms": m._evicted_ms(),
                  "priority_range": torch.cuda.Stream.priority_range(),
                  "dir_files": {d: {f.rsplit("/", 1)[1]: (open(f).read(80).strip() if os.path.isfile(f) else "dir")
                                    for f in sorted(glob.glob(d + "/*"))[:12]}
                                for d in sorted(glob.glob("/sys/class/kfd/kfd/proc/*"))[:8]}}))
' > $O/probe.json 2> $O/probe.err || exit $?
for run in ${RUNS:-answer:}; do
  tag=${run%%:*}; extra=${run#*:}; extra=${extra//,/ }
  timeout -k 10 420 python -u tools/bench_colocate.py --mode-a decode --batch 32 --seq-a 1024 --batch-b 4 --seconds 12 $extra --out $O/$tag.json > $O/$tag.log 2>&1 || { rc=$?; echo "rc=$rc ($tag)"; exit $rc; }
done
echo "rc=0"
