# kernel trace of a short broker bench (every pod process and the brokers are traced): per-kernel
# time, the pods' GEMMs against the brokers' scrubs. Fresh pod interpreters (--no-pod-zygote): the
# profiler's library is preloaded into every process, and a pod should start under it, not be
# forked from a parent that loaded it.
set -o pipefail
D=gpurun_out/r5prof
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
GS_POD_CLEAN_EXIT=1 timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $D/prof -o run_%pid% -- python3 bench.py --gpus 1 --steps 10 --warmup 3 --driver-path-steps 0 --compare-rtts "" --fill-orders "" --no-pod-zygote > $D/bench.json 2> $D/bench.err
echo "prof rc=$?" >> $D/steps.log
