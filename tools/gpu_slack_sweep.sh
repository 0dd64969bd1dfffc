set -o pipefail
mkdir -p gpurun_out/slack
for sl in 2 8 16; do
  GS_BENCH_POD_TRACE=gpurun_out/slack/trace_$sl.jsonl timeout -k 10 200 python bench.py --gpus 1 --steps 12 --warmup 3 --compare-rtts "" --room-slack-gib $sl --json-out gpurun_out/slack/b_$sl.json > gpurun_out/slack/b_$sl.log 2>&1 || exit $?
done
