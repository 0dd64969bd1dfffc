set -o pipefail
O=gpurun_out/r6ex; mkdir -p $O
timeout -k 10 200 python -u tools/diag/exit_path_probe.py $O/logs --shim > $O/exit_shim.jsonl 2> $O/exit_shim.err &&
timeout -k 10 400 python -u bench.py --steps 12 --warmup 1 --tenant-stop exit --comparator-steps 0 \
    --driver-path-steps 0 --compare-rtts "" --fill-orders "" --no-ref-churn --json-out $O/exit_bench.json > $O/exit_bench.log 2>&1
