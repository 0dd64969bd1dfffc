set -o pipefail
# the unmodified-tenant comparator on its own, twice, with the slowest pod's phases in each line
mkdir -p gpurun_out/r6z
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --steps 12 --warmup 1 --tenant-stop sigterm --comparator-steps 0 \
    --driver-path-steps 0 --compare-rtts "" --fill-orders "" --no-ref-churn \
    --json-out gpurun_out/r6z/sig$i.json > gpurun_out/r6z/sig$i.log 2>&1 || exit $?
done
