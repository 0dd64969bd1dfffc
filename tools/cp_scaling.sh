#!/bin/bash
# Control-plane-only scaling (no GPU work): bench.py --no-gpu at N = 1, 2, 4, 8 single-process
# (rank 0's control plane is the part that grows with N; the GPU phase per rank is fixed).
set -o pipefail
mkdir -p gpurun_out/cp
for n in 1 2 4 8; do
  timeout -k 10 300 python bench.py --no-gpu --gpus $n --steps 30 --warmup 3 --json-out gpurun_out/cp/cp_n$n.json > gpurun_out/cp/cp_n$n.log 2>&1 || exit $?
done
python - <<'PY'
import json
for n in (1, 2, 4, 8):
    d = json.load(open(f"gpurun_out/cp/cp_n{n}.json"))
    print(n, {k: d[k] for k in ("value", "ms_per_step", "allocate_p50_ms", "allocate_p99_ms", "admission_p50_ms", "pods_per_node", "failed_admissions")})
PY
