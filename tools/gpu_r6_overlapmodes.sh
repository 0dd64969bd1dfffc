set -o pipefail
O=gpurun_out/r6om3; mkdir -p $O
nproc > $O/nproc.txt; python3 -c "import os; print(sorted(os.sched_getaffinity(0)))" > $O/affinity.txt
timeout -k 10 500 python -u tools/diag/exit_overlap_modes.py --trials 3 --pin "/;2/2;2/6;2/6,7,8,9" > $O/pin.jsonl 2> $O/pin.err
