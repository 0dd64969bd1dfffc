set -o pipefail
O=gpurun_out/r6om7; mkdir -p $O
timeout -k 10 500 python -u tools/diag/exit_overlap_modes.py --trials 3 --tenants initonly,small,full > $O/tenants.jsonl 2> $O/tenants.err
