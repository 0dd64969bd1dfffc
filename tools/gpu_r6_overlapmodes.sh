set -o pipefail
O=gpurun_out/r6om8; mkdir -p $O
timeout -k 10 600 python -u tools/diag/exit_overlap_modes.py --trials 3 --modes shim,shimfast,shimfastall --whens reaped > $O/shimfast.jsonl 2> $O/shimfast.err
