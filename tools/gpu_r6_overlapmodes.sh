set -o pipefail
O=gpurun_out/r6om; mkdir -p $O
timeout -k 10 500 python -u tools/diag/exit_overlap_modes.py --trials 3 > $O/modes.jsonl 2> $O/modes.err
