"""Command-line entry points: plugin daemon, kubectl-inspect-gpushare, podgetter, smi."""
