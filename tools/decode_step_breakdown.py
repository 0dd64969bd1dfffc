#!/usr/bin/env python3
"""Per-step kernel breakdown of graph-replayed decode steps from a rocprofv3 kernel trace
(tools/gpu_prof_decode.sh): takes the last N steps (a step starts at each embedding gather),
prints per-kernel time per step, busy time per step and the step's wall span.

python tools/decode_step_breakdown.py gpurun_out/decprof/dec_kernel_trace.csv [--steps 10]"""
import argparse
import collections
import csv
import re


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    return name.replace("void ", "")[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--marker", default="gather", help="substring of the kernel that starts a step")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    starts = starts[-(a.steps + 1):]
    per = collections.defaultdict(float)
    calls = collections.Counter()
    busy = span = 0.0
    for s0, s1 in zip(starts, starts[1:]):
        step = rows[s0:s1]
        span += (int(rows[s1]["Start_Timestamp"]) - int(rows[s0]["Start_Timestamp"])) / 1e3
        for r in step:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            per[short(r["Kernel_Name"])] += d
            calls[short(r["Kernel_Name"])] += 1
            busy += d
    n = len(starts) - 1
    print(f"## decode step: {n} steps, busy {busy / n:.0f} us/step, wall span {span / n:.0f} us/step\n")
    print("| kernel | calls/step | us/step | avg us |")
    print("|---|---:|---:|---:|")
    for k, v in sorted(per.items(), key=lambda kv: -kv[1]):
        print(f"| `{k}` | {calls[k] / n:.0f} | {v / n:.0f} | {v / calls[k]:.2f} |")


if __name__ == "__main__":
    main()
