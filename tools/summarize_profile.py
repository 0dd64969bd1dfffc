#!/usr/bin/env python3
"""Condense rocprofv3 --stats CSV output into a short markdown table for profiles/.

python tools/summarize_profile.py gpurun_out/prof/bench_kernel_stats.csv [--title T] > profiles/x.md
"""
import argparse
import csv
import re


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)          # drop argument lists
    name = re.sub(r"<.*", "", name)           # drop template args
    return name.replace("void ", "")[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--title", default="rocprofv3 kernel stats")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    print(f"## {a.title}\n")
    print("| kernel | calls | total ms | avg us | min us | max us | % |")
    print("|---|---:|---:|---:|---:|---:|---:|")
    for r in rows[:15]:
        print(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['TotalDurationNs'])/1e6:.2f} | "
              f"{float(r['AverageNs'])/1e3:.1f} | {float(r['MinNs'])/1e3:.1f} | {float(r['MaxNs'])/1e3:.1f} | "
              f"{float(r['Percentage']):.2f} |")


if __name__ == "__main__":
    main()
