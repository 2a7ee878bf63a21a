#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats run (rocpd SQLite .db or the
CSV *_kernel_stats.csv) into a markdown table: per kernel, launches and
average / min / max / total duration.

    python tools/prof_summary.py gpurun_out/r1/prof/run_results.db > profiles/r01_kernels.md
"""
import csv
import glob
import os
import sqlite3
import sys


def from_db(path):
    c = sqlite3.connect(path)
    rows = c.execute("select name, count(*), avg(end-start), min(end-start), max(end-start), "
                     "sum(end-start) from kernels group by name order by sum(end-start) desc")
    return [(r[0], r[1], r[2], r[3], r[4], r[5]) for r in rows]


def from_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((r["Name"], int(r["Calls"]), float(r["AverageNs"]), float(r["MinNs"]),
                        float(r["MaxNs"]), float(r["TotalDurationNs"])))
    return sorted(out, key=lambda r: -r[5])


def main(path):
    if os.path.isdir(path):
        dbs = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
        csvs = glob.glob(os.path.join(path, "**", "*kernel_stats.csv"), recursive=True)
        path = (csvs or dbs)[0]
    rows = from_csv(path) if path.endswith(".csv") else from_db(path)
    print(f"source: `{path}` (rocprofv3 --kernel-trace --stats)\n")
    print("| kernel | launches | avg us | min us | max us | total ms |")
    print("|---|---|---|---|---|---|")
    for name, n, avg, mn, mx, tot in rows:
        short = name.replace("(anonymous namespace)::", "").split("(")[0]
        short = short.replace("void ", "")
        print(f"| `{short}` | {n} | {avg / 1e3:.1f} | {mn / 1e3:.1f} | {mx / 1e3:.1f} | "
              f"{tot / 1e6:.3f} |")


if __name__ == "__main__":
    main(sys.argv[1])
