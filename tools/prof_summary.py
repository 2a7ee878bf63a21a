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
    """Per kernel and launch grid (a kernel launched over different grid sizes
    -- e.g. lz4_tiles over the 1 GiB bench corpus and over the 8 GiB config-4
    share -- gets one row per grid, labelled with it)."""
    c = sqlite3.connect(path)
    grids = dict(c.execute("select name, count(distinct grid_x * 65536 + grid_y) from kernels "
                           "group by name"))
    rows = c.execute("select name, grid_x, grid_y, count(*), avg(end-start), min(end-start), "
                     "max(end-start), sum(end-start) from kernels group by name, grid_x, grid_y "
                     "order by sum(end-start) desc")
    out = []
    for name, gx, gy, n, avg, mn, mx, tot in rows:
        label = name + (f" [grid {gx}x{gy}]" if grids[name] > 1 else "")
        out.append((label, n, avg, mn, mx, tot))
    return out


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
        grid = name[name.index(" [grid"):] if " [grid" in name else ""
        short = name.replace("(anonymous namespace)::", "").split("(")[0]
        short = short.replace("void ", "") + grid
        print(f"| `{short}` | {n} | {avg / 1e3:.1f} | {mn / 1e3:.1f} | {mx / 1e3:.1f} | "
              f"{tot / 1e6:.3f} |")


if __name__ == "__main__":
    main(sys.argv[1])
