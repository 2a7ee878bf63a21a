#!/usr/bin/env python3
"""The last N dispatches of a rocprofv3 --kernel-trace run (rocpd .db) in
time order: gap since the previous dispatch ended, duration, name.

    python tools/trace_gaps.py gpurun_out/x/run_results.db [N]
"""
import sqlite3
import sys


def main(path, n=12):
    c = sqlite3.connect(path)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    rows = rows[-n:]
    prev = None
    for name, s, e in rows:
        gap = "" if prev is None else f"{(s - prev) / 1e3:8.2f}"
        short = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        print(f"gap us {gap:>8s}  dur us {(e - s) / 1e3:8.2f}  {short[:70]}")
        prev = e


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 12)
