#!/usr/bin/env python3
"""Per-kernel, per-dispatch PMC totals from a rocprofv3 --pmc run (rocpd .db).

    python tools/pmc_summary.py gpurun_out/pmc1/run_results.db [kernel-substring]
"""
import sqlite3
import sys
from collections import defaultdict


def load(path, sub=""):
    c = sqlite3.connect(path)
    rows = c.execute("select dispatch_id, kernel_name, counter_name, sum(value), "
                     "max(end) - min(start) from counters_collection "
                     "group by dispatch_id, kernel_name, counter_name").fetchall()
    out = defaultdict(dict)
    for did, name, cn, v, dur in rows:
        if sub in name:
            out[(did, name)][cn] = v
            out[(did, name)]["_dur_ns"] = dur
    return out


if __name__ == "__main__":
    res = load(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
    for (did, name), cs in sorted(res.items()):
        print(f"dispatch {did} {name[:60]}")
        for k in sorted(cs):
            print(f"   {k:28s} {cs[k]:.6g}")
