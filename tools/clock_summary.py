"""Effective clock per kernel from a GRBM_GUI_ACTIVE --pmc pass (tools/clock_pmc.sh):
GRBM_GUI_ACTIVE is summed over the 8 XCDs, so clock = value / 8 / duration
(MI355X_MICROARCH.md, DVFS give-back; it reads high on dispatches under ~0.3 ms,
which are skipped)."""
import glob
import json
import os
import sqlite3
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/clock"
res = {}
for db in sorted(glob.glob(os.path.join(root, "*", "run_results.db"))):
    c = sqlite3.connect(db)
    per = {}
    for name, v, dur in c.execute(
            "select kernel_name, sum(value), max(end) - min(start) from counters_collection "
            "where counter_name = 'GRBM_GUI_ACTIVE' group by dispatch_id, kernel_name"):
        if not dur or dur < 300e3:                    # ns
            continue
        short = name.replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1]
        per.setdefault(short, []).append(v / 8 / dur)    # cycles per ns = GHz
    for k, v in per.items():
        v.sort()
        res[os.path.basename(os.path.dirname(db)) + ":" + k] = {"ghz_median": round(v[len(v) // 2], 3), "ghz_min": round(v[0], 3),
                  "ghz_max": round(v[-1], 3), "dispatches": len(v)}
print(json.dumps(res, indent=1))
