#!/usr/bin/env python3
"""Summarise tools/issue.sh: per-launch wave-instruction counts of lz4_tiles
(mean over the profiled launches) and the SIMD issue rates measured by
tools/valu_rate.hip at full occupancy (wave-instructions per second, chip)."""
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load  # noqa: E402

d = sys.argv[1]
rates = {}
for line in open(os.path.join(d, "valu_rate.log")):
    m = re.match(r"(.+?)\s+grid\s+(\d+)\s+([\d.]+) ms", line)
    if m and int(m.group(2)) == 8192:                      # 8 waves per SIMD on 256 CUs
        winstr = 8192 * 4096 * 8                             # grid x REP x 8 per iteration
        rates[m.group(1).strip()] = winstr / (float(m.group(3)) * 1e-3)
res = load(os.path.join(d, "lz4", "run_results.db"), "lz4_tiles")
per = [cs for (_, _), cs in sorted(res.items())]
keys = ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_BRANCH"]
mean = {k: sum(c.get(k, 0) for c in per) / max(1, len(per)) for k in keys}
print(json.dumps({
    "lz4": {"kernel": "lz4_tiles", "launches": len(per), "bytes_per_launch": 1 << 30,
            "per_launch": mean},
    "issue_rates_winstr_per_s": rates,
    "note": "rates: tools/valu_rate.hip, 8192 one-wave workgroups (8 waves per SIMD), "
            "REP 4096 x 8 independent instructions per wave; counts: rocprofv3 --pmc",
}, indent=1))
