"""Per-dispatch durations and gaps of jpeg_strip_kernel from a rocprofv3
kernel-trace database (tools/jpeg_trace.sh)."""
import glob
import sqlite3
import sys

db = glob.glob(sys.argv[1] + "/**/*.db", recursive=True)[0]
con = sqlite3.connect(db)
tabs = [r[0] for r in con.execute("select name from sqlite_master where type='table'")]
kt = [t for t in tabs if t.startswith("rocpd_kernel_dispatch")][0]
rows = con.execute(f"select start, end, grid_size_y from {kt} where grid_size_x = 1036800 "
                   "order by start").fetchall()
for g in sorted({r[2] for r in rows}):
    rs = [r for r in rows if r[2] == g]
    d = sorted((e - s) / 1e3 for s, e, _ in rs)
    gaps = sorted((rs[i + 1][0] - rs[i][1]) / 1e3 for i in range(len(rs) - 1))
    pct = lambda a, q: a[min(len(a) - 1, int(q * len(a)))]
    print(f"images {g}: n {len(d)} dur p5 {pct(d, .05):.1f} p50 {pct(d, .5):.1f} p95 {pct(d, .95):.1f}"
          f" | gap p5 {pct(gaps, .05):.1f} p50 {pct(gaps, .5):.1f} p95 {pct(gaps, .95):.1f} us")
    seq = [(e - s) / 1e3 for s, e, _ in rs[:40]]
    print("   first 40:", " ".join(f"{x:.0f}" for x in seq))
