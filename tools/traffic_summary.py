#!/usr/bin/env python3
"""Per-launch HBM traffic of lz4_tiles, lz4_emit, jpeg_strip_kernel and the others from the PMC
passes written by tools/traffic.sh.

FETCH_SIZE / WRITE_SIZE are rocprofv3 derived counters in KiB (summed over
the XCD L2 channels).  gfx950 correction (MI355X_MICROARCH.md, HBM): for
16-B-per-lane streaming reads FETCH_SIZE reports half the bytes, so it is
doubled; both kernels read their inputs with 16-B loads.  WRITE_SIZE is
exact for 16-B-per-lane stores.  The first launch of each kernel is dropped
(cold caches, first-touch)."""
import json
import os
import sqlite3
import sys


def per_launch(db, counter, kernel_sub):
    c = sqlite3.connect(db)
    rows = c.execute("select dispatch_id, kernel_name, sum(value) from counters_collection "
                     "where counter_name = ? group by dispatch_id order by dispatch_id",
                     (counter,)).fetchall()
    vals = [v for _, name, v in rows if kernel_sub in name]
    return vals[1:] if len(vals) > 1 else vals


def main(d):
    out = {}
    for kern, run, sub in (("lz4", "lz4", "lz4_tiles"), ("lz4_emit", "lz4", "lz4_emit"),
                           ("jpeg", "jpeg", "jpeg_strip_kernel"),
                           ("lz4_decode", "dec", "lz4_decode_blocks"),
                           ("entropy_encode", "ent", "entropy_encode_lane"),
                           ("entropy_decode", "ent", "entropy_decode_kernel")):
        f = per_launch(os.path.join(d, f"{run}_fetch", "run_results.db"), "FETCH_SIZE", sub)
        w = per_launch(os.path.join(d, f"{run}_write", "run_results.db"), "WRITE_SIZE", sub)
        if not f or not w:
            continue
        # the x2 rule is stated for 16-B-per-lane streaming reads (lz4_tiles,
        # jpeg); the decoder / entropy kernels read 2..16 B per lane, so their
        # doubled figure is an upper estimate -- the raw KiB are kept beside it
        fetch = 2 * 1024 * sum(f) / len(f)
        write = 1024 * sum(w) / len(w)
        out[kern] = {"kernel": sub, "fetch_bytes": fetch, "write_bytes": write,
                     "traffic_bytes": fetch + write, "launches": [len(f), len(w)],
                     "raw_fetch_kib": f, "raw_write_kib": w}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
