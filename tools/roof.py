#!/usr/bin/env python3
"""The binding roof of lz4_tiles from one box's measurements (tools only).

    python3 tools/roof.py <dir> [out.json]

<dir> is a tools/r05_roof.sh output: pa/run_results.db (rocprofv3 --pmc pass
A over the 1 GiB compress: SQ_INSTS_*, SQ_LDS_IDX_ACTIVE, SQ_WAVES with the
kernel's duration and GRBM_GUI_ACTIVE -- counts, time and clock of one run),
bbcounts_prod.json (tools/bbcount.py: dynamic count of every basic block of
the same kernel build), valu_rate.log (tools/valu_rate.hip on the same box).

Per 300-B block (= one wave):
  VALU  a LOWER bound on the SIMD cycles its vector instructions occupy: every
        dynamic VALU instruction priced at the cheapest rate the micro-
        benchmarks show for its class at 8 waves per SIMD -- 2.33 cycles for
        the ops that issue at the dual rate beside v_add (v_add/sub/and/or/
        xor/mov, v_cndmask, 32-bit shifts, v_writelane), ~4.1 for the
        VOP3-only, compare, DPP, mbcnt, readlane, max/min and 64-bit ops,
        which cost the same alone and interleaved with v_add;
  SALU  SQ_INSTS_SALU x the s_add/xor rate (4.2 cycles per wave-instruction
        per SIMD; SALU issues beside VALU: "4 v_perm + 4 s_add" runs at the
        VALU rate);
  LDS   SQ_LDS_IDX_ACTIVE per block (LDS-array cycles, one array per CU).
A CU runs four SIMDs, so the roof in CU cycles per block is
max(VALU / 4, SALU / 4, LDS), against the measured CU cycles per block
(duration x clock x 256 CUs / blocks, clock = GRBM_GUI_ACTIVE / 8 XCDs /
duration).  frac = roof / measured <= 1 by construction of the lower bounds.
"""
import json
import os
import re
import sqlite3
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import bbcount  # noqa: E402

CUS = 256
XCDS = 8
KERNEL = "lz4_tiles<true>"

# classes whose measured rate beside v_add is the dual rate (valu_rate.log:
# "4 v_cndmask + 4 v_add" 2.38, "4 v_lshrrev + 4 v_add" 2.35, "4 v_writelane
# + 4 v_add" 2.33, "4 v_add sgpr + 4 v_add" 2.34, "4 v_mov from sgpr + 4 v_add"
# 2.36); every other class measured ~4.1 both alone and beside v_add
DUAL = {"v_add_u32", "v_sub_u32", "v_subrev_u32", "v_and_b32", "v_or_b32", "v_xor_b32",
        "v_mov_b32", "v_cndmask_b32", "v_lshlrev_b32", "v_lshrrev_b32", "v_ashrrev_i32",
        "v_writelane_b32", "v_not_b32", "v_bfrev_b32"}


def rates(log):
    """name -> cycles per wave-instruction per SIMD (grid 8192 lines)."""
    out = {}
    for line in open(log):
        m = re.match(r"(.+?)\s+grid\s+8192\s.*per SIMD\s+([\d.]+)", line)
        if m:
            out[m.group(1).strip()] = float(m.group(2))
    return out


def classes(r):
    """Lower-bound cycles per wave-instruction per SIMD of each class: the dual
    class at the v_add/mov/sub rate (they reach it beside v_add); every other
    VALU class at the cheapest solo rate of the group (beside v_add they cost
    at least as much: "4 X + 4 v_add" streams run at ~4.1 per instruction)."""
    dual = min(r["v_add/xor/and/or"], r["v_mov_b32_e32"], r["v_sub_u32_e32"])
    slow = min(r[k] for k in ("v_perm_b32", "v_alignbyte_b32", "v_mbcnt_lo/hi",
                              "v_max/min_u32_e32", "v_bfi/xad/min3/max3", "v_bfe / v_and_or",
                              "v_add3 / v_lshl_add", "v_mul_lo_u32", "v_ffbl_b32_e32",
                              "v_readfirstlane/readlane", "v_cmp_e64 -> sgpr",
                              "v_lshl_or/add_lshl/lshl_add"))
    dpp = min(r["v_max_u32_dpp"], r["v_mov_b32_dpp wave_shr"])
    return {"dual": dual, "slow": slow, "dpp": dpp, "shift64": r["v_lshl/lshrrev_b64"],
            "salu": r["s_add/xor"]}


def vcost(ins, c):
    op = ins.split()[0]
    base = re.sub(r"_e(32|64)$", "", op)
    if "_dpp" in op or " row_" in ins or "wave_sh" in ins:
        return c["dpp"]
    if base in DUAL:
        return c["dual"]
    if base in ("v_lshlrev_b64", "v_lshrrev_b64", "v_ashrrev_i64"):
        return c["shift64"]
    return c["slow"]


def pmc(db, sub=KERNEL):
    """{dispatch: {counter: value, _dur_ns}} from a rocpd .db, or from the
    JSON this tool saves beside its result (profiles/r05_roof_pmc_pa.json)."""
    if db.endswith(".json"):
        return {int(k): v for k, v in json.load(open(db)).items()}
    con = sqlite3.connect(db)
    rows = con.execute("select dispatch_id, kernel_name, counter_name, sum(value), "
                       "max(end) - min(start) from counters_collection "
                       "group by dispatch_id, kernel_name, counter_name").fetchall()
    per = {}
    for did, name, cn, v, dur in rows:
        if sub in name:
            per.setdefault(did, {})[cn] = v
            per[did]["_dur_ns"] = dur
    return per


def main(d, out=None, rates_log=None, counts=None, static=None, pmc_src=None):
    """d: a tools/r05_roof.sh output directory, or None with every input
    given (the committed profiles/r05_* copies reproduce profiles/r05_roof.json)."""
    rates_log = rates_log or os.path.join(d, "valu_rate.log")
    counts = counts or os.path.join(d, "bbcounts_prod.json")
    static = static or os.path.join(os.path.dirname(HERE), "tools", "ab", "bb_static_prod.json")
    pmc_src = pmc_src or os.path.join(d, "pa", "run_results.db")
    r = rates(rates_log)
    c = classes(r)
    C = json.load(open(counts))
    S = json.load(open(static))
    nb = C["blocks"]
    valu_n = valu_cyc = 0.0
    for (lab, ins), k in zip(S["bbs"], C["counts"]):
        for x in ins:
            if bbcount.classify(x) == "valu":
                valu_n += k
                valu_cyc += k * vcost(x, c)
    valu_n /= nb
    valu_cyc /= nb
    disp = pmc(pmc_src)
    # the timed dispatches (the last three of the run), each with its own time and clock
    runs = []
    for did in sorted(disp)[-3:]:
        p = disp[did]
        waves = p["SQ_WAVES"]
        dur = p["_dur_ns"] * 1e-9
        ghz = p["GRBM_GUI_ACTIVE"] / XCDS / dur / 1e9
        cyc = dur * ghz * 1e9 * CUS / waves
        runs.append({"dispatch": did, "ms": round(dur * 1e3, 4), "clock_ghz": round(ghz, 4),
                     "cu_cycles_per_block": round(cyc, 2),
                     "valu": p["SQ_INSTS_VALU"] / waves, "salu": p["SQ_INSTS_SALU"] / waves,
                     "lds_instr": p["SQ_INSTS_LDS"] / waves,
                     "lds_cycles": p["SQ_LDS_IDX_ACTIVE"] / waves,
                     "lds_conflict_cycles": p["SQ_LDS_BANK_CONFLICT"] / waves})
    best = min(runs, key=lambda x: x["cu_cycles_per_block"])
    med = sorted(runs, key=lambda x: x["cu_cycles_per_block"])[len(runs) // 2]
    assert abs(best["valu"] - valu_n) / valu_n < 0.005, (best["valu"], valu_n)
    pipes = {"valu": valu_cyc / 4, "salu": best["salu"] * c["salu"] / 4,
             "lds": best["lds_cycles"]}
    bind = max(pipes, key=pipes.get)
    res = {
        "kernel": "lz4_tiles<true>", "blocks": nb,
        "cost_classes_cycles_per_winstr_per_simd": {k: round(v, 3) for k, v in c.items()},
        "per_block": {
            "valu_instr": round(valu_n, 2), "valu_instr_pmc": round(best["valu"], 2),
            "salu_instr_pmc": round(best["salu"], 2), "lds_instr_pmc": round(best["lds_instr"], 2),
            "valu_simd_cycles_lower_bound": round(valu_cyc, 1),
            "salu_simd_cycles": round(best["salu"] * c["salu"], 1),
            "lds_cycles": round(best["lds_cycles"], 1),
            "lds_conflict_cycles": round(best["lds_conflict_cycles"], 1)},
        "roof_cu_cycles_per_block": {k: round(v, 1) for k, v in pipes.items()},
        "binding_pipe": bind,
        "measured": {"median": med, "best": best, "runs": runs},
        "frac": round(pipes[bind] / med["cu_cycles_per_block"], 4),
        "frac_by_pipe": {k: round(v / med["cu_cycles_per_block"], 4) for k, v in pipes.items()},
    }
    txt = json.dumps(res, indent=1)
    if out:
        open(out, "w").write(txt + "\n")
        if not pmc_src.endswith(".json"):     # the PMC rows beside it, for a re-run
            base = out.replace("_roof.json", "_roof_pmc_pa.json")
            json.dump({str(k): v for k, v in disp.items()}, open(base, "w"), indent=1)
    print(txt)
    return res


if __name__ == "__main__":
    if sys.argv[1] == "--from":      # --from rates.log counts.json static.json pmc.json [out]
        main(None, *(sys.argv[6:7] or [None]), rates_log=sys.argv[2], counts=sys.argv[3],
             static=sys.argv[4], pmc_src=sys.argv[5])
    else:
        main(*sys.argv[1:3])
