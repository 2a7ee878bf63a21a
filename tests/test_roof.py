"""lz4_tiles' binding roof is reproducible from the committed round-5 profiles
(VERDICT r04 item 1): tools/roof.py over profiles/r05_valu_rate_solo.log,
r05_bbcounts.json, r05_bb_static.json and r05_roof_pmc_pa.json gives exactly
profiles/r05_roof.json, whose VALU lower bound agrees with the PMC count of
the same kernel and whose fraction is a bound (<= 1)."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
P = os.path.join(REPO, "profiles")


def test_roof_reproduces_from_profiles(tmp_path):
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import roof
    out = tmp_path / "roof.json"
    got = roof.main(None, str(out), rates_log=os.path.join(P, "r05_valu_rate_solo.log"),
                    counts=os.path.join(P, "r05_bbcounts.json"),
                    static=os.path.join(P, "r05_bb_static.json"),
                    pmc_src=os.path.join(P, "r05_roof_pmc_pa.json"))
    ref = json.load(open(os.path.join(P, "r05_roof.json")))
    assert got == ref
    pb = ref["per_block"]
    # the dynamic opcode counts and the PMC agree on the VALU instructions
    assert abs(pb["valu_instr"] - pb["valu_instr_pmc"]) < 0.5
    assert 0 < ref["frac"] <= 1 and all(0 < f <= 1 for f in ref["frac_by_pipe"].values())
    assert ref["binding_pipe"] == max(ref["roof_cu_cycles_per_block"],
                                      key=ref["roof_cu_cycles_per_block"].get)


def test_bench_reports_the_roof():
    sys.path.insert(0, REPO)
    import bench
    r = bench.issue_roof(1 << 30, 1.95)
    assert r is not None and r["binding_pipe"] in ("valu", "salu", "lds")
    # frac is this call's own time priced at the profile's clock: it moves
    # with the live kernel time; profile_frac is the profiled run's
    assert 0 < r["frac"] and 0 < r["profile_frac"] <= 1
    slower = bench.issue_roof(1 << 30, 2 * 1.95)
    assert abs(slower["frac"] - r["frac"] / 2) < 1e-3
    assert slower["profile_frac"] == r["profile_frac"]
