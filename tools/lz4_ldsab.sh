# lz4_tiles PMC A/B: instruction mix, wave-cycle breakdown and LDS array
# counters per block (per wave) for the product build and each variant
# tools/ab/liblz4_<v>.so named as an argument.
# usage: bash tools/lz4_ldsab.sh v1 v2 ...  -> gpurun_out/ldsab/summary.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/ldsab
mkdir -p $D
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"
P2="SQ_WAVES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
run() {  # name lib
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    LZ4JPEG_LIB=$2 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P -d $D/$1_$i -o run -- python3 tools/lz4_one.py 268435456 1 1 > $D/$1_$i.log 2>&1 || { echo "pass $1 $i failed"; tail -5 $D/$1_$i.log; return 1; }
  done
  echo "== $1"
  python3 - $D/$1_1/run_results.db $D/$1_2/run_results.db <<'PY'
import sqlite3, sys
out = {}
for db in sys.argv[1:]:
    c = sqlite3.connect(db)
    for name, cn, v, nd, dur in c.execute(
            "select k.name, cc.counter_name, sum(cc.value), count(distinct cc.dispatch_id), "
            "avg(k.end - k.start) from counters_collection cc join kernels k "
            "on k.dispatch_id = cc.dispatch_id where k.name like '%lz4_tiles%' "
            "group by cc.counter_name"):
        out[cn] = v / nd
        out["_ns"] = dur
w = out.pop("SQ_WAVES")
ns = out.pop("_ns")
print(f"   lz4_tiles {ns / 1e3:.1f} us / 256 MiB; per block: " +
      ", ".join(f"{k.replace('SQ_', '')} {v / w:.1f}" for k, v in sorted(out.items())))
PY
}
run product $PWD/lz4-jpeg_amd/lz4jpeg/liblz4jpeg.so || exit 1
for v in "$@"; do run $v $PWD/tools/ab/liblz4_$v.so || exit 1; done
