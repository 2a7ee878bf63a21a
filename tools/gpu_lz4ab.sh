# LZ4 compressor A/B on the GPU box: for the product build and each variant
# tools/variants/liblz4_<v>.so given as an argument: the LZ4 parity tests
# (variants only; not slow), 1 GiB timing (medians of 12 calls) and PMC
# instruction counts per block of lz4_tiles plus the per-kernel durations.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab
mkdir -p $O
C1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH"
run() {  # name lib
  LZ4JPEG_LIB=$2 timeout -k 10 120 python3 tools/lz4_one.py 1073741824 12 > $O/time_$1.log 2>&1 || return 1
  LZ4JPEG_LIB=$2 timeout -k 10 200 rocprofv3 --kernel-trace --stats --pmc $C1 -d $O/p_$1 -o run -- python3 tools/lz4_one.py 268435456 2 1 > $O/p_$1.log 2>&1 || return 1
  echo "== $1: $(tail -1 $O/time_$1.log)"
  python3 tools/pmc_summary.py $O/p_$1/run_results.db lz4_tiles | python3 -c "
import sys
v = {}
for line in sys.stdin:
    p = line.split()
    if len(p) == 2 and p[0].startswith('SQ_'): v[p[0]] = v.get(p[0], 0) + float(p[1])
w = v.get('SQ_WAVES', 1)
print('   lz4_tiles per block: ' + ', '.join(f'{k[8:]} {v[k] / w:.1f}' for k in sorted(v) if k != 'SQ_WAVES'))"
  python3 - $O/p_$1/run_results.db <<'PY'
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
for name, n, avg in c.execute("select name, count(*), avg(end-start) from kernels "
                              "group by name"):
    if "lz4_" in name:
        short = name.split("(")[0].split("::")[-1]
        print(f"   {short:20s} x{n}  {avg / 1e3:8.1f} us (256 MiB)")
        v = dict(c.execute("select counter_name, sum(value) / count(distinct dispatch_id) "
                           "from counters_collection where kernel_name = ? "
                           "group by counter_name", (name,)).fetchall())
        if v.get("SQ_WAVES"):
            w = v["SQ_WAVES"]
            print("      per wave: " + ", ".join(f"{k[8:]} {v[k] / w:.1f}" for k in sorted(v)
                                                if k != "SQ_WAVES") + f"  (waves {w:.0f})")
PY
}
run product $PWD/lz4-jpeg_amd/lz4jpeg/liblz4jpeg.so || exit 1
for v in "$@"; do
  L=$PWD/tools/variants/liblz4_$v.so
  LZ4JPEG_LIB=$L timeout -k 10 400 python -m pytest tests/test_gpu_lz4.py tests/test_gpu_decode.py tests/test_gpu_compat.py -x -q -m "gpu and not slow" > $O/t_$v.log 2>&1 || { echo "tests $v failed"; tail -30 $O/t_$v.log; exit 1; }
  echo "-- $v tests: $(tail -1 $O/t_$v.log)"
  run $v $L || exit 1
done
