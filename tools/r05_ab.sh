# Round-5 A/B step: issue-rate micro-benchmarks, per-basic-block counts of the
# product and of every variant named (tools/ab/bbcnt_<v>.co), then
# tools/ab4.sh (parity tests of each variant library tools/ab/liblz4_<v>.so,
# two alternating kernel-trace passes).   -> gpurun_out/r05ab/
#   gpurun -- 'bash tools/r05_ab.sh a [b ...]'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05ab
mkdir -p $O
[ -n "$AB_NORATE" ] || timeout -k 10 120 tools/ab/valu_rate > $O/valu_rate.log 2>&1 || exit 1
for v in prod "$@"; do
  if [ -f tools/ab/bbcnt_$v.co ]; then
    timeout -k 10 120 python3 tools/bbcount.py run $O $v > $O/bbcount_$v.log 2>&1 || { tail -5 $O/bbcount_$v.log; exit 1; }
  fi
  if [ -f tools/ab/bbcnt_emit_$v.co ]; then
    timeout -k 10 120 python3 tools/bbcount.py run_emit $O $v > $O/bbcount_emit_$v.log 2>&1 || { tail -5 $O/bbcount_emit_$v.log; exit 1; }
  fi
done
AB_NOPMC=1 bash tools/ab4.sh "$@"
rc=$?
if [ $rc = 0 ] && [ -n "$AB_FETCH" ]; then
  # FETCH_SIZE (KiB, x2 for 16-B streaming reads) of the compressor kernels per variant
  for v in prod "$@"; do
    lib=""; [ $v = prod ] || lib=$PWD/tools/ab/liblz4_$v.so
    LZ4JPEG_LIB=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/f_$v -o run -- python3 tools/lz4_one.py 1073741824 2 1 > $O/f_$v.log 2>&1 || { echo "fetch $v failed"; rc=1; break; }
    echo "== fetch $v"; python3 tools/pmc_summary.py $O/f_$v/run_results.db lz4_ | grep -E "dispatch|FETCH" | tail -4
  done
fi
tail -20 $O/valu_rate.log 2>/dev/null
cat $O/bbcount_*.log
exit $rc
