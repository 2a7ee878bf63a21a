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
  [ -f tools/ab/bbcnt_$v.co ] || continue
  timeout -k 10 120 python3 tools/bbcount.py run $O $v > $O/bbcount_$v.log 2>&1 || { tail -5 $O/bbcount_$v.log; exit 1; }
done
AB_NOPMC=1 bash tools/ab4.sh "$@"
rc=$?
tail -20 $O/valu_rate.log 2>/dev/null
cat $O/bbcount_*.log
exit $rc
