# lz4_tiles / lz4_pairs kernel time at several input sizes (the smaller ones
# stay in the Infinity Cache between calls) for the product and variants:
#   gpurun -- 'bash tools/ab_small.sh v1 v2 ...'  -> gpurun_out/abs/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/abs
mkdir -p $O
for n in 33554432 134217728 1073741824; do
  for v in prod "$@"; do
    lib=""; [ $v = prod ] || lib=$PWD/tools/variants/liblz4_$v.so
    LZ4JPEG_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/p_${v}_$n -o run -- python3 tools/lz4_one.py $n 20 3 > $O/p_${v}_$n.log 2>&1 || { tail -5 $O/p_${v}_$n.log; exit 1; }
    echo "$v $n: $(python3 tools/prof_summary.py $O/p_${v}_$n/run_results.db | grep -E 'lz4_(tiles|pairs)' | awk -F'|' '{printf "%s %s  ", $2, $4}')"
  done
done
