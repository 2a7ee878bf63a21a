# round 6: kernel trace of the entropy stage (product and the merged decode
# variant): dispatch durations and the gaps between them
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06o
mkdir -p $O
for v in prod merged; do
  L=""; [ $v = prod ] || L=$PWD/tools/ab/libjpegr_entropy_$v.so
  LZ4JPEG_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-trace -d $O/$v -o run -- python3 tools/ent_one.py 4 > $O/$v.log 2>&1 || exit 1
  python3 tools/trace_gaps.py $(ls $O/$v/*/run_results.db $O/$v/run_results.db 2>/dev/null | head -1) 14 > $O/${v}_gaps.txt
  cat $O/${v}_gaps.txt; grep "decode ms" $O/$v.log | tail -2
done
