# lz4_emit A/B on the GPU box: LZ4 parity tests on the product build, then
# 1 GiB timing and kernel-trace durations of the product and of the
# LDS-image emission (tools/variants/liblz4_v0.so, built with
# EXTRA=-DLZ4R_EMIT_IMG), then the scattered-store rate micro-benchmark.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/emit
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_lz4.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1; rc=$?
tail -3 $O/t.log
[ $rc -eq 0 ] || { tail -60 $O/t.log; exit $rc; }
for v in prod img; do
  lib=""; [ $v = img ] && lib=$PWD/tools/variants/liblz4_v0.so
  LZ4JPEG_LIB=$lib timeout -k 10 120 python3 tools/lz4_one.py 1073741824 12 > $O/time_$v.log 2>&1 || exit 1
  echo "== $v: $(tail -1 $O/time_$v.log)"
  LZ4JPEG_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/p_$v -o run -- python3 tools/lz4_one.py 1073741824 5 2 > $O/p_$v.log 2>&1 || exit 1
  python3 tools/prof_summary.py $O/p_$v | grep -E 'lz4_' | head -8
done
timeout -k 10 60 ./tools/store_rate
