# Round-4 A/B of lz4_tiles builds: the product's LZ4 parity tests (full
# lz4 file incl. the full-size md5s, compat, decode), then kernel-trace timing
# of the product and every variant tools/ab/liblz4_<v>.so named as an
# argument, two passes in alternating order (1 GiB, 8 calls after 3 warm-up),
# then per-block PMC (tools/lz4_ldsab.sh) of all of them.
#   gpurun -- 'bash tools/ab4.sh base [v2 ...]'   -> gpurun_out/ab4/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab4
mkdir -p $O
if [ -z "$AB_NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_lz4.py tests/test_gpu_compat.py tests/test_gpu_decode.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  echo "tests: $(tail -1 $O/tests.log)"
  for v in "$@"; do
    LZ4JPEG_LIB=$PWD/tools/ab/liblz4_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_lz4.py tests/test_gpu_compat.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_$v.log 2>&1 || { echo "tests $v failed"; tail -30 $O/tests_$v.log; exit 1; }
    echo "tests $v: $(tail -1 $O/tests_$v.log)"
  done
fi
for pass in 1 2; do
  for v in prod "$@"; do
    lib=""; [ $v = prod ] || lib=$PWD/tools/ab/liblz4_$v.so
    LZ4JPEG_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/p_${v}_$pass -o run -- python3 tools/lz4_one.py 1073741824 8 3 > $O/p_${v}_$pass.log 2>&1 || { tail -5 $O/p_${v}_$pass.log; exit 1; }
    echo "== $v pass $pass: $(tail -1 $O/p_${v}_$pass.log)"
    python3 tools/prof_summary.py $O/p_${v}_$pass/run_results.db | grep -E 'lz4_(tiles|emit|pairs)' | head -3
  done
done
[ -n "$AB_NOPMC" ] || bash tools/lz4_ldsab.sh "$@"
