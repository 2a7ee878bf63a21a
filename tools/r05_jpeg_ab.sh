# JPEG A/B (round 5): the JPEG parity tests of each variant tools/ab/libjpeg_<v>.so,
# then tools/jpeg_time.py of the product and the variants, three passes in
# alternating order.   gpurun -- 'bash tools/r05_jpeg_ab.sh v1 [v2 ...]'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05jab
mkdir -p $O
for v in "$@"; do
  LZ4JPEG_LIB=$PWD/tools/ab/libjpeg_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_jpeg.py tests/test_gpu_exe.py -m gpu -x -q --timeout 300 --timeout-method thread -k "jpeg or JPEG" > $O/tests_$v.log 2>&1 || { echo "tests $v failed"; tail -30 $O/tests_$v.log; exit 1; }
  echo "tests $v: $(tail -1 $O/tests_$v.log)"
done
for pass in 1 2 3; do
  for v in prod "$@"; do
    lib=""; [ $v = prod ] || lib=$PWD/tools/ab/libjpeg_$v.so
    echo "== $v pass $pass"; LZ4JPEG_LIB=$lib timeout -k 10 120 python3 tools/jpeg_time.py || exit 1
  done
done
