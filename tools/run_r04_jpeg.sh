# round 4: JPEG strip-width A/B (tools/variants/libjpeg_<v>.so): the variant's JPEG parity
# tests, then alternating timing passes (one-image launches repeated: the first warms the clock)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in "$@"; do
  LZ4JPEG_LIB=$PWD/tools/variants/libjpeg_$v.so timeout -k 10 400 python -m pytest tests/test_gpu_jpeg.py -x -q > gpurun_out/jt_$v.log 2>&1 || { tail -20 gpurun_out/jt_$v.log; exit 1; }
  echo "tests $v: $(tail -1 gpurun_out/jt_$v.log)"
done
for pass in 1 2; do
  echo "== product pass $pass"; timeout -k 10 120 python3 tools/jpeg_scan.py 1 1 1 128 || exit 1
  for v in "$@"; do
    echo "== $v pass $pass"; LZ4JPEG_LIB=$PWD/tools/variants/libjpeg_$v.so timeout -k 10 120 python3 tools/jpeg_scan.py 1 1 1 128 || exit 1
  done
done
