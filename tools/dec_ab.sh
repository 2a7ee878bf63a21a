# LZ4 decoder A/B on the GPU box: the product build, then each variant
# tools/variants/liblz4r_gpudec_<v>.so given as an argument: the decode
# parity tests (variants only) and the 1 GiB decode timing (tools/dec_one.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/decab
mkdir -p $O
echo "== product"; timeout -k 10 120 python3 tools/dec_one.py 1073741824 5 || exit 1
for v in "$@"; do
  L=$PWD/tools/variants/liblz4r_gpudec_$v.so
  LZ4JPEG_LIB=$L timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_bare_decode.py tests/test_gpu_compat.py -x -q -m "gpu and not slow" --timeout 200 --timeout-method thread > $O/t_$v.log 2>&1 || { echo "tests $v failed"; tail -30 $O/t_$v.log; exit 1; }
  echo "== $v: $(tail -1 $O/t_$v.log)"
  LZ4JPEG_LIB=$L timeout -k 10 120 python3 tools/dec_one.py 1073741824 5 || exit 1
done
