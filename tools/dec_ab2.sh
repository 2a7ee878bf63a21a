# LZ4 decoder A/B on the GPU box: the decode parity tests on the product
# build, then the 1 GiB decode timing (tools/dec_one.py) of the product and of
# each tools/variants/liblz4_<v>.so given as an argument.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/decab2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_bare_decode.py tests/test_gpu_compat.py tests/test_gpu_lz4.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
for v in prod "$@"; do
  lib=""; [ $v = prod ] || lib=$PWD/tools/variants/liblz4_$v.so
  echo "== $v"; LZ4JPEG_LIB=$lib timeout -k 10 120 python3 tools/dec_one.py 1073741824 8 || exit 1
done
for v in prod "$@"; do
  lib=""; [ $v = prod ] || lib=$PWD/tools/variants/liblz4_$v.so
  echo "== $v (again)"; LZ4JPEG_LIB=$lib timeout -k 10 120 python3 tools/dec_one.py 1073741824 8 || exit 1
done
