set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bare_decode.py tests/test_gpu_compat.py -x -q --timeout 200 --timeout-method thread > gpurun_out/bare_t.log 2>&1 || { tail -30 gpurun_out/bare_t.log; exit 1; }
tail -1 gpurun_out/bare_t.log
echo "== new"; timeout -k 10 120 python3 tools/dec_one.py 1073741824 5 || exit 1
echo "== old"; LZ4JPEG_LIB=$PWD/tools/variants/liblz4r_gpudec_old.so timeout -k 10 120 python3 tools/dec_one.py 1073741824 5
