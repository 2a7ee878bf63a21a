# A/B check of compressor variant libraries (tools/variants/liblz4_<name>.so):
# GPU LZ4 parity tests through each, then 1 GiB timings of the product build and them.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "$@"; do
  LZ4JPEG_LIB=$PWD/tools/variants/liblz4_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_lz4.py tests/test_gpu_decode.py -x -q --timeout 120 --timeout-method thread -m "gpu and not slow" > gpurun_out/var_t_$v.log 2>&1 || { tail -30 gpurun_out/var_t_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/var_t_$v.log)"
done
timeout -k 10 120 python3 tools/lz4_one.py 1073741824 4 > gpurun_out/var_base.log 2>&1 || exit 1
echo "base: $(tail -1 gpurun_out/var_base.log)"
for v in "$@"; do
  LZ4JPEG_LIB=$PWD/tools/variants/liblz4_$v.so timeout -k 10 120 python3 tools/lz4_one.py 1073741824 4 > gpurun_out/var_$v.log 2>&1 || exit 1
  echo "$v: $(tail -1 gpurun_out/var_$v.log)"
done
