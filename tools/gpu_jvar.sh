# A/B of JPEG variant libraries: GPU JPEG parity tests through each, then 4K encode timings
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "$@"; do
  LZ4JPEG_LIB=$PWD/tools/variants/liblz4_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_jpeg.py tests/test_gpu_reconstruct.py -x -q --timeout 120 --timeout-method thread -m "gpu and not slow" > gpurun_out/jvar_t_$v.log 2>&1 || { tail -30 gpurun_out/jvar_t_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/jvar_t_$v.log)"
done
echo "base: $(timeout -k 10 120 python3 tools/jpeg_time.py)" || exit 1
for v in "$@"; do
  echo "$v: $(LZ4JPEG_LIB=$PWD/tools/variants/liblz4_$v.so timeout -k 10 120 python3 tools/jpeg_time.py)" || exit 1
done
