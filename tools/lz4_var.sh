# time variant .so builds of the compressor (tools/variants/) against the product build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/lz4_one.py 1073741824 3 > gpurun_out/var_base.log 2>&1 || exit 1
for v in "$@"; do
  LZ4JPEG_LIB=$PWD/tools/variants/liblz4_v$v.so timeout -k 10 120 python3 tools/lz4_one.py 1073741824 3 > gpurun_out/var_$v.log 2>&1 || exit 1
done
echo "base: $(tail -1 gpurun_out/var_base.log)"
for v in "$@"; do echo "variant $v: $(tail -1 gpurun_out/var_$v.log)"; done
