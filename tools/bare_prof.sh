set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/bp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/bp/new -o run -- python3 tools/dec_one.py 1073741824 5 > gpurun_out/bp/new.log 2>&1 && \
LZ4JPEG_LIB=$PWD/tools/variants/liblz4r_gpudec_old.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/bp/old -o run -- python3 tools/dec_one.py 1073741824 5 > gpurun_out/bp/old.log 2>&1 && \
for v in new old; do echo "== $v"; python3 tools/prof_summary.py gpurun_out/bp/$v | grep -E "bare|decode_blocks"; done
