# round 6: kernel times of the bare-stream decode, product vs a gpudec variant
#   bash tools/r06_u.sh <variant>
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06u
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prod -o run -- python3 tools/dec_one.py 1073741824 5 > $O/prod.log 2>&1 && \
LZ4JPEG_LIB=$PWD/tools/ab/liblz4r_gpudec_$1.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/$1 -o run -- python3 tools/dec_one.py 1073741824 5 > $O/$1.log 2>&1 && \
for v in prod $1; do echo "== $v"; python3 tools/prof_summary.py $O/$v | grep -E "bare|decode_blocks"; done
