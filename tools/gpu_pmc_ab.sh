# PMC instruction mix + LDS bank conflicts of lz4_tiles: product build vs variant libs
# usage: bash tools/gpu_pmc_ab.sh <variant names (tools/variants/liblz4_<name>.so)>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
C1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM"
C2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
run() {  # name lib
  LZ4JPEG_LIB=$2 timeout -k 10 200 rocprofv3 --kernel-trace --pmc $C1 -d gpurun_out/pa_$1 -o run -- python3 tools/lz4_one.py 268435456 1 > gpurun_out/pa_$1.log 2>&1 || return 1
  LZ4JPEG_LIB=$2 timeout -k 10 200 rocprofv3 --kernel-trace --pmc $C2 -d gpurun_out/pb_$1 -o run -- python3 tools/lz4_one.py 268435456 1 > gpurun_out/pb_$1.log 2>&1 || return 1
  echo "== $1"
  python3 tools/pmc_summary.py gpurun_out/pa_$1/run_results.db lz4_tiles | grep -v _dur
  python3 tools/pmc_summary.py gpurun_out/pb_$1/run_results.db lz4_tiles | grep -v _dur
}
run base $PWD/lz4-jpeg_amd/lz4jpeg/liblz4jpeg.so || exit 1
for v in "$@"; do run $v $PWD/tools/variants/liblz4_$v.so || exit 1; done
