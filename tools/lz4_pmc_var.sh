# PMC instruction mix of the compressor: product build vs variant builds (256 MiB)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
C1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM"
C2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
run() {  # name lib
  LZ4JPEG_LIB=$2 timeout -k 10 200 rocprofv3 --kernel-trace --pmc $C1 -d gpurun_out/lpA_$1 -o run -- python3 tools/lz4_one.py 268435456 1 > gpurun_out/lpA_$1.log 2>&1 || return 1
  LZ4JPEG_LIB=$2 timeout -k 10 200 rocprofv3 --kernel-trace --pmc $C2 -d gpurun_out/lpB_$1 -o run -- python3 tools/lz4_one.py 268435456 1 > gpurun_out/lpB_$1.log 2>&1 || return 1
  echo "== $1"
  python3 tools/pmc_summary.py gpurun_out/lpA_$1/run_results.db lz4_tiles | grep -v _dur
  python3 tools/pmc_summary.py gpurun_out/lpB_$1/run_results.db lz4_tiles | grep -v _dur
}
run base $PWD/lz4-jpeg_amd/lz4jpeg/liblz4jpeg.so || exit 1
for v in "$@"; do run v$v $PWD/tools/variants/liblz4_v$v.so || exit 1; done
