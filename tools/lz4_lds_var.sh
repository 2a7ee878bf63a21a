# LDS cost of lz4_tiles per variant build (tools/variants/liblz4_<name>.so), 256 MiB:
# array-busy cycles, bank-conflict cycles, unaligned stalls, LDS instructions.
# usage: bash tools/lz4_lds_var.sh <names...>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
C="SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU"
for v in "$@"; do
  LZ4JPEG_LIB=$PWD/tools/variants/liblz4_$v.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d gpurun_out/lds_$v -o run -- python3 tools/lz4_one.py 268435456 1 > gpurun_out/lds_$v.log 2>&1 || exit 1
  echo "== $v"
  python3 tools/pmc_summary.py gpurun_out/lds_$v/run_results.db lz4_tiles
done
