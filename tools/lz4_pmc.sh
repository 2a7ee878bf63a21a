# PMC passes over both compressor kernels (lz4_tiles, lz4_emit) on 1 GiB:
# instruction mix, wave-cycle breakdown, LDS stalls, HBM traffic.
# usage: bash tools/lz4_pmc.sh [lib.so]  -> gpurun_out/lz4pmc/summary.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/lz4pmc
mkdir -p $D
LIB=${1:-$PWD/lz4-jpeg_amd/lz4jpeg/liblz4jpeg.so}
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"
P2="SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_UNALIGNED_STALL SQ_BUSY_CYCLES"
i=0
for P in "$P1" "$P2" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  LZ4JPEG_LIB=$LIB timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P -d $D/p$i -o run -- python3 tools/lz4_one.py 1073741824 2 1 > $D/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $D/p$i.log; exit 1; }
done
for i in 1 2 3 4; do python3 tools/pmc_summary.py $D/p$i/run_results.db lz4_ ; done > $D/summary.txt
cat $D/summary.txt
