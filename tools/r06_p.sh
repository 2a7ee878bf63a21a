# round 6: PMC of the merged entropy decode kernel (bm variant): issue, wait,
# LDS / VMEM latency (INST_LEVEL / INSTS)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06p
mkdir -p $O
L=$PWD/tools/ab/libjpegr_entropy_${1:-bm}.so
A="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_INSTS_VALU"
B="SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM"
C="SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_BUSY_CYCLES"
for p in A B C; do
  eval cs=\$$p
  LZ4JPEG_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $cs -d $O/$p -o run -- python3 tools/ent_one.py 3 > $O/$p.log 2>&1 || { tail -5 $O/$p.log; exit 1; }
  python3 tools/pmc_summary.py $O/$p/run_results.db entropy_decode | tail -10
done
