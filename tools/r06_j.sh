# round 6: PMC of lz4_decode_seq (instruction mix, wave cycles, LDS)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06j
mkdir -p $O
L=$PWD/tools/ab/liblz4r_gpudec_seq.so
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"
B="SQ_WAVES SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
LZ4JPEG_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $A -d $O/pa -o run -- python3 tools/dec_one.py 1073741824 2 > $O/pa.log 2>&1 && \
LZ4JPEG_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $B -d $O/pb -o run -- python3 tools/dec_one.py 1073741824 2 > $O/pb.log 2>&1
rc=$?
for p in pa pb; do python3 tools/pmc_summary.py $O/$p/run_results.db lz4_decode_seq > $O/$p.txt 2>&1; done
exit $rc
