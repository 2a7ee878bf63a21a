# round 6: vector-memory pipe and wave-state counters of lz4_decode_blocks
# (is the TA the bound?): two passes
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06w
mkdir -p $O
C="TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES"
D="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD"
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C -d $O/pa -o run -- python3 tools/dec_one.py 1073741824 2 > $O/pa.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $D -d $O/pb -o run -- python3 tools/dec_one.py 1073741824 2 > $O/pb.log 2>&1
rc=$?
for p in pa pb; do python3 tools/pmc_summary.py $O/$p/run_results.db lz4_decode_blocks > $O/$p.txt 2>&1; head -10 $O/$p.txt; done
exit $rc
