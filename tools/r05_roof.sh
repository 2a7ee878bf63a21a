# lz4_tiles roof inputs, one box: per-basic-block dynamic
# counts (tools/bbcount.py), the VALU/SALU issue costs (tools/valu_rate.hip),
# and two PMC passes over the same 1 GiB compress that each carry the
# kernel's own time and clock (GRBM_GUI_ACTIVE beside the SQ counters):
# A = instruction counts + LDS cycles, B = the wave-cycle breakdown.
# -> gpurun_out/r05roof/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05roof
mkdir -p $O
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
B="SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU2 GRBM_GUI_ACTIVE GRBM_COUNT"
C="SQ_WAVES SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -k 10 120 python3 tools/bbcount.py run $O prod > $O/bbcount.log 2>&1 && \
timeout -k 10 120 tools/ab/valu_rate > $O/valu_rate.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $A -d $O/pa -o run -- python3 tools/lz4_one.py 1073741824 3 20 > $O/pa.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $B -d $O/pb -o run -- python3 tools/lz4_one.py 1073741824 3 20 > $O/pb.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d $O/pc -o run -- python3 tools/lz4_one.py 1073741824 3 20 > $O/pc.log 2>&1
rc=$?
cat $O/bbcount.log; cat $O/valu_rate.log | tail -40
for p in pa pb pc; do python3 tools/pmc_summary.py $O/$p/run_results.db lz4_tiles > $O/$p.txt 2>&1; tail -14 $O/$p.txt; done
exit $rc
