set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/decpmc
mkdir -p $O
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
B="SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $A -d $O/pa -o run -- python3 tools/dec_one.py 1073741824 3 > $O/pa.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $B -d $O/pb -o run -- python3 tools/dec_one.py 1073741824 3 > $O/pb.log 2>&1
rc=$?
for p in pa pb; do python3 tools/pmc_summary.py $O/$p/run_results.db lz4_decode_blocks > $O/$p.txt 2>&1; tail -12 $O/$p.txt; done
exit $rc
