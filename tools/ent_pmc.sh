# entropy-stage timing + PMC (instructions, waits, LDS conflicts)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
C1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT"
C2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"
timeout -k 10 120 python3 tools/ent_one.py 4 > gpurun_out/ent_one.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --pmc $C1 -d gpurun_out/epmcA -o run -- python3 tools/ent_one.py 1 > gpurun_out/epmcA.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --pmc $C2 -d gpurun_out/epmcB -o run -- python3 tools/ent_one.py 1 > gpurun_out/epmcB.log 2>&1
rc=$?
cat gpurun_out/ent_one.log
python3 tools/pmc_summary.py gpurun_out/epmcA/run_results.db entropy_ | grep -v "^   _dur" 
python3 tools/pmc_summary.py gpurun_out/epmcB/run_results.db entropy_ | grep -v "^   _dur"
exit $rc
