# PMC profile of the placement kernel lz4_gather (256 MiB corpus): instruction
# mix, LDS cycles, wave time and waits
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
C1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT"
C2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C1 -d gpurun_out/gp1 -o run -- python3 tools/lz4_one.py 268435456 1 > gpurun_out/gp1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C2 -d gpurun_out/gp2 -o run -- python3 tools/lz4_one.py 268435456 1 > gpurun_out/gp2.log 2>&1 && \
python3 tools/pmc_summary.py gpurun_out/gp1/run_results.db lz4_gather && \
python3 tools/pmc_summary.py gpurun_out/gp2/run_results.db lz4_gather
