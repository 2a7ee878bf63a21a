# decoder PMC: staged (default) vs global path, 256 MiB
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
C1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT"
C2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE"
for v in 0; do
  LZ4R_DECODE_STAGE_BYTES=$v timeout -k 10 120 python3 tools/dec_one.py 268435456 3 > gpurun_out/dec_$v.log 2>&1 || exit 1
  LZ4R_DECODE_STAGE_BYTES=$v timeout -k 10 200 rocprofv3 --kernel-trace --pmc $C1 -d gpurun_out/dpmcA_$v -o run -- python3 tools/dec_one.py 268435456 2 > gpurun_out/dpmcA_$v.log 2>&1 || exit 1
  LZ4R_DECODE_STAGE_BYTES=$v timeout -k 10 200 rocprofv3 --kernel-trace --pmc $C2 -d gpurun_out/dpmcB_$v -o run -- python3 tools/dec_one.py 268435456 2 > gpurun_out/dpmcB_$v.log 2>&1 || exit 1
  echo "== stage $v"; cat gpurun_out/dec_$v.log
  python3 tools/pmc_summary.py gpurun_out/dpmcA_$v/run_results.db decode_blocks | tail -12
  python3 tools/pmc_summary.py gpurun_out/dpmcB_$v/run_results.db decode_blocks | tail -12
done
