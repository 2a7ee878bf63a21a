set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in 0 1; do
LZ4JPEG_LIB=$PWD/tools/variants/liblz4_v$v.so timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/pmcv$v -o run -- python3 tools/lz4_one.py 268435456 2 > gpurun_out/pmcv$v.log 2>&1 || exit 1
LZ4JPEG_LIB=$PWD/tools/variants/liblz4_v$v.so timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM -d gpurun_out/pmcw$v -o run -- python3 tools/lz4_one.py 268435456 2 > gpurun_out/pmcw$v.log 2>&1 || exit 1
done
