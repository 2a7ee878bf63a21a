# Instruction-issue roof of lz4_tiles: the measured wave64 issue rates of the
# SIMDs (tools/valu_rate.hip at 8 waves per SIMD) and the kernel's per-launch
# instruction counts (rocprofv3 --pmc, 1 GiB corpus).  -> gpurun_out/issue/issue.json
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/issue
mkdir -p $D
timeout -k 10 60 tools/ab/valu_rate > $D/valu_rate.log 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH -d $D/lz4 -o run -- python3 tools/lz4_one.py 1073741824 3 > $D/lz4.log 2>&1 && \
python3 tools/issue_summary.py $D > $D/issue.json && cat $D/issue.json
