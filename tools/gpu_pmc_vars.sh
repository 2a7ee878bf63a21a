# issue-rate microbenchmark + PMC instruction mix of lz4_tiles per ablation variant
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 tools/variants/valu_rate > gpurun_out/valu_rate.log 2>&1 && cat gpurun_out/valu_rate.log && \
bash tools/lz4_pmc_var.sh "$@" > gpurun_out/pmc_vars.log 2>&1
rc=$?
cat gpurun_out/pmc_vars.log
exit $rc
