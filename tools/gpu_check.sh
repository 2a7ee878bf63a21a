# Re-entry check on the GPU box: parity tests + PMC instruction mix of lz4_tiles
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t1.log 2>&1 && \
bash tools/lz4_pmc_var.sh > gpurun_out/pmc_base.log 2>&1
rc=$?
tail -3 gpurun_out/t1.log; cat gpurun_out/pmc_base.log
exit $rc
