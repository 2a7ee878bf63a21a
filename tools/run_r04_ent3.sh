# round 4: entropy encode phase cuts (ca: after the count, cb: after the tree; timing only,
# the streams are wrong on purpose), PMC mix of the product's entropy kernels, kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/ent_time_ab.sh ca cb && bash tools/gpu_pmc_ent.sh > gpurun_out/pent.txt 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/entprof -o run -- python3 tools/ent_scan.py > gpurun_out/entprof.log 2>&1 && \
python3 tools/prof_summary.py gpurun_out/entprof/run_results.db | grep entropy
