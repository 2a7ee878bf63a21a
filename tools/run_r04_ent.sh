# round 4: entropy decode variants (tools/variants/libjpegr_entropy_<v>.so), twice, plus a
# kernel trace of the product's entropy calls
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_ent.sh side fill pf2 both newloop && bash tools/gpu_ent.sh side fill pf2 both && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/entprof -o run -- python3 tools/ent_scan.py > gpurun_out/entprof.log 2>&1 && \
python3 tools/prof_summary.py gpurun_out/entprof/run_results.db | grep entropy
