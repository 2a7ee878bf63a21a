set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ent_time_ab.sh la lb && bash tools/gpu_pmc_ent.sh
