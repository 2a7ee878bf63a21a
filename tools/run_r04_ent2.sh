# round 4: entropy encode variants (tools/variants/libjpegr_entropy_<v>.so): tests + timing,
# then a timing-only repeat
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_ent.sh "$@" && bash tools/ent_time_ab.sh "$@"
