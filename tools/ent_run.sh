set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ent
timeout -k 10 300 python -u -m pytest tests/test_gpu_entropy.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ent/t.log 2>&1; rc=$?
tail -15 gpurun_out/ent/t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 tools/ent_scan.py
