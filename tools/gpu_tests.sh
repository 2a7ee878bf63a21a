# GPU box: selected -m gpu test files (args), verbose, each test time-limited.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t2.log 2>&1
rc=$?
tail -15 gpurun_out/t2.log
exit $rc
