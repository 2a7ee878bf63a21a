# Round check on the GPU box: parity tests, bench line, kernel-trace profile,
# HBM traffic PMC passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t1.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/b1.json 2> gpurun_out/b1.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/p1.log 2>&1 && \
bash tools/traffic.sh > gpurun_out/traffic.log 2>&1 && \
bash tools/issue.sh > gpurun_out/issue.log 2>&1
rc=$?
tail -3 gpurun_out/t1.log; cat gpurun_out/b1.json
exit $rc
