# round 6 check on the GPU box, in two calls:
#   bash tools/r06_round.sh tests   -> the -m gpu suite
#   bash tools/r06_round.sh bench   -> the default bench line, the rocprofv3
#        --kernel-trace --stats summary of the same command, HBM traffic passes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06round
mkdir -p $O
if [ "$1" = tests ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
  rc=$?; tail -3 $O/gpu_tests.log; exit $rc
fi
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.log && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py > $O/prof_bench.json 2> $O/prof_bench.log && \
python3 tools/prof_summary.py $O/prof > $O/kernels.md && \
bash tools/traffic.sh > $O/traffic.log 2>&1 && cp gpurun_out/traffic/traffic.json $O/traffic.json
rc=$?
grep -E "^\[bench\]" $O/bench.log | tail -14; head -30 $O/kernels.md
exit $rc
