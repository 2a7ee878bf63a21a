# Round-5 check on one GPU box: every -m gpu test, the default bench line, a
# kernel-trace profile of the same bench command, the HBM traffic passes, the
# lz4_tiles roof inputs (tools/r05_roof.sh) and the held clocks.
#   -> gpurun_out/r05round/ (+ gpurun_out/traffic, r05roof, clock)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05round
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.log && \
python3 tools/prof_summary.py $O/prof > $O/kernels.md && \
bash tools/traffic.sh > $O/traffic.log 2>&1 && \
bash tools/r05_roof.sh > $O/roof.log 2>&1 && \
bash tools/clock_pmc.sh > $O/clock.json 2> $O/clock.log
rc=$?
tail -2 $O/tests.log; grep -E "^\[bench\]" $O/bench.err | tail -12; cat $O/kernels.md | head -30
exit $rc
