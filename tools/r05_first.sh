# Round 5, first box: the new tests (RCCL at world size 1, allocation-end
# inputs, lz4r_check's own verdict), the whole -m gpu suite, the gfx950
# counter list, and the default bench line.  -> gpurun_out/r05a/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05a
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_lz4.py -m gpu -x -v --timeout 300 --timeout-method thread -k "rccl or allocation_end or own_verdict" > $O/new_tests.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 ; \
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $O/bench.json 2> $O/bench.err
rc=$?
tail -5 $O/new_tests.log; tail -3 $O/tests.log; grep -E "^\[bench\]" $O/bench.err | tail -14
exit $rc
