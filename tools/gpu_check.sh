# GPU box: the -m gpu parity suite, then one default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t1.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/b1.json 2> gpurun_out/b1.err
rc=$?
tail -5 gpurun_out/t1.log; grep -E "^\[bench\]" gpurun_out/b1.err | tail -20
exit $rc
