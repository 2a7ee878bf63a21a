set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/qc
timeout -k 10 700 python -u -m pytest tests/test_gpu_lz4.py tests/test_gpu_entropy.py tests/test_gpu_decode.py tests/test_gpu_bare_decode.py -x -q --timeout 300 --timeout-method thread > gpurun_out/qc/t.log 2>&1; rc=$?
tail -3 gpurun_out/qc/t.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/qc/t.log; exit $rc; }
timeout -k 10 120 python3 tools/lz4_one.py 1073741824 10 | tail -1 && \
timeout -k 10 120 python3 tools/dec_one.py | tail -2 && \
timeout -k 10 120 python3 tools/ent_scan.py
