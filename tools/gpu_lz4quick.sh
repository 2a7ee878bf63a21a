# LZ4 compressor: GPU parity tests (not slow) + 1 GiB timing
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_lz4.py tests/test_gpu_decode.py -x -q -m "gpu and not slow" > gpurun_out/lq_t.log 2>&1 && \
timeout -k 10 120 python3 tools/lz4_one.py 1073741824 4 > gpurun_out/lq_time.log 2>&1
rc=$?
tail -2 gpurun_out/lq_t.log; cat gpurun_out/lq_time.log
exit $rc
