# GPU decoder + reconstruction check: decode tests, reconstruct tests, bench (no CPU leg)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_decode.py tests/test_gpu_reconstruct.py -x -q -m "gpu and not slow" > gpurun_out/dec_t.log 2>&1 && \
timeout -k 10 300 python -m pytest tests/test_gpu_decode.py -x -q -m "gpu and slow" > gpurun_out/dec_slow.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 5 --no-cpu-baseline > gpurun_out/dec_bench.json 2> gpurun_out/dec_bench.log
rc=$?
tail -3 gpurun_out/dec_t.log; tail -3 gpurun_out/dec_slow.log; grep -E "lz4|jpeg" gpurun_out/dec_bench.log
exit $rc
