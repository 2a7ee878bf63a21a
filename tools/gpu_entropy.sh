# GPU entropy stage: its tests + the other JPEG tests, then a short bench (no CPU leg)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_entropy.py tests/test_gpu_jpeg.py tests/test_gpu_reconstruct.py -x -q > gpurun_out/ent_t.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 3 --no-cpu-baseline > gpurun_out/ent_bench.json 2> gpurun_out/ent_bench.log
rc=$?
tail -15 gpurun_out/ent_t.log; grep -E "lz4|jpeg" gpurun_out/ent_bench.log
exit $rc
