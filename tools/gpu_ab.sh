# Product-build LZ4 parity, chunk-size timings, then A/B of variant libraries.
# usage: bash tools/gpu_ab.sh <variant names...>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_lz4.py tests/test_gpu_decode.py -x -q --timeout 120 --timeout-method thread -m "gpu and not slow" > gpurun_out/ab_t.log 2>&1 || { tail -30 gpurun_out/ab_t.log; exit 1; }
echo "product: $(tail -1 gpurun_out/ab_t.log)"
for cp in ${CHUNKS:-64}; do
  LZ4R_CHUNK_PARTS=$cp timeout -k 10 120 python3 tools/lz4_one.py 1073741824 4 > gpurun_out/ab_c$cp.log 2>&1 || exit 1
  echo "chunk_parts $cp: $(tail -1 gpurun_out/ab_c$cp.log)"
done
bash tools/gpu_var.sh "$@"
