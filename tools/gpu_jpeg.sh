# JPEG encoder on the GPU box: time per image vs batch for the product build
# and the A/B variant tools/variants/libjpeg_<name>.so given as $1 (optional),
# and one PMC pass of the strip kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/jp
mkdir -p $O
timeout -k 10 400 python -m pytest tests/test_gpu_jpeg.py -x -q > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 1; }
tail -1 $O/t.log
echo "== product"; timeout -k 10 120 python3 tools/jpeg_scan.py 1 2 4 16 64 || exit 1
for v in "$@"; do
  L=$PWD/tools/variants/libjpeg_$v.so
  LZ4JPEG_LIB=$L timeout -k 10 400 python -m pytest tests/test_gpu_jpeg.py tests/test_gpu_configs.py -x -q -k "not rank7_shard" > $O/t_$v.log 2>&1 || { tail -20 $O/t_$v.log; exit 1; }
  echo "== $v: $(tail -1 $O/t_$v.log)"; LZ4JPEG_LIB=$L timeout -k 10 120 python3 tools/jpeg_scan.py 1 2 4 16 64 || exit 1
done
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"
timeout -k 10 200 rocprofv3 --kernel-trace --pmc $C -d $O/pmc -o run -- python3 tools/jpeg_one.py 3 > $O/pmc.log 2>&1 && \
python3 tools/pmc_summary.py $O/pmc/run_results.db jpeg_strip | tail -12
