# Entropy stage A/B on the GPU box: product vs tools/variants/libjpegr_entropy_<v>.so
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ent
mkdir -p $O
echo "== product: $(timeout -k 10 120 python3 tools/ent_scan.py 2>/dev/null)" || exit 1
for v in "$@"; do
  L=$PWD/tools/variants/libjpegr_entropy_$v.so
  LZ4JPEG_LIB=$L timeout -k 10 400 python -m pytest tests/test_gpu_entropy.py -x -q > $O/t_$v.log 2>&1 || { tail -20 $O/t_$v.log; exit 1; }
  echo "== $v: $(tail -1 $O/t_$v.log) | $(LZ4JPEG_LIB=$L timeout -k 10 120 python3 tools/ent_scan.py 2>/dev/null)" || exit 1
done
