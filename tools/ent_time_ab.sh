# Entropy encode/decode timing only (phase-ablation builds produce wrong
# streams on purpose): product and tools/variants/libjpegr_entropy_<v>.so
set -o pipefail
cd $GRAFT_REPO_ROOT
echo "== product: $(timeout -k 10 120 python3 tools/ent_scan.py 2>/dev/null)" || exit 1
for v in "$@"; do
  echo "== $v: $(LZ4JPEG_LIB=$PWD/tools/variants/libjpegr_entropy_$v.so timeout -k 10 120 python3 tools/ent_scan.py 2>/dev/null)" || exit 1
done
