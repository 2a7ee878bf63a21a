# lz4_tiles phase ablations (tools/build_variants.sh builds liblz4_v<k>.so):
# 1 GiB timing of the product and of each variant, no parity (they are wrong
# on purpose).  usage: bash tools/lz4_ablate.sh 1 3 4 11
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ablate
mkdir -p $O
echo "== product: $(timeout -k 10 120 python3 tools/lz4_one.py 1073741824 8 2>&1 | tail -1)" || exit 1
for v in "$@"; do
  echo "== v$v: $(LZ4JPEG_LIB=$PWD/tools/variants/liblz4_v$v.so timeout -k 10 120 python3 tools/lz4_one.py 1073741824 8 2>&1 | tail -1)" || exit 1
done
