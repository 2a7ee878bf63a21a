# JPEG encoder timing only (no parity: timing ablations such as noload /
# nostore compute wrong output on purpose): product and each
# tools/variants/libjpeg_<name>.so given as arguments, images per launch 1..64.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
echo "== product"; timeout -k 10 120 python3 tools/jpeg_scan.py 1 2 4 64 || exit 1
for v in "$@"; do
  echo "== $v"; LZ4JPEG_LIB=$PWD/tools/variants/libjpeg_$v.so timeout -k 10 120 python3 tools/jpeg_scan.py 1 2 4 64 || exit 1
done
