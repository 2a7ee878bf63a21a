# lz4_emit per-phase ablation on the GPU box: kernel-trace durations on 1 GiB
# of the product build and of each tools/variants/liblz4_v<v>.so given as an
# argument (31 = no literal words, 32 = no header bytes; outputs are wrong,
# only the times count).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/emitab
mkdir -p $O
for v in prod "$@"; do
  lib=""; [ $v = prod ] || lib=$PWD/tools/variants/liblz4_v$v.so
  LZ4JPEG_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/p_$v -o run -- python3 tools/lz4_one.py 1073741824 8 3 > $O/p_$v.log 2>&1 || exit 1
  echo "== $v: $(tail -1 $O/p_$v.log)"
  python3 tools/prof_summary.py $O/p_$v | grep -E 'lz4_(tiles|emit)' | head -4
done
