# lz4_emit A/B on the GPU box: the LZ4 parity tests (incl. full-size md5s,
# configs, decoder, compat) on the product build, then 1 GiB kernel-trace
# durations of the product and of each tools/variants/liblz4_<v>.so given as
# an argument (e.g. old = the previous product source, 31 / 32 = ablations).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/emit2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_lz4.py tests/test_gpu_configs.py tests/test_gpu_decode.py tests/test_gpu_bare_decode.py tests/test_gpu_compat.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1; rc=$?
tail -3 $O/t.log
[ $rc -eq 0 ] || { tail -60 $O/t.log; exit $rc; }
for v in prod "$@"; do
  lib=""; [ $v = prod ] || lib=$PWD/tools/variants/liblz4_$v.so
  LZ4JPEG_LIB=$lib timeout -k 10 120 python3 tools/lz4_one.py 1073741824 12 > $O/time_$v.log 2>&1 || exit 1
  echo "== $v: $(tail -1 $O/time_$v.log)"
  LZ4JPEG_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/p_$v -o run -- python3 tools/lz4_one.py 1073741824 8 3 > $O/p_$v.log 2>&1 || exit 1
  python3 tools/prof_summary.py $O/p_$v | grep -E 'lz4_(tiles|emit)' | head -4
done
