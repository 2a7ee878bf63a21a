# LZ4 compressor A/B on the GPU box: parity tests (not slow), 1 GiB timing of
# the product build and of tools/variants/liblz4_base.so (if present), and
# their PMC instruction counts per block (256 MiB).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/lq
mkdir -p $O
C1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH"
timeout -k 10 400 python -m pytest tests/test_gpu_lz4.py tests/test_gpu_decode.py -x -q -m "gpu and not slow" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
run() {  # name lib
  LZ4JPEG_LIB=$2 timeout -k 10 120 python3 tools/lz4_one.py 1073741824 12 > $O/time_$1.log 2>&1 || return 1
  LZ4JPEG_LIB=$2 timeout -k 10 200 rocprofv3 --kernel-trace --pmc $C1 -d $O/p_$1 -o run -- python3 tools/lz4_one.py 268435456 1 1 > $O/p_$1.log 2>&1 || return 1
  echo "== $1: $(tail -1 $O/time_$1.log)"
  python3 tools/pmc_summary.py $O/p_$1/run_results.db lz4_tiles | python3 -c "
import sys
v = {}
for line in sys.stdin:
    p = line.split()
    if len(p) == 2 and p[0].startswith('SQ_'): v[p[0]] = float(p[1])
w = v.get('SQ_WAVES', 1)
print('   per block: ' + ', '.join(f'{k[8:]} {v[k] / w:.1f}' for k in sorted(v) if k != 'SQ_WAVES'))"
}
run new $PWD/lz4-jpeg_amd/lz4jpeg/liblz4jpeg.so || exit 1
if [ -f tools/variants/liblz4_base.so ]; then run base $PWD/tools/variants/liblz4_base.so || exit 1; fi
