# round 6: bare-stream candidate-search variants: parity (decode + bare tests),
# then kernel times under rocprofv3 (product and each variant)
#   bash tools/r06_v.sh "<variants>"
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06v
mkdir -p $O
A=$PWD/tools/ab
for v in $1; do
  LZ4JPEG_LIB=$A/liblz4r_gpudec_$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_decode.py tests/test_gpu_bare_decode.py > $O/tests_$v.log 2>&1 || { echo "$v TESTS FAILED"; tail -30 $O/tests_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/tests_$v.log)"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prod -o run -- python3 tools/dec_one.py 1073741824 5 > $O/prod.log 2>&1 || exit 1
for v in $1; do
  LZ4JPEG_LIB=$A/liblz4r_gpudec_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/$v -o run -- python3 tools/dec_one.py 1073741824 5 > $O/$v.log 2>&1 || exit 1
done
for v in prod $1; do echo "== $v"; python3 tools/prof_summary.py $O/$v | grep -E "bare|decode_blocks"; done
