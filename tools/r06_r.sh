# round 6: LZ4 block decoder variants (tools/ab/liblz4r_gpudec_<v>.so):
# decode + bare-stream parity, then in-process A/B
#   bash tools/r06_r.sh "<variants to test>" "<A/B libs>"
set -o pipefail
O=gpurun_out/r06r
mkdir -p $O
A=$PWD/tools/ab
for v in $1; do
  LZ4JPEG_LIB=$A/liblz4r_gpudec_$v.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_decode.py tests/test_gpu_bare_decode.py > $O/tests_$v.log 2>&1 || { echo "$v TESTS FAILED"; tail -30 $O/tests_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/tests_$v.log)"
done
libs=""; for v in $2; do [ $v = prod ] && libs="$libs prod" || libs="$libs $A/liblz4r_gpudec_$v.so"; done
timeout -k 10 300 python -u tools/ab_dec_inproc.py 20 $libs $libs > $O/ab.log 2>&1; rc=$?; tail -12 $O/ab.log
[ $rc = 0 ] || exit $rc
[ -n "$3" ] || exit 0
libs=""; for v in $3; do [ $v = prod ] && libs="$libs prod" || libs="$libs $A/liblz4r_gpudec_$v.so"; done
DEC_MODE=bare timeout -k 10 300 python -u tools/ab_dec_inproc.py 10 $libs $libs > $O/ab_bare.log 2>&1; rc=$?; tail -8 $O/ab_bare.log; exit $rc
