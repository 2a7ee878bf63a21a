# round 6: entropy decode variants (tools/ab/libjpegr_entropy_<v>.so):
# variant parity (entropy + reconstruction tests), then in-process A/B
#   bash tools/r06_l.sh "<variants to test>" "<A/B libs>"
set -o pipefail
O=gpurun_out/r06l
mkdir -p $O
A=$PWD/tools/ab
for v in $1; do
  LZ4JPEG_LIB=$A/libjpegr_entropy_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_entropy.py tests/test_gpu_reconstruct.py > $O/tests_$v.log 2>&1 || { echo "$v TESTS FAILED"; tail -30 $O/tests_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/tests_$v.log)"
done
libs=""; for v in $2; do [ $v = prod ] && libs="$libs prod" || libs="$libs $A/libjpegr_entropy_$v.so"; done
timeout -k 10 200 python -u tools/ab_ent_inproc.py 40 $libs $libs > $O/ab.log 2>&1 && cat $O/ab.log && \
ENT_COEF=defer_all timeout -k 10 200 python -u tools/ab_ent_inproc.py 5 $libs > $O/ab_defer.log 2>&1 && cat $O/ab_defer.log
