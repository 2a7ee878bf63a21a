# round 6: the -m gpu suite of the product, then the entropy fill-loop A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06round
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log
[ $rc = 0 ] || exit $rc
timeout -k 10 200 python -u tools/ab_ent_inproc.py 40 prod tools/ab/libjpegr_entropy_fill.so prod tools/ab/libjpegr_entropy_fill.so > $O/ent_fill_ab.log 2>&1
