# round 6: JPEG / entropy parity after the reconstruction and deferred-stream
# changes, then the deferred-path A/B (product vs the round-5 pass at b407805)
set -o pipefail
O=gpurun_out/r06e
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_entropy.py tests/test_gpu_reconstruct.py tests/test_gpu_jpeg.py tests/test_gpu_exe.py > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for m in rand defer_y defer_all; do ENT_COEF=$m timeout -k 10 200 python -u tools/ab_ent_inproc.py 20 prod tools/ab/libjpegr_entropy_olddefer.so > $O/ent_$m.log 2>&1 || exit 1; done
timeout -k 10 200 python -u tools/ab_recon_inproc.py 30 prod tools/ab/libjpeg_ro0.so > $O/recon_ab.log 2>&1
