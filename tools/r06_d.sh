set -o pipefail
mkdir -p gpurun_out/r06d
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_overread.py tests/test_gpu_reconstruct.py > gpurun_out/r06d/tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r06d/tests.log; exit 1; }
timeout -k 10 200 python -u tools/ab_recon_inproc.py 30 prod tools/ab/libjpeg_ro0.so tools/ab/libjpeg_ro1.so tools/ab/libjpeg_ro3.so tools/ab/libjpeg_ro5.so > gpurun_out/r06d/recon_ab.log 2>&1 || exit 1
for m in rand defer_y defer_all; do ENT_COEF=$m timeout -k 10 200 python -u tools/ab_ent_inproc.py 40 prod tools/ab/libjpegr_entropy_olddefer.so > gpurun_out/r06d/ent_$m.log 2>&1 || exit 1; done
