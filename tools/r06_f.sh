# round 6: lz4_emit 17x17 mask table A/B; JPEG encoder hoisted table loads A/B
set -o pipefail
O=gpurun_out/r06f
mkdir -p $O
timeout -k 10 300 python -u tools/ab_inproc.py 30 prod tools/ab/liblz4_mask2.so prod tools/ab/liblz4_mask2.so > $O/emit_mask2.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/ab_jpeg_inproc.py 40 prod tools/ab/libjpeg_hoist.so prod tools/ab/libjpeg_hoist.so > $O/jpeg_hoist.log 2>&1 || exit 1
