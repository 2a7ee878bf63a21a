# round 6: sequence-parallel decoder lz4_decode_seq -- parity of the variant
# library (decode, bare-stream decode, config and LZ4 tests), then A/B timing
set -o pipefail
O=gpurun_out/r06i
mkdir -p $O
A=$PWD/tools/ab
LZ4JPEG_LIB=$A/liblz4r_gpudec_seq.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_decode.py tests/test_gpu_bare_decode.py > $O/tests_seq.log 2>&1 || { echo SEQ TESTS FAILED; tail -40 $O/tests_seq.log; exit 1; }
tail -1 $O/tests_seq.log
timeout -k 10 300 python -u tools/ab_dec_inproc.py 30 prod $A/liblz4r_gpudec_seq.so prod $A/liblz4r_gpudec_seq.so > $O/ab.log 2>&1
