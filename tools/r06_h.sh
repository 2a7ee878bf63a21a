# round 6: persistent prefetching lz4_emit_p -- parity of the variant library
# (LZ4 GPU tests incl. the full-size md5s), then in-process A/B timing
set -o pipefail
O=gpurun_out/r06h
mkdir -p $O
A=$PWD/tools/ab
LZ4JPEG_LIB=$A/liblz4_P28.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lz4.py tests/test_gpu_decode.py tests/test_gpu_overread.py > $O/tests_P28.log 2>&1 || { echo P28 TESTS FAILED; tail -30 $O/tests_P28.log; exit 1; }
tail -1 $O/tests_P28.log
timeout -k 10 400 python -u tools/ab_inproc.py 30 prod $A/liblz4_P28.so $A/liblz4_P24.so $A/liblz4_N28.so prod $A/liblz4_P28.so > $O/ab.log 2>&1
# the block decoder's LDS behaviour (misaligned slot accesses?)
export TMPDIR=/tmp
D=gpurun_out/r06h/decpmc
mkdir -p $D
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_UNALIGNED_STALL SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $D/pc -o run -- python3 tools/dec_one.py 1073741824 3 > $D/pc.log 2>&1 && python3 tools/pmc_summary.py $D/pc/run_results.db lz4_decode_blocks > $D/pc.txt 2>&1
