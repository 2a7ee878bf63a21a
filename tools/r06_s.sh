set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/o1prof
mkdir -p $O
LZ4JPEG_LIB=$PWD/tools/ab/liblz4r_gpudec_o1.so timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $O/p -o run -- python3 tools/dec_one.py 1073741824 5 > $O/run.log 2>&1 || { tail -5 $O/run.log; exit 1; }
python3 tools/prof_summary.py $O/p | head -12
python3 tools/trace_gaps.py $(ls $O/p/*/run_results.db $O/p/run_results.db 2>/dev/null | head -1) 8
