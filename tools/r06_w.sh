# round 6: vector-memory pipe counters of lz4_decode_blocks (is the TA the bound?)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06w
mkdir -p $O
C="TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum TD_BUSY_avr GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES"
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C -d $O/pa -o run -- python3 tools/dec_one.py 1073741824 2 > $O/pa.log 2>&1
rc=$?
tail -5 $O/pa.log
python3 tools/pmc_summary.py $O/pa/run_results.db lz4_decode_blocks > $O/pa.txt 2>&1; tail -10 $O/pa.txt
exit $rc
