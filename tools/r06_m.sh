# round 6: PMC of the entropy decode kernels, product and the pair2 variant
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06m
mkdir -p $O
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"
B="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES"
for v in prod pair2; do
  L=""; [ $v = prod ] || L=$PWD/tools/ab/libjpegr_entropy_$v.so
  LZ4JPEG_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $A -d $O/${v}_a -o run -- python3 tools/ent_one.py 3 > $O/${v}_a.log 2>&1 && \
  LZ4JPEG_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $B -d $O/${v}_b -o run -- python3 tools/ent_one.py 3 > $O/${v}_b.log 2>&1 || exit 1
  for p in a b; do python3 tools/pmc_summary.py $O/${v}_$p/run_results.db entropy_decode > $O/${v}_$p.txt 2>&1; done
done
