# PMC instruction mix of the luma entropy encoder for the product and each
# tools/variants/libjpegr_entropy_<v>.so (phase-cut builds), one 4K image.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pentab
mkdir -p $O
C1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES"
run() {
  LZ4JPEG_LIB=$2 timeout -k 10 120 rocprofv3 --kernel-trace --pmc $C1 -d $O/$1 -o run -- python3 tools/ent_one.py 2 > $O/$1.log 2>&1 || return 1
  echo "== $1"
  python3 tools/pmc_summary.py $O/$1/run_results.db "entropy_encode_lane<true>" | tail -10
}
run product $PWD/lz4-jpeg_amd/lz4jpeg/liblz4jpeg.so || exit 1
for v in "$@"; do run $v $PWD/tools/variants/libjpegr_entropy_$v.so || exit 1; done
