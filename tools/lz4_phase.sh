# lz4_tiles phase budget on the GPU box: per-phase cycles (LZ4R_PROF build)
# and PMC instruction counts of the product build and of the ablation
# variants given as arguments (tools/build_variants.sh builds them).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/phase
O=gpurun_out/phase
C1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH"
LZ4JPEG_LIB=$PWD/tools/variants/liblz4_p0.so timeout -k 10 120 python3 tools/lz4_prof.py 1073741824 3 > $O/prof.log 2>&1 || exit 1
cat $O/prof.log
run() {  # name lib
  LZ4JPEG_LIB=$2 timeout -k 10 120 python3 tools/lz4_one.py 1073741824 3 > $O/t_$1.log 2>&1 || return 1
  LZ4JPEG_LIB=$2 timeout -k 10 200 rocprofv3 --kernel-trace --pmc $C1 -d $O/p_$1 -o run -- python3 tools/lz4_one.py 268435456 1 > $O/p_$1.log 2>&1 || return 1
  echo "== $1 $(tail -1 $O/t_$1.log)"
  python3 tools/pmc_summary.py $O/p_$1/run_results.db lz4_tiles | grep -v _dur
}
run base $PWD/lz4-jpeg_amd/lz4jpeg/liblz4jpeg.so || exit 1
for v in "$@"; do run v$v $PWD/tools/variants/liblz4_v$v.so || exit 1; done
