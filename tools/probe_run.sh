# smoke() on the product build, then the lz4_tiles binding-resource probes:
# 1 GiB kernel-trace durations of the product and of tools/variants/
# liblz4_{40,41,42}.so (40: +16 LDS reads, 41: +16 VOP3 VALU, 42: +32 plain
# VALU per block), twice in alternating order.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/probe
mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for pass in 1 2; do
  for v in prod 40 41 42; do
    lib=""; [ $v = prod ] || lib=$PWD/tools/variants/liblz4_$v.so
    LZ4JPEG_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/p_${v}_$pass -o run -- python3 tools/lz4_one.py 1073741824 8 3 > $O/p_${v}_$pass.log 2>&1 || exit 1
    echo "== $v pass $pass: $(python3 tools/prof_summary.py $O/p_${v}_$pass | grep -E 'lz4_tiles<' | head -1)"
  done
done
