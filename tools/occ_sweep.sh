cd $GRAFT_REPO_ROOT
for x in 0 1100 2200 3500 5400; do
  LZ4R_EXTRA_LDS=$x timeout -k 10 120 python3 tools/lz4_one.py 1073741824 3 > gpurun_out/occ_$x.log 2>&1 || exit 1
  echo "extra $x: $(tail -1 gpurun_out/occ_$x.log)"
done
