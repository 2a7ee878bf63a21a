# PMC instruction / wait mix of the entropy kernels (one 4K image, 3 reps).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pent
mkdir -p $O
C1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
C2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU"
timeout -k 10 120 rocprofv3 --kernel-trace --pmc $C1 -d $O/a -o run -- python3 tools/ent_one.py 3 > $O/a.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --pmc $C2 -d $O/b -o run -- python3 tools/ent_one.py 3 > $O/b.log 2>&1
rc=$?
for k in "entropy_encode_lane<true>" "entropy_encode_lane<false>" "entropy_decode_kernel<true>"; do
  echo "== $k"
  python3 tools/pmc_summary.py $O/a/run_results.db "$k" | tail -9
  python3 tools/pmc_summary.py $O/b/run_results.db "$k" | tail -7
done
exit $rc
