# Kernel-trace durations of the JPEG encoder at 1, 2 and 4 images per launch
# (GPU-side durations vs the event timing of tools/jpeg_scan.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/jtrace
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/p -o run -- python3 tools/jpeg_scan.py 1 2 4 > $O/scan.log 2>&1 && \
python3 tools/prof_summary.py $O/p > $O/kernels.md && cat $O/scan.log && head -12 $O/kernels.md && \
python3 tools/jpeg_trace_stats.py $O/p
