# Effective shader clock under each hot kernel's own load (MI355X_MICROARCH.md
# "DVFS give-back": GRBM_GUI_ACTIVE / 8 XCDs / kernel wall time), from one
# rocprofv3 --pmc pass per workload.  -> gpurun_out/clock/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/clock
mkdir -p $D
timeout -k 10 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $D/lz4 -o run -- python3 tools/lz4_one.py 1073741824 3 > $D/lz4.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $D/jpeg -o run -- python3 tools/jpeg_one.py 10 16 > $D/jpeg.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $D/valu -o run -- tools/ab/valu_rate > $D/valu.log 2>&1 && \
python3 tools/clock_summary.py $D
