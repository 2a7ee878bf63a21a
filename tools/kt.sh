cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/kt -o run -- python3 tools/lz4_one.py 1073741824 3 > gpurun_out/kt.log 2>&1
python3 tools/prof_summary.py gpurun_out/kt/run_results.db
