set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 240 python tools/lz4_debug.py > gpurun_out/dbg.log 2>&1 && \
timeout -k 10 600 python -m pytest tests -m "gpu and not slow" -x -q > gpurun_out/t1.log 2>&1 && \
timeout -k 10 120 python3 tools/lz4_one.py 268435456 3 > gpurun_out/var_0.log 2>&1 && \
for v in 1; do LZ4JPEG_LIB=$PWD/tools/variants/liblz4_v$v.so timeout -k 10 120 python3 tools/lz4_one.py 268435456 3 > gpurun_out/var_$v.log 2>&1 || exit 1; done
rc=$?
[ $rc -eq 0 ] && timeout -k 10 120 python3 tools/lz4_prof.py liblz4_p0.so > gpurun_out/prof.log 2>&1
cat gpurun_out/prof.log
grep -E "==|bad" gpurun_out/dbg.log; tail -2 gpurun_out/t1.log
for v in 0 1; do echo "variant $v: $(tail -1 gpurun_out/var_$v.log)"; done

timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/kt -o run -- python3 tools/lz4_one.py 1073741824 3 > gpurun_out/kt.log 2>&1 && python3 tools/prof_summary.py gpurun_out/kt/run_results.db
