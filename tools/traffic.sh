# HBM traffic per launch of the hot kernels, from rocprofv3 PMC counters:
# FETCH_SIZE and WRITE_SIZE in separate passes (MI355X_MICROARCH.md, HBM).
# Writes gpurun_out/traffic/{lz4,jpeg}_{fetch,write}/ and a JSON summary.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/traffic
mkdir -p $D
timeout -k 10 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $D/lz4_fetch -o run -- python3 tools/lz4_one.py 1073741824 3 > $D/lz4_fetch.log 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $D/lz4_write -o run -- python3 tools/lz4_one.py 1073741824 3 > $D/lz4_write.log 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $D/jpeg_fetch -o run -- python3 tools/jpeg_one.py 5 > $D/jpeg_fetch.log 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $D/jpeg_write -o run -- python3 tools/jpeg_one.py 5 > $D/jpeg_write.log 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $D/dec_fetch -o run -- python3 tools/dec_one.py 1073741824 3 > $D/dec_fetch.log 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $D/dec_write -o run -- python3 tools/dec_one.py 1073741824 3 > $D/dec_write.log 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $D/ent_fetch -o run -- python3 tools/ent_one.py 3 > $D/ent_fetch.log 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $D/ent_write -o run -- python3 tools/ent_one.py 3 > $D/ent_write.log 2>&1 && \
python3 tools/traffic_summary.py $D > $D/traffic.json && cat $D/traffic.json
