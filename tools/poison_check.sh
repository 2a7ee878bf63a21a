# The corrupt-head error path of lz4_tiles: a tools build
# (LZ4R_VARIANT=20) plants one stale, forward-pointing bucket head in every
# block.  The walk must still end (chains strictly decrease) and the call must
# return LZ4R_ERR_CORRUPT, not hang.  Built here by tools/build_variants.sh 20.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/poison
LZ4JPEG_LIB=$PWD/tools/variants/liblz4_v20.so timeout -k 10 120 python3 - <<'PY' 2>&1 | tee gpurun_out/poison/poison.log
import os, sys, time
sys.path[:0] = [os.path.join(os.environ["GRAFT_REPO_ROOT"], "lz4-jpeg_amd")]
import torch
from lz4jpeg import lz4, synth
n = 1 << 28
d_in = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
synth.random_passages_device(d_in, n, length=30000, seed=1)
c = lz4.Compressor()
t = time.perf_counter()
try:
    c.compress_device(d_in, n)
    print("NO ERROR REPORTED")
    sys.exit(1)
except lz4.Lz4Error as e:
    print(f"poisoned head, 256 MiB: {e} after {time.perf_counter() - t:.3f} s")
    assert e.code == -6
# the async and sharded paths: the verdict rides in
# bit 63 of the length word, so the segment compressor raises before its
# segment can reach the gather
d_len = torch.zeros(1, dtype=torch.int64, device="cuda")
d_out = torch.empty(lz4.compress_bound(n), dtype=torch.uint8, device="cuda")
c.compress_async(d_in, n, d_out, d_len, segment=True, final_shard=True)
try:
    c.async_length(d_len)
    print("ASYNC: NO ERROR REPORTED")
    sys.exit(1)
except lz4.Lz4Error as e:
    print(f"async segment: {e} (length word {int(d_len.item()) & (2**63 - 1)} | bit 63)")
    assert e.code == -6
try:
    c.check()
    print("CHECK: NO ERROR REPORTED")
    sys.exit(1)
except lz4.Lz4Error as e:
    print(f"lz4r_check after the async call: {e}")
    assert e.code == -6
import torch.distributed as dist
from lz4jpeg import dist as ldist
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29533")
dist.init_process_group("gloo", rank=0, world_size=1)
try:
    ldist.compress_sharded(d_in[:n], n, ldist.hip_segment_compressor(c, final_shard=True))
    print("SHARDED: NO ERROR REPORTED")
    sys.exit(1)
except lz4.Lz4Error as e:
    print(f"compress_sharded (hip_segment_compressor): {e}")
    assert e.code == -6
dist.destroy_process_group()
print("every path reports the poisoned index")
PY
