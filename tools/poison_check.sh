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
c.check()                           # the call cleared the status: a later check is clean
print("status cleared after the report")
PY
