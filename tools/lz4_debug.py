"""Debug helper: compress named inputs on the GPU, compare every block with
the oracle, print the first mismatches (block index, tile, bytes)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "lz4-jpeg_amd"), os.path.join(REPO, "tests")]
import golden_inputs  # noqa: E402
import oracle_api  # noqa: E402
import torch  # noqa: E402
from lz4jpeg.lz4 import Compressor  # noqa: E402

orc = oracle_api.load()
comp = Compressor()
names = sys.argv[1:] or ["file:Metamorphosis.txt", "metamorphosis_spaces", "text_10000"]
for name in names:
    data = golden_inputs.lz4_input(name)
    n = len(data)
    nb = (n + 299) // 300
    d_in = torch.from_numpy(np.frombuffer(data, dtype=np.uint8).copy()).cuda()
    d_out, length = comp.compress_device(d_in)
    torch.cuda.synchronize()
    got = d_out[:length].cpu().numpy().tobytes()
    ref = orc.lz4_compress(data)
    sizes = np.empty(nb, np.uint16)
    import ctypes
    from lz4jpeg import _lib
    _lib.lib().lz4r_copy_block_sizes(comp._h, sizes.ctypes.data_as(ctypes.c_void_p), nb, None)
    print(f"== {name}: n={n} nb={nb} len got={len(got)} ref={len(ref)} equal={got == ref}")
    off = 1
    bad = 0
    for b in range(nb):
        exp = orc.lz4_blocks(data, b, b + 1)
        g = got[off:off + int(sizes[b])]
        if int(sizes[b]) != len(exp) or g != exp:
            bad += 1
            if bad <= 3:
                print(f" block {b} tile {b // 16} k {b % 16}: size got {sizes[b]} exp {len(exp)}")
                print("  exp", exp[:64].hex())
                print("  got", g[:64].hex())
                d = next((i for i in range(min(len(g), len(exp))) if g[i] != exp[i]), None)
                print("  first diff at", d, "exp tail", exp[max(0, (d or 0) - 8):(d or 0) + 16].hex(),
                      "got tail", g[max(0, (d or 0) - 8):(d or 0) + 16].hex())
        off += int(sizes[b])
    print(f" bad blocks: {bad}")
comp.close()
