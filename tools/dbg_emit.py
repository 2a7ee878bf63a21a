import os, sys, ctypes
sys.path[:0] = ["lz4-jpeg_amd", "tests"]
import numpy as np, torch
import golden_inputs
data = golden_inputs.lz4_input("file:lz4_input.txt")
ref = open("tests/golden/lz4_input.compressed.bin", "rb").read()
from lz4jpeg import lz4
c = lz4.Compressor()
d_in = torch.from_numpy(np.frombuffer(data, dtype=np.uint8).copy()).cuda()
d_out, n = c.compress_device(d_in)
got = d_out[:n].cpu().numpy().tobytes()
print("len", n, len(ref))
diff = [i for i in range(min(n, len(ref))) if got[i] != ref[i]]
print("first diffs", diff[:20])
print("ref", ref[:80].hex())
print("got", got[:80].hex())
if diff:
    i = diff[0]
    print("ref@", ref[max(0,i-8):i+24].hex())
    print("got@", got[max(0,i-8):i+24].hex())
