"""In-process A/B timing of LZ4 compressor builds (tools only).

    python3 tools/ab_inproc.py [rounds] prod|<lib.so> ...

Loads every build in one process (separate ctypes handles, RTLD_LOCAL), one
context each, and compresses the 1 GiB bench corpus round-robin: 40 warm-up
calls (past the clock ramp), then `rounds` rounds of one call per build, so
clock drift and box noise hit every build alike.  Prints, per build, the
median / min of the whole call and of lz4_tiles (the library's own events)
and checks every build's stream length against the first's."""
import ctypes
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "lz4-jpeg_amd")]
import torch  # noqa: E402
from lz4jpeg import synth  # noqa: E402

PROD = os.path.join(REPO, "lz4-jpeg_amd", "lz4jpeg", "liblz4jpeg.so")


class Build:
    def __init__(self, name, path):
        self.name = name
        self.lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
        self.h = ctypes.c_void_p()
        assert self.lib.lz4r_ctx_create(ctypes.byref(self.h)) == 0
        assert self.lib.lz4r_set_timing(self.h, 1) == 0
        self.calls, self.tiles, self.lens = [], [], set()

    def run(self, d_in, n, d_out, record):
        got = ctypes.c_size_t(0)
        rc = self.lib.lz4r_compress_device(self.h, ctypes.c_void_p(d_in.data_ptr()),
                                           ctypes.c_size_t(n), ctypes.c_void_p(d_out.data_ptr()),
                                           ctypes.c_size_t(d_out.numel()), ctypes.byref(got), None)
        assert rc == 0, (self.name, rc)
        if record:
            a, b = ctypes.c_float(0), ctypes.c_float(0)
            assert self.lib.lz4r_last_timing(self.h, ctypes.byref(a), ctypes.byref(b)) == 0
            self.calls.append(a.value)
            self.tiles.append(b.value)
            self.lens.add(got.value)


def main():
    rounds = int(sys.argv[1])
    builds = []
    for a in sys.argv[2:]:
        builds.append(Build("prod", PROD) if a == "prod" else
                      Build(os.path.basename(a), os.path.abspath(a)))
    n = 1 << 30
    d_in = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    synth.random_passages_device(d_in, n, length=30000, seed=1)
    d_out = torch.empty(n + n // 8 + (1 << 20), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    for i in range(40):
        builds[i % len(builds)].run(d_in, n, d_out, False)
    for _ in range(rounds):
        for b in builds:
            b.run(d_in, n, d_out, True)
    ref = builds[0].lens
    for b in builds:
        print(f"{b.name:24s} tiles median {statistics.median(b.tiles):.4f} min {min(b.tiles):.4f}"
              f"  call median {statistics.median(b.calls):.4f} min {min(b.calls):.4f}"
              f"  len {'ok' if b.lens == ref and len(ref) == 1 else b.lens}", flush=True)


if __name__ == "__main__":
    main()
