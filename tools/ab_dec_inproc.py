"""In-process A/B timing of GPU LZ4 decoder builds (tools only).

    python3 tools/ab_dec_inproc.py [rounds] prod|<lib.so> ...

The product library compresses the 1 GiB bench corpus once; every build
(its own ctypes handle, RTLD_LOCAL) then decodes it with the compressor's
device-resident block offsets (lz4r_decompress_device; DEC_MODE=bare: the
stream alone, lz4r_decompress_stream_device), round-robin after 30 warm-up
calls.  Kernel time from torch events on the current stream;
every build's output is compared with the input once."""
import ctypes
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "lz4-jpeg_amd")]
import torch  # noqa: E402
from lz4jpeg import lz4, synth  # noqa: E402

PROD = os.path.join(REPO, "lz4-jpeg_amd", "lz4jpeg", "liblz4jpeg.so")


def main():
    rounds = int(sys.argv[1])
    names = sys.argv[2:]
    libs = [ctypes.CDLL(PROD if a == "prod" else os.path.abspath(a), mode=ctypes.RTLD_LOCAL)
            for a in names]
    n = 1 << 30
    d_in = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    synth.random_passages_device(d_in, n, length=30000, seed=1)
    c = lz4.Compressor()
    d_stream, length = c.compress_device(d_in, n)
    nb = (n + 299) // 300
    d_offs, _ = c.block_offsets_device()
    d_out = torch.empty(n + 300, dtype=torch.uint8, device="cuda")
    d_res = torch.zeros(2, dtype=torch.int64, device="cuda")
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    bare = os.environ.get("DEC_MODE") == "bare"
    got = ctypes.c_size_t(0)

    def dec(lib):
        if bare:                  # the stream alone (lz4r_decompress_stream_device, synchronous)
            rc = lib.lz4r_decompress_stream_device(ctypes.c_void_p(d_stream.data_ptr()),
                                                   ctypes.c_size_t(length),
                                                   ctypes.c_void_p(d_out.data_ptr()),
                                                   ctypes.c_size_t(n + 300), ctypes.byref(got), stream)
            assert rc == 0 and got.value == n, (rc, got.value)
            d_res[0] = n
            return
        rc = lib.lz4r_decompress_device(ctypes.c_void_p(d_stream.data_ptr()), ctypes.c_size_t(length),
                                        ctypes.c_void_p(d_offs), ctypes.c_size_t(nb),
                                        ctypes.c_void_p(d_out.data_ptr()), ctypes.c_size_t(n + 300),
                                        ctypes.c_void_p(d_res.data_ptr()), stream)
        assert rc == 0, rc

    ok = []
    for lib in libs:
        d_out.zero_()
        dec(lib)
        torch.cuda.synchronize()
        ok.append(bool(torch.equal(d_out[:n], d_in[:n])) and int(d_res[0].item()) == n)
    for i in range(30):
        dec(libs[i % len(libs)])
    times = [[] for _ in libs]
    for _ in range(rounds):
        for k, lib in enumerate(libs):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            dec(lib)
            e1.record()
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1))
    for name, t, o in zip(names, times, ok):
        print(f"{os.path.basename(name):24s} decode median {statistics.median(t):.4f} min {min(t):.4f} ms"
              f"  {'ok' if o else 'MISMATCH'}", flush=True)
    c.close()


if __name__ == "__main__":
    main()
