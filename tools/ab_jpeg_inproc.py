"""In-process A/B timing of JPEG encoder builds (tools only).

    python3 tools/ab_jpeg_inproc.py [rounds] prod|<lib.so> ...

A 4K random image; every build (its own
ctypes handle, RTLD_LOCAL) encodes it with jpegr_encode_device (one image per launch),
round-robin after 100 ms of warm-up, 20 launches per timed batch (torch
events on the current stream); every build's coefficients are compared with the
first build's."""
import ctypes
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "lz4-jpeg_amd")]
import torch  # noqa: E402
from lz4jpeg import jpeg, synth  # noqa: E402

PROD = os.path.join(REPO, "lz4-jpeg_amd", "lz4jpeg", "liblz4jpeg.so")


def main():
    rounds = int(sys.argv[1])
    names = sys.argv[2:]
    libs = [ctypes.CDLL(PROD if a == "prod" else os.path.abspath(a), mode=ctypes.RTLD_LOCAL)
            for a in names]
    W, H = 3840, 2160
    d_img = torch.from_numpy(synth.rand_rgba(W, H, seed=1)).cuda()
    outs = [torch.zeros(jpeg.coef_count(W, H), dtype=torch.int16, device="cuda") for _ in libs]
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = ctypes.c_void_p

    def rec(k):
        rc = libs[k].jpegr_encode_device(P(d_img.data_ptr()), W, H, 1, P(outs[k].data_ptr()),
                                         stream)
        assert rc == 0, (names[k], rc)

    for k in range(len(libs)):
        rec(k)
    torch.cuda.synchronize()
    same = [bool(torch.equal(o, outs[0])) for o in outs]
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.1:
        for k in range(len(libs)):
            rec(k)
    torch.cuda.synchronize()
    times = [[] for _ in libs]
    for _ in range(rounds):
        for k in range(len(libs)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                rec(k)
            e1.record()
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) / 20)
    for name, t, s in zip(names, times, same):
        m = statistics.median(t)
        print(f"{os.path.basename(name):28s} encode median {m * 1e3:.2f} us min "
              f"{min(t) * 1e3:.2f} us  {W * H / m / 1e6:.1f} Gpix/s  {'same' if s else 'DIFFERENT'}",
              flush=True)


if __name__ == "__main__":
    main()
