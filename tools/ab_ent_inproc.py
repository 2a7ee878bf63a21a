"""In-process A/B timing of entropy-stage builds (tools only).

    python3 tools/ab_ent_inproc.py [rounds] prod|<lib.so> ...

A 4K random image's coefficients (the product DCT); every build (its own
ctypes handle, RTLD_LOCAL) encodes them with jpegr_entropy_encode_device,
round-robin after 100 ms of warm-up; per call torch events on the current
stream; then each build decodes its own encoding (jpegr_entropy_decode_device,
timed the same way).  Every build's bits / meta / table / status are compared
with the first build's, and every decode with the coefficients.

ENT_COEF=rand (default) | defer_y | defer_all: the coefficients.  defer_y
gives every luma stream 64 distinct values (a per-tile permutation of
-32..31: 65 distinct RLE symbols, past the 24 of the direct table), so every
luma stream of every wave is deferred to the hashed encoder (the
worst case of the deferred path); defer_all does the same to both chroma
streams (-16..15)."""
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
    d_coef = jpeg.encode_device(d_img, W, H)
    nt = jpeg.tiles(W, H)
    mode = os.environ.get("ENT_COEF", "rand")
    if mode != "rand":
        g = torch.Generator(device="cuda").manual_seed(7)
        c = d_coef.view(nt, 128)
        c[:, :64] = (torch.argsort(torch.rand(nt, 64, device="cuda", generator=g), dim=1) - 32).to(torch.int16)
        if mode == "defer_all":
            for lo in (64, 96):
                c[:, lo:lo + 32] = (torch.argsort(torch.rand(nt, 32, device="cuda", generator=g),
                                                  dim=1) - 16).to(torch.int16)
    print("coefficients:", mode, flush=True)
    sb = 0
    for lib in libs:
        lib.jpegr_entropy_scratch_bytes.restype = ctypes.c_size_t
        sb = max(sb, lib.jpegr_entropy_scratch_bytes(ctypes.c_size_t(nt)))
    outs = []
    for _ in libs:
        outs.append(dict(bits=torch.zeros(nt * 256, dtype=torch.uint8, device="cuda"),
                         meta=torch.zeros(nt * 3, dtype=torch.int32, device="cuda"),
                         table=torch.zeros(nt * 256, dtype=torch.int32, device="cuda"),
                         status=torch.zeros(4, dtype=torch.int32, device="cuda"),
                         scratch=torch.zeros(sb, dtype=torch.uint8, device="cuda"),
                         back=torch.zeros_like(d_coef)))
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = ctypes.c_void_p

    def enc(k):
        o = outs[k]
        rc = libs[k].jpegr_entropy_encode_device(P(d_coef.data_ptr()), ctypes.c_size_t(nt),
                                                 P(o["bits"].data_ptr()), P(o["meta"].data_ptr()),
                                                 P(o["table"].data_ptr()), P(o["scratch"].data_ptr()),
                                                 P(o["status"].data_ptr()), stream)
        assert rc == 0, (names[k], rc)

    def dec(k):
        o = outs[k]
        rc = libs[k].jpegr_entropy_decode_device(P(o["bits"].data_ptr()), P(o["meta"].data_ptr()),
                                                 P(o["table"].data_ptr()), ctypes.c_size_t(nt),
                                                 P(o["back"].data_ptr()), P(o["status"].data_ptr()),
                                                 stream)
        assert rc == 0, (names[k], rc)

    for k in range(len(libs)):
        enc(k)
    torch.cuda.synchronize()
    for k in range(len(libs)):
        dec(k)
    torch.cuda.synchronize()
    back_ok = [bool(torch.equal(o["back"], d_coef)) for o in outs]
    for k in range(len(libs)):
        enc(k)
    torch.cuda.synchronize()
    # status[2] is the decoder's call tag: it differs between builds
    same = [all(torch.equal(outs[k][f], outs[0][f]) for f in ("bits", "meta", "table")) and
            torch.equal(outs[k]["status"][:2], outs[0]["status"][:2]) for k in range(len(libs))]
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.1:
        for k in range(len(libs)):
            enc(k)
    torch.cuda.synchronize()
    times = [[] for _ in libs]
    dtimes = [[] for _ in libs]
    for _ in range(rounds):
        for k in range(len(libs)):
            e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            e0.record()
            enc(k)
            e1.record()
            dec(k)
            e2.record()
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1))
            dtimes[k].append(e1.elapsed_time(e2))
    for name, t, d, s, b in zip(names, times, dtimes, same, back_ok):
        print(f"{os.path.basename(name):28s} encode median {statistics.median(t):.4f} min {min(t):.4f} ms"
              f"  {'same' if s else 'DIFFERENT'}  decode median {statistics.median(d):.4f}"
              f" min {min(d):.4f} ms  {'ok' if b else 'DECODE MISMATCH'}", flush=True)


if __name__ == "__main__":
    main()
