#!/usr/bin/env python3
"""Headline benchmark (BASELINE.json): LZ4 compress GB/s + JPEG DCT Gpixel/s
on 1..8 MI355X, with % of the HBM roofline and the CPU path timed beside it.

    python bench.py [--gpus N --steps K --warmup W]
    (N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N)

One JSON line on rank 0.  Top level = LZ4 (BASELINE.json configs[1]: 1 GiB of
random_extract-style text per GPU, weak scaling: every rank compresses its own
1 GiB shard of a global corpus, block-aligned); "jpeg" = configs[2] (one
3840x2160 random RGB image per GPU per step).  A step is one pass of the hot
path over one rank's batch with inputs resident in HBM; for N>1 it includes
the all_gather of segment lengths (every rank learns its offset in the global
stream).  The gatherv of all segments to rank 0 over RCCL is timed separately
("lz4_gather_ms") because it moves output, not compute.
"""
import argparse
import ctypes
import json
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(REPO, "lz4-jpeg_amd"), os.path.join(REPO, "tests")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
# per-launch HBM bytes from rocprofv3 FETCH_SIZE / WRITE_SIZE passes
# (tools/traffic.sh -> tools/traffic_summary.py, gfx950 FETCH correction applied)
TRAFFIC_JSON = os.path.join(REPO, "profiles", "r01_traffic.json")
# per-launch instruction counts of lz4_tiles + measured SIMD issue rates
# (tools/issue.sh -> tools/issue_summary.py)
ISSUE_JSON = os.path.join(REPO, "profiles", "r01_issue.json")


def issue_roof(bytes_now, launch_ms):
    """The compressor's binding roof: wave-instruction issue.  Counts per
    launch from PMC (scaled to this input), rates from the micro-benchmark."""
    try:
        d = json.load(open(ISSUE_JSON))
        pl, rates = d["lz4"]["per_launch"], d["issue_rates_winstr_per_s"]
        scale = bytes_now / d["lz4"]["bytes_per_launch"]
        valu = pl["SQ_INSTS_VALU"] * scale
        salu = pl["SQ_INSTS_SALU"] * scale
        peak_mix = rates["4 valu + 4 salu"]
        peak_valu = rates["v_add/xor/and/or"]
    except (OSError, KeyError, ValueError, ZeroDivisionError):
        return None
    sec = launch_ms / 1e3
    return {
        "bound": "issue (VALU + SALU wave-instructions)", "unit": "Gwinstr/s",
        "achieved": round((valu + salu) / sec / 1e9, 1), "peak": round(peak_mix / 1e9, 1),
        "frac": round((valu + salu) / sec / peak_mix, 4),
        "valu_frac": round(valu / sec / peak_valu, 4),
        "per_block": {"valu": round(pl["SQ_INSTS_VALU"] / pl["SQ_WAVES"], 1),
                      "salu": round(pl["SQ_INSTS_SALU"] / pl["SQ_WAVES"], 1),
                      "lds": round(pl["SQ_INSTS_LDS"] / pl["SQ_WAVES"], 1),
                      "branch": round(pl["SQ_INSTS_BRANCH"] / pl["SQ_WAVES"], 1)},
        "note": "achieved = PMC SQ_INSTS_VALU + SQ_INSTS_SALU per launch (profiles/r01_issue.json, "
                "scaled to this input) / lz4_tiles time; peak = the chip's measured rate for an "
                "interleaved 4 VALU + 4 SALU stream at 8 waves per SIMD (tools/valu_rate.hip); "
                "valu_frac = VALU alone against the measured v_add rate",
    }


def measured_traffic(kind, bytes_now, bytes_profiled):
    """HBM bytes per launch of the profiled kernel, scaled to this launch's
    input size (the profile ran the same configuration), or None."""
    try:
        t = json.load(open(TRAFFIC_JSON))[kind]
    except (OSError, KeyError, ValueError):
        return None
    return int(round(t["traffic_bytes"] * bytes_now / bytes_profiled))
FP64_VALU_PEAK_TOPS = 39.3     # 78.6 TFLOPS fp64 vector spec counts FMA as 2


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--lz4-bytes-per-rank", type=int, default=1 << 30)
    ap.add_argument("--jpeg-w", type=int, default=3840)
    ap.add_argument("--jpeg-h", type=int, default=2160)
    ap.add_argument("--jpeg-images-per-rank", type=int, default=1)
    ap.add_argument("--jpeg-steps", type=int, default=0, help="default: max(50, 10*steps)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-jpeg", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="target wall time of each CPU-baseline sample")
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist
    from lz4jpeg import dist as ldist
    from lz4jpeg import jpeg, lz4, synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    def barrier():
        if world > 1:
            dist.barrier()

    def max_over_ranks(x):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    # ------------------------------------------------------------------ LZ4
    n_total = args.lz4_bytes_per_rank * world
    lo, hi = ldist.shard_bytes(n_total, world, rank)
    log(f"rank {rank}: synthesising LZ4 shard [{lo}, {hi}) of {n_total} B")
    host = synth.random_passages(hi - lo, length=30000, seed=1, first=lo)
    d_in = torch.from_numpy(host).to(dev)
    n = hi - lo
    comp = lz4.Compressor()
    cap = lz4.compress_bound(n)
    d_out = torch.empty(cap, dtype=torch.uint8, device=dev)
    d_len = torch.zeros(1, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream()

    def lz4_step():
        if world == 1:
            _, got = comp.compress_device(d_in, n, d_out)
            return got
        comp.compress_async(d_in, n, d_out, d_len, segment=True)
        seg = int(d_len.item())
        ldist.exchange_lengths(seg, dev)
        return seg

    for _ in range(args.warmup):
        out_len = lz4_step()
    torch.cuda.synchronize()
    barrier()
    comp.set_timing(True)
    match_ms, call_ms = [], []
    torch.cuda.synchronize()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out_len = lz4_step()
        c_ms, m_ms = comp.last_timing()
        call_ms.append(c_ms)
        match_ms.append(m_ms)
    torch.cuda.synchronize()
    barrier()
    dt = max_over_ranks(time.perf_counter() - t0)
    comp.set_timing(False)
    lz4_ms = dt / args.steps * 1e3
    lz4_gbs = n_total / (dt / args.steps) / 1e9
    avg_match_ms = sum(match_ms) / len(match_ms)
    avg_call_ms = sum(call_ms) / len(call_ms)
    log(f"lz4: {lz4_ms:.3f} ms/step, {lz4_gbs:.1f} GB/s aggregate, analyze kernel "
        f"{avg_match_ms:.3f} ms, call {avg_call_ms:.3f} ms, out {out_len} B")

    gather_ms = None
    if world > 1:
        seg = lz4_step()
        lens, offs = ldist.exchange_lengths(seg, dev)
        torch.cuda.synchronize()
        barrier()
        g0 = time.perf_counter()
        ldist.gather_stream(d_out, seg, ldist.nblocks(n_total), lens, offs, dst=0)
        torch.cuda.synchronize()
        barrier()
        gather_ms = max_over_ranks(time.perf_counter() - g0) * 1e3

    # decoder: this rank's framed stream -> bytes, in HBM
    _, flen = comp.compress_device(d_in, n, d_out)
    nb_local = ldist.nblocks(n)
    d_boff = torch.from_numpy(comp.block_offsets(nb_local).astype(np.int64)).to(dev)
    d_dec = torch.empty(n + 300, dtype=torch.uint8, device=dev)
    _, got = lz4.decompress_device(d_out, flen, d_boff, nb_local, n + 300, d_out=d_dec)
    dec_ok = got == n and bool(torch.equal(d_dec[:n], d_in))
    torch.cuda.synchronize()
    barrier()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(args.steps):
        lz4.decompress_device(d_out, flen, d_boff, nb_local, n + 300, d_out=d_dec,
                              check=False)
    e1.record(stream)
    torch.cuda.synchronize()
    barrier()
    ddt = max_over_ranks(time.perf_counter() - t0)
    dec_kern_ms = e0.elapsed_time(e1) / args.steps
    lz4_dec = {
        "metric": "LZ4 block-parallel decode GB/s (decoded bytes, stream resident in HBM)",
        "value": round(n_total / (ddt / args.steps) / 1e9, 3), "unit": "GB/s",
        "kernel": "lz4_decode_blocks", "avg_launch_ms": round(dec_kern_ms, 4),
        "roundtrip_ok": dec_ok,
        "roofline": {
            "bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS,
            "achieved": round((n + flen) / (dec_kern_ms / 1e3) / 1e9, 2),
            "frac": round((n + flen) / (dec_kern_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
            "note": "algorithmic bytes = compressed bytes read + decoded bytes written"},
    }
    del d_dec
    log(f"lz4 decode: {dec_kern_ms:.3f} ms/launch, {lz4_dec['value']} GB/s, ok={dec_ok}")

    roof_lz4 = {
        "bound": "hbm", "kernel": "lz4_tiles",
        "achieved": round(n / (avg_match_ms / 1e3) / 1e9, 2), "peak": HBM_PEAK_GBS,
        "unit": "GB/s", "frac": round(n / (avg_match_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
        "traffic": measured_traffic("lz4", n, 1 << 30),
        "binding_roof": issue_roof(n, avg_match_ms),
        "algorithmic_bytes_per_launch": n,
        "avg_launch_ms": round(avg_match_ms, 4),
        "whole_call_ms": round(avg_call_ms, 4),
        "note": "algorithmic bytes = 1 B read per input byte (SURVEY §8d: the HBM-read "
                "roofline); achieved = that / lz4_tiles time from HIP events on its launch "
                "stream in each timed step; traffic = FETCH_SIZE(x2, gfx950) + WRITE_SIZE "
                "per launch from profiles/r01_traffic.json; the kernel is issue-bound "
                "(DESIGN.md), not HBM-bound",
    }

    # ----------------------------------------------------------------- JPEG
    jres = None
    if not args.no_jpeg:
        W, H, B = args.jpeg_w, args.jpeg_h, args.jpeg_images_per_rank
        img = synth.rand_rgba(W, H, seed=1 + rank)
        d_img = torch.from_numpy(np.ascontiguousarray(np.broadcast_to(img, (B,) + img.shape))).to(dev)
        d_coef = torch.empty(B * jpeg.coef_count(W, H), dtype=torch.int16, device=dev)
        jsteps = args.jpeg_steps or max(50, 10 * args.steps)
        for _ in range(max(args.warmup, 3)):
            jpeg.encode_device(d_img, W, H, B, d_coef)
        torch.cuda.synchronize()
        barrier()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record(stream)
        for _ in range(jsteps):
            jpeg.encode_device(d_img, W, H, B, d_coef)
        ev1.record(stream)
        torch.cuda.synchronize()
        barrier()
        jdt = max_over_ranks(time.perf_counter() - t0)
        kern_ms = ev0.elapsed_time(ev1) / jsteps
        px_total = W * H * B * world
        gpix = px_total / (jdt / jsteps) / 1e9
        px_rank = W * H * B
        tiles = ((W + 7) // 8) * ((H + 7) // 8) * B
        jres = {
            "metric": "JPEG DCT+quant+zigzag Gpixel/s (bit-exact int16 coefficients)",
            "value": round(gpix, 3), "unit": "Gpixel/s", "n_gpus": world, "steps": jsteps,
            "ms_per_step": round(jdt / jsteps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "dtype": "f64",
            "data": "synthetic: glibc rand() RGBA noise (random_image.c), seed 1+rank",
            "config": {"workload": "jpeg_encode_3840x2160_rgb", "w": W, "h": H,
                       "images_per_rank": B, "parallelism": f"images{world}"},
            "roofline": {
                "bound": "hbm", "kernel": "jpeg_strip_kernel",
                "achieved": round(8 * px_rank / (kern_ms / 1e3) / 1e9, 2), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(8 * px_rank / (kern_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                "traffic": measured_traffic("jpeg", px_rank, 3840 * 2160),
                "algorithmic_bytes_per_launch": 8 * px_rank,
                "avg_launch_ms": round(kern_ms, 4),
                "binding_roof": {
                    "bound": "valu_fp64", "unit": "Tops/s",
                    "achieved": round(tiles * 13312 / (kern_ms / 1e3) / 1e12, 2),
                    "peak": FP64_VALU_PEAK_TOPS,
                    "frac": round(tiles * 13312 / (kern_ms / 1e3) / 1e12 / FP64_VALU_PEAK_TOPS, 4),
                    "note": "13312 non-fused fp64 mul/add per tile in reference order "
                            "(8704 luma + 2x2304 chroma); peak = 78.6 TF fp64 vector spec / 2",
                },
                "note": "8 B/pixel algorithmic (4 B RGBA read + 4 B int16 written); traffic "
                        "from profiles/r01_traffic.json (PMC FETCH_SIZE x2 + WRITE_SIZE)",
            },
        }
        log(f"jpeg: {jres['ms_per_step']} ms/step, {gpix:.2f} Gpix/s aggregate, kernel {kern_ms:.4f} ms")

        # reconstruction: coefficients -> reconstructed RGBA
        d_rec_out = jpeg.reconstruct_device(d_coef, W, H, B, d_orig=d_img)
        torch.cuda.synchronize()
        r0, r1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        r0.record(stream)
        for _ in range(jsteps):
            jpeg.reconstruct_device(d_coef, W, H, B, d_orig=d_img)
        r1.record(stream)
        torch.cuda.synchronize()
        rec_ms = r0.elapsed_time(r1) / jsteps
        del d_rec_out
        jres["reconstruct"] = {
            "metric": "JPEG reconstruction (dequant + fp64 IDCT + YCbCr->RGB) Gpixel/s",
            "value": round(px_rank / (rec_ms / 1e3) / 1e9, 3), "unit": "Gpixel/s",
            "kernel": "jpeg_recon_kernel", "avg_launch_ms": round(rec_ms, 4),
            "roofline": {
                "bound": "valu_fp64", "unit": "Tops/s", "peak": FP64_VALU_PEAK_TOPS,
                "achieved": round(tiles * 13568 / (rec_ms / 1e3) / 1e12, 2),
                "frac": round(tiles * 13568 / (rec_ms / 1e3) / 1e12 / FP64_VALU_PEAK_TOPS, 4),
                "hbm_gbs": round(8 * px_rank / (rec_ms / 1e3) / 1e9, 2),
                "note": "13568 non-fused fp64 mul/add per tile (dequant x alpha 2x128, luma 8x(64 + 1024), "
                        "chroma 2x8x(32 + 256)); 8 B/px algorithmic HBM "
                        "(4 B int16 read + 4 B RGBA written)"},
        }
        log(f"jpeg reconstruct: {rec_ms:.4f} ms, {jres['reconstruct']['value']} Gpix/s")

        # entropy stage: RLE + per-stream Huffman + bits, and back
        ntl = jpeg.tiles(W, H) * B
        ent = jpeg.Entropy(ntl, device=dev)
        ent.encode(d_coef)
        d_back = torch.empty_like(d_coef)
        ent.decode(d_back)
        torch.cuda.synchronize()
        ent_ok = bool(torch.equal(d_back, d_coef)) and int(ent.status[0].item()) == 0 \
            and int(ent.status[1].item()) == 0
        meta = ent.meta.to(torch.int64) & 0xFFFFFFFF
        sum_bits = int((meta & 0xFFFF).sum().item())
        sum_codes = int((meta >> 24).sum().item())
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record(stream)
        for _ in range(jsteps):
            ent.encode(d_coef)
        e1.record(stream)
        for _ in range(jsteps):
            ent.decode(d_back)
        e2.record(stream)
        torch.cuda.synchronize()
        enc_ms, dec_ms = e0.elapsed_time(e1) / jsteps, e1.elapsed_time(e2) / jsteps
        # algorithmic bytes: coefficients (256 B/tile) + bits + table + meta
        ebytes = 256 * ntl + sum_bits // 8 + 4 * sum_codes + 12 * ntl
        jres["entropy"] = {
            "metric": "JPEG entropy stage (RLE + per-block Huffman, JPEG.c:767-1097) Gpixel/s",
            "value": round(px_rank / (enc_ms / 1e3) / 1e9, 3), "unit": "Gpixel/s",
            "encode_ms": round(enc_ms, 4), "decode_ms": round(dec_ms, 4),
            "decode_gpix_s": round(px_rank / (dec_ms / 1e3) / 1e9, 3),
            "kernels": ["entropy_encode_fast", "entropy_encode_deferred", "entropy_decode_kernel"],
            "bits_per_pixel": round(sum_bits / px_rank, 4), "roundtrip_ok": ent_ok,
            "roofline": {"bound": "issue (serial per-stream integer work)", "unit": "GB/s",
                         "hbm_achieved": round(ebytes / (enc_ms / 1e3) / 1e9, 2),
                         "peak": HBM_PEAK_GBS,
                         "frac": round(ebytes / (enc_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                         "note": "one lane per (tile, channel) stream; algorithmic bytes = "
                                 "256 B coefficients + bits + code table + meta per tile"},
        }
        del ent, d_back
        log(f"jpeg entropy: encode {enc_ms:.4f} ms, decode {dec_ms:.4f} ms, "
            f"{jres['entropy']['value']} Gpix/s, {sum_bits / px_rank:.3f} bits/px, ok={ent_ok}")

    # --------------------------------------------------------- CPU baselines
    cpu_lz4 = cpu_jpeg = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu_lz4, cpu_jpeg = cpu_baselines(host, args, None if args.no_jpeg else img)

    if rank == 0:
        line = {
            "metric": "LZ4 compress GB/s + JPEG DCT Mpixel/s at 1/2/4/8 MI355X; % HBM roofline",
            "value": round(lz4_gbs, 3), "unit": "GB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(lz4_ms, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic: random_extract-style 30000-B passages of Metamorphosis.txt, "
                    "newlines->spaces, glibc rand seed 1; each rank synthesises its shard",
            "config": {"workload": "lz4_compress_1GiB_text_per_gpu", "bytes_per_rank": n,
                       "bytes_total": n_total, "block": 300, "parallelism": f"shard{world}",
                       "compressed_bytes_rank0": out_len},
            "roofline": roof_lz4,
            "cpu_baseline": cpu_lz4,
            "lz4_gather_ms": None if gather_ms is None else round(gather_ms, 3),
            "lz4_decode": lz4_dec,
            "jpeg": jres,
        }
        if jres is not None:
            jres["cpu_baseline"] = cpu_jpeg
        print(json.dumps(line), flush=True)
    comp.close()
    if world > 1:
        dist.destroy_process_group()


def cpu_baselines(text, args, img):
    """Reference-path CPU throughput on this host's cores (rank 0, N=1 only),
    on bounded samples of the same workloads."""
    import numpy as np
    import oracle_api
    threads = max(1, min(16, os.cpu_count() or 1))
    o = oracle_api.load()
    # LZ4: oracle port (the reference LZ4.c cannot be built: Windows <direct.h>)
    calib = 2 << 20
    scratch = np.empty((calib // 300 + 1) * o.L.lz4o_block_bound(), np.uint8)
    t = time.perf_counter()
    o.L.lz4o_encode_parallel(text.ctypes.data, calib, threads, scratch.ctypes.data)
    rate = calib / max(time.perf_counter() - t, 1e-6)
    sample = int(min(text.size, max(calib, rate * args.cpu_seconds)))
    sample -= sample % 300
    scratch = np.empty((sample // 300 + 1) * o.L.lz4o_block_bound(), np.uint8)
    t = time.perf_counter()
    o.L.lz4o_encode_parallel(text.ctypes.data, sample, threads, scratch.ctypes.data)
    dt = time.perf_counter() - t
    cpu_lz4 = {"value": round(sample / dt / 1e9, 5), "unit": "GB/s", "cores": threads,
               "kind": "port", "sample": f"first {sample} B of the rank-0 1 GiB corpus, "
               f"{threads} pthreads over contiguous 300-B block ranges, {dt:.2f} s"}
    log(f"cpu lz4: {cpu_lz4}")
    cpu_jpeg = None
    if img is not None:
        h, w = img.shape[:2]
        ref = oracle_api.ref_jpeg()
        band = 8 * ((h // 8 + threads - 1) // threads)
        bands = [(y, min(h, y + band)) for y in range(0, h, band)]
        out = np.empty(((w + 7) // 8) * ((h + 7) // 8) * 128, np.int16)

        def run_band(y0, y1):
            sub = np.ascontiguousarray(img[y0:y1])
            o_sub = np.empty(((w + 7) // 8) * ((y1 - y0 + 7) // 8) * 128, np.int16)
            if ref is not None:
                ref.ref_jpeg_encode_image(sub.ctypes.data, w, y1 - y0, o_sub.ctypes.data)
            else:
                o.L.jo_encode_image(sub.ctypes.data, w, y1 - y0, o_sub.ctypes.data)
            out[(y0 // 8) * ((w + 7) // 8) * 128:][:o_sub.size] = o_sub

        t = time.perf_counter()
        ths = [threading.Thread(target=run_band, args=b) for b in bands]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        dt = time.perf_counter() - t
        cpu_jpeg = {"value": round(w * h / dt / 1e9, 6), "unit": "Gpixel/s", "cores": len(bands),
                    "kind": "reference" if ref is not None else "port",
                    "sample": f"one {w}x{h} image in {len(bands)} tile-row bands on "
                              f"{len(bands)} threads, {dt:.2f} s"
                              + (" (reference JPEG.c built from its sources, oracle/_ref)"
                                 if ref is not None else " (oracle port)")}
        log(f"cpu jpeg: {cpu_jpeg}")
    return cpu_lz4, cpu_jpeg


if __name__ == "__main__":
    main()
