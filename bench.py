#!/usr/bin/env python3
"""Headline benchmark (BASELINE.json): LZ4 compress GB/s + JPEG DCT Gpixel/s
on 1..8 MI355X, with % of the HBM roofline and the CPU path timed beside it.

    python bench.py [--gpus N --steps K --warmup W]

--gpus N > 1 without a launcher: bench.py starts N rank processes itself
(torch.distributed.run, one per GPU, before this process touches the GPU)
and exits with their status; under torchrun (WORLD_SIZE set) it is a rank.

Workloads (BASELINE.json configs):
  N = 1  top level = configs[1]: LZ4 compress of 1 GiB of random_extract-style
         text; "jpeg" = configs[2]: one 3840x2160 random RGB image.
  N > 1  top level = configs[3]: LZ4 compress of a 64 GiB corpus, static
         whole-300-B-block shards (64 GiB / N per rank, strong scaling), each
         rank's segment length all_gather'ed inside the step; the RCCL
         gatherv of all segments to rank 0 is timed apart as lz4_gather_ms.
         "jpeg" = configs[4]: 1024 distinct 4K images from one continuous
         rand() stream, 1024 / N per rank, no exchange.
Every rank synthesises its own share in HBM (csrc/synth_dev.hip) from the
seeded generators; a step is one pass of the hot path over the rank's share
with inputs resident in HBM.  Rank 0 prints one JSON line.
"""
import argparse
import datetime
import faulthandler
import json
import os
import socket
import subprocess
import sys
import threading
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(REPO, "lz4-jpeg_amd"), os.path.join(REPO, "tests")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_VALU_PEAK_TOPS = 39.3     # 78.6 TFLOPS fp64 vector spec counts FMA as 2
# per-launch HBM bytes from rocprofv3 FETCH_SIZE / WRITE_SIZE passes
# (tools/traffic.sh -> tools/traffic_summary.py, gfx950 FETCH correction applied)
TRAFFIC_JSON = os.path.join(REPO, "profiles", "r04_traffic.json")
# lz4_tiles' per-pipe roof from one profiled run (tools/r05_roof.sh ->
# tools/roof.py): dynamic opcode counts, PMC counts, time and clock together
ROOF_JSON = os.path.join(REPO, "profiles", "r05_roof.json")
# clock each kernel holds under its own load (DVFS give-back), from a
# GRBM_GUI_ACTIVE PMC pass (tools/clock_pmc.sh -> tools/clock_summary.py)
CLOCK_JSON = os.path.join(REPO, "profiles", "r04_clock.json")
SPEC_CLOCK_GHZ = 2.4

CFG4_BYTES = 64 << 30          # configs[3]
CFG5_IMAGES = 1024             # configs[4]
W4K, H4K = 3840, 2160


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def _profile_json(path):
    """This round's profile, else the latest earlier round's."""
    base = os.path.basename(path)[:4]
    for r in ("r06_", "r05_", "r04_", "r03_", "r02_", "r01_"):
        p = path.replace(base, r)
        if os.path.exists(p):
            return p
    return path


def held_clock(key):
    """Median clock (GHz) the profiled kernel `key` held, or None.  `key` may be
    a list of names, the first one profiled wins (kernel names change with
    their template arguments across rounds)."""
    keys = key if isinstance(key, (list, tuple)) else [key]
    try:
        prof = json.load(open(_profile_json(CLOCK_JSON)))
    except (OSError, ValueError):
        return None
    for k in keys:
        try:
            return float(prof[k]["ghz_median"])
        except (KeyError, ValueError, TypeError):
            continue
    return None


def settle(fn, sync, ms=60.0, chunk=8):
    """Untimed warm-up of a sub-line until `ms` of back-to-back work has run:
    the chip's clock ramps over ~40 ms of sustained load (a 4K single-image
    JPEG launch takes 83.5 us over its first 100 launches and settles at
    64.8 us after ~500, tools/jpeg_settle.py; an LZ4 call 3.19 -> 2.87 ms over
    6 calls), so a sub-line timed after a few warm-up launches measures the
    ramp.  Returns the number of warm-up calls.  (The top-level line keeps
    exactly the driver's W warm-up steps.)"""
    t0, n = time.perf_counter(), 0
    while time.perf_counter() - t0 < ms / 1e3:
        for _ in range(chunk):
            fn()
        n += chunk
        sync()
    return n


def at_held_clock(achieved, peak_spec, key):
    """The spec peak rescaled to the clock `key` holds under load, and the
    fraction of that; {} when no clock profile is present."""
    f = held_clock(key)
    if not f:
        return {}
    p = peak_spec * f / SPEC_CLOCK_GHZ
    return {"held_clock_ghz": f, "peak_at_held_clock": round(p, 2),
            "frac_at_held_clock": round(achieved / p, 4)}


def issue_roof(bytes_now, launch_ms):
    """lz4_tiles' binding roof (tools/roof.py -> ROOF_JSON): per 300-B block,
    lower bounds on the SIMD cycles of its VALU instructions (the dynamic
    opcode counts of tools/bbcount.py priced at the cheapest issue rate the
    micro-benchmarks measure for each class), its SALU instructions and its
    LDS-array cycles, all from one profiled run on one box (counts, time and
    clock of the same dispatches).  frac = the largest pipe's CU cycles per
    block / the measured CU cycles per block of that run (<= 1: lower
    bounds) of this bench's own lz4_tiles time priced at the profile's
    clock; profile_frac is the profiled run's fraction."""
    try:
        d = json.load(open(_profile_json(ROOF_JSON)))
        roof = d["roof_cu_cycles_per_block"]
        bind = d["binding_pipe"]
        meas = d["measured"]["median"]
    except (OSError, KeyError, ValueError):
        return None
    nb = (bytes_now + 299) // 300
    live_cyc = launch_ms / 1e3 * meas["clock_ghz"] * 1e9 * 256 / nb
    return {
        "bound": f"{bind} issue", "unit": "CU cycles per 300-B block",
        "roof_cu_cycles_per_block": roof, "binding_pipe": bind,
        "measured_cu_cycles_per_block": meas["cu_cycles_per_block"],
        "profile_clock_ghz": meas["clock_ghz"], "profile_ms": meas["ms"],
        # frac: this run's lz4_tiles time priced at the profile's clock;
        # profile_frac: the profiled run's own fraction (static, from the file)
        "frac": round(roof[bind] / live_cyc, 4),
        "profile_frac": d["frac"], "profile_frac_by_pipe": d["frac_by_pipe"],
        "live_cu_cycles_per_block_at_profile_clock": round(live_cyc, 1),
        "per_block": d["per_block"],
        "note": "from " + os.path.basename(_profile_json(ROOF_JSON)) + " (tools/roof.py): "
                "VALU = lower bound of the vector-issue cycles per block per SIMD "
                "(per-opcode dynamic counts x the cheapest measured rate of each class, "
                "tools/valu_rate.hip), SALU = SQ_INSTS_SALU x the s_add rate, LDS = "
                "SQ_LDS_IDX_ACTIVE; four SIMDs share a CU's LDS, so the roof is "
                "max(VALU/4, SALU/4, LDS) CU cycles per block",
    }


def measured_traffic(kind, bytes_now, bytes_profiled):
    """HBM bytes per launch of the profiled kernel, scaled to this launch's
    input size (the profile ran the same configuration), or None."""
    try:
        t = json.load(open(_profile_json(TRAFFIC_JSON)))[kind]
    except (OSError, KeyError, ValueError):
        return None
    return int(round(t["traffic_bytes"] * bytes_now / bytes_profiled))


# --------------------------------------------------------------- launcher
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launcher_cmd(nproc, argv, port):
    """The command that runs this script as `nproc` ranks on one node."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={nproc}", "--master-addr=127.0.0.1", f"--master-port={port}",
            os.path.abspath(__file__)] + list(argv)


def maybe_self_launch(args, argv, env=None):
    """--gpus N > 1 outside a launcher: start the N ranks as child processes
    (this process never touches the GPU; a process that has may not exec) and
    return their exit status.  None when this process is a rank itself."""
    env = os.environ if env is None else env
    if (args.gpus <= 1 and not getattr(args, "dist", False)) or "WORLD_SIZE" in env:
        return None
    cmd = launcher_cmd(args.gpus, argv, _free_port())
    log("launching", args.gpus, "ranks:", " ".join(cmd[2:]))
    child_env = dict(env)
    child_env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=child_env)


def phase(name, rank, limit_s):
    """Mark the start of a bench phase on this rank.  If the phase has not
    ended `limit_s` seconds later (a collective that never completes, a
    stuck kernel), every thread's stack is dumped to stderr and the rank
    exits non-zero, so a first-time 8-GPU run fails with the phase named
    instead of being killed silently at the driver's limit."""
    log(f"rank {rank}: phase {name}")
    faulthandler.dump_traceback_later(limit_s, exit=True)


def rank_env(env=None):
    env = os.environ if env is None else env
    return (int(env.get("WORLD_SIZE", "1")), int(env.get("RANK", "0")),
            int(env.get("LOCAL_RANK", "0")))


def workloads(world, args):
    """(lz4 bytes in total, jpeg images in total, scaling) for this job."""
    if world == 1 and not getattr(args, "dist", False):
        return args.lz4_bytes_per_rank, args.jpeg_images_per_rank, "weak"
    total = args.lz4_total_bytes or CFG4_BYTES
    imgs = args.jpeg_total_images or CFG5_IMAGES
    return total, imgs, "strong"


def image_share(total, world, rank):
    """Contiguous images [i0, i1) of a `total`-image batch for `rank`."""
    return (total * rank) // world, (total * (rank + 1)) // world


def host_cpu_cores():
    """Cores this process may use: its affinity set, capped by a cgroup CPU
    quota when one is set (a GPU box shares its node's CPUs)."""
    n = len(os.sched_getaffinity(0))
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


# ------------------------------------------------------------------- main
def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--lz4-bytes-per-rank", type=int, default=1 << 30,
                    help="N = 1 workload (configs[1])")
    ap.add_argument("--lz4-total-bytes", type=int, default=0,
                    help="N > 1 workload; default 64 GiB (configs[3])")
    ap.add_argument("--jpeg-w", type=int, default=W4K)
    ap.add_argument("--jpeg-h", type=int, default=H4K)
    ap.add_argument("--jpeg-images-per-rank", type=int, default=1,
                    help="N = 1 workload (configs[2])")
    ap.add_argument("--jpeg-total-images", type=int, default=0,
                    help="N > 1 workload; default 1024 (configs[4])")
    ap.add_argument("--jpeg-steps", type=int, default=0, help="default: max(50, 10*steps)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-jpeg", action="store_true")
    ap.add_argument("--no-cfg4-share", action="store_true",
                    help="skip the 8 GiB config-4 per-GPU share line at N = 1")
    ap.add_argument("--no-jpeg-batch", action="store_true",
                    help="skip the 128-image single-launch JPEG line at N = 1")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="target wall time of the all-core CPU-baseline sample")
    ap.add_argument("--dist", action="store_true",
                    help="run the N > 1 code path (RCCL process group, sharded config-4/5 "
                         "workloads, length all_gather, gatherv) even at one rank: the "
                         "world-size-1 rehearsal of the 8-GPU job")
    ap.add_argument("--dist-timeout", type=float, default=120.0,
                    help="seconds: the process group's collective timeout (RCCL watchdog "
                         "aborts the rank) and the per-phase watchdog of every rank")
    ap.add_argument("--launch-check", action="store_true",
                    help="print each rank's (rank, world, local rank, shares) and exit "
                         "without touching the GPU (tests the launcher plumbing)")
    args = ap.parse_args(argv)

    rc = maybe_self_launch(args, argv)
    if rc is not None:
        sys.exit(rc)
    if args.launch_check:
        from lz4jpeg import dist as ldist
        world, rank, local = rank_env()
        lz4_total, jpeg_total, scaling = workloads(world, args)
        print(json.dumps({"rank": rank, "world": world, "local_rank": local,
                          "lz4_shard": list(ldist.shard_bytes(lz4_total, world, rank)),
                          "jpeg_images": list(image_share(jpeg_total, world, rank)),
                          "scaling": scaling}), flush=True)
        return

    import torch
    import torch.distributed as dist

    world, rank, local = rank_env()
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    multi = world > 1 or args.dist       # the distributed code path
    if multi:
        # a collective that has not completed after dist_timeout aborts the
        # rank (the RCCL watchdog tears the communicator down, the process
        # exits non-zero) -- well inside the driver's 600 s for the run
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "3")
        phase("init_process_group", rank, args.dist_timeout + 60)
        dist.init_process_group("nccl", device_id=dev,
                                timeout=datetime.timedelta(seconds=args.dist_timeout))
    ctx = Ctx(world, rank, dev, args, torch, dist, multi)
    lz4_total, jpeg_total, scaling = workloads(world, args)

    line = run_lz4(ctx, lz4_total, scaling)
    if not args.no_jpeg:
        ctx.phase("jpeg")
        line["jpeg"] = run_jpeg(ctx, jpeg_total, scaling)
    else:
        line["jpeg"] = None

    if rank == 0 and not multi and not args.no_cpu_baseline:
        cpu_lz4, cpu_jpeg = cpu_baselines(ctx.host_text, args, ctx.host_img)
        line["cpu_baseline"] = cpu_lz4
        if line["jpeg"] is not None:
            line["jpeg"]["cpu_baseline"] = cpu_jpeg
    if rank == 0:
        print(json.dumps(line), flush=True)
    if multi:
        phase("destroy_process_group", rank, args.dist_timeout + 60)
        dist.destroy_process_group()
    faulthandler.cancel_dump_traceback_later()


class Ctx:
    def __init__(self, world, rank, dev, args, torch, dist, multi=None):
        self.world, self.rank, self.dev, self.args = world, rank, dev, args
        self.torch, self.dist = torch, dist
        # the distributed code path (a process group exists): world > 1, or the
        # --dist rehearsal at one rank
        self.multi = world > 1 if multi is None else multi
        self.host_text = None
        self.host_img = None

    def phase(self, name):
        if self.multi:
            phase(name, self.rank, self.args.dist_timeout + 60)

    def barrier(self):
        if self.multi:
            self.dist.barrier()

    def all_ranks(self, x):
        """[x of rank 0, ..., x of rank W-1] (a float per rank)."""
        if not self.multi:
            return [x]
        t = self.torch.tensor([x], dtype=self.torch.float64, device=self.dev)
        g = self.torch.empty(self.world, dtype=self.torch.float64, device=self.dev)
        self.dist.all_gather_into_tensor(g, t)
        return [float(v) for v in g.cpu().tolist()]

    def max_over_ranks(self, x):
        if not self.multi:
            return x
        t = self.torch.tensor([x], dtype=self.torch.float64, device=self.dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum_over_ranks(self, x):
        if not self.multi:
            return x
        t = self.torch.tensor([x], dtype=self.torch.int64, device=self.dev)
        self.dist.all_reduce(t)
        return int(t.item())


def run_lz4(ctx, n_total, scaling):
    import numpy as np
    torch = ctx.torch
    from lz4jpeg import dist as ldist
    from lz4jpeg import lz4, synth
    args, world, rank, dev = ctx.args, ctx.world, ctx.rank, ctx.dev
    lo, hi = ldist.shard_bytes(n_total, world, rank)
    n = hi - lo
    final_shard = hi == n_total
    log(f"rank {rank}: synthesising LZ4 shard [{lo}, {hi}) of {n_total} B in HBM")
    if rank == 0 and not ctx.multi:
        # bounded host copy for the CPU baseline (the same bytes); made before
        # the device input so that seconds of host work do not sit between the
        # device synthesis and the warm-up steps (the clock ramps back up over
        # ~40 ms of load, see settle())
        ctx.host_text = synth.random_passages(min(n, 1 << 30), length=30000, seed=1, first=lo)
    d_in = torch.empty(n + 16, dtype=torch.uint8, device=dev)
    synth.random_passages_device(d_in, n, length=30000, seed=1, first=lo)
    # clock pre-warm, not a warm-up step: ~100 ms of unrelated device work
    # (elementwise passes over 256 MB) so that the W warm-up steps already run
    # at the held clock and a kernel trace's average over every launch of the
    # run agrees with the timed steps (settle())
    d_warm = torch.zeros(256 << 20, dtype=torch.uint8, device=dev)
    settle(lambda: d_warm.add_(1), torch.cuda.synchronize, ms=100.0, chunk=16)
    del d_warm
    comp = lz4.Compressor()
    # text grows by ~3.5 %; the call reports the need if a shard ever exceeds this
    cap = n + n // 8 + (1 << 20)
    d_out = torch.empty(1 + cap, dtype=torch.uint8, device=dev)   # [frame byte] + segment
    d_len = torch.zeros(1, dtype=torch.int64, device=dev)
    # N = 1: one int64 length slot per call (warm-up and timed), so every
    # call's length -- and its corrupt-index bit 63 -- survives to be checked
    # after the timed region
    d_lens = torch.zeros(max(1, args.warmup + args.steps), dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream()

    def lz4_step(i):
        if not ctx.multi:
            # stream-ordered, as a device-resident pipeline runs it: the length
            # stays in HBM (slot i of d_lens) and is read after the timed steps,
            # so consecutive calls queue back to back with no host round trip
            comp.compress_async(d_in, n, d_out, d_lens[i:i + 1])
            return None
        comp.compress_async(d_in, n, d_out[1:], d_len, segment=True, final_shard=final_shard)
        # the raw signed length (negative: a corrupt LDS index); exchange_lengths
        # gathers it first and then raises on every rank (raising here would
        # leave the other ranks waiting in the collective).  This read-back +
        # all_gather is part of the N > 1 step: the gather offsets need it
        seg = int(d_len.item())
        ldist.exchange_lengths(seg, dev)
        return seg

    def slot_lengths(i0, i1):
        """Lengths of the N = 1 calls i0..i1-1 (one read-back); raises on a
        corrupt verdict in any of them."""
        vals = [int(v) for v in d_lens[i0:i1].cpu().tolist()]
        bad = [i0 + k for k, v in enumerate(vals) if v < 0]
        if bad:
            raise lz4.Lz4Error(-6, f"lz4: calls {bad} flagged a corrupt LDS index")
        return vals

    # the per-call timing events are created and first recorded in the warm-up
    # steps (their one-off cost would otherwise land in the timed steps)
    ctx.phase("lz4 warm-up")
    comp.set_timing(True)
    out_len = None
    for i in range(args.warmup):
        out_len = lz4_step(i)
    if args.warmup and not ctx.multi:
        warm = slot_lengths(0, args.warmup)
        if len(set(warm)) != 1:
            raise RuntimeError(f"lz4: warm-up call lengths differ: {sorted(set(warm))}")
        out_len = warm[-1]
    if out_len is not None and out_len > cap:
        raise RuntimeError(f"lz4: output {out_len} B exceeds the bench buffer {cap} B")
    torch.cuda.synchronize()
    ctx.barrier()
    comp.set_timing(True)                  # a new record: the timed calls only
    torch.cuda.synchronize()
    ctx.phase("lz4 timed steps")
    ctx.barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        got = lz4_step(args.warmup + i)
    torch.cuda.synchronize()
    t_rank = time.perf_counter() - t0      # this rank's own time, before the barrier
    ctx.barrier()
    dt = ctx.max_over_ranks(time.perf_counter() - t0)
    if not ctx.multi:
        lens_timed = slot_lengths(args.warmup, args.warmup + args.steps)
        if out_len is not None and any(v != out_len for v in lens_timed):
            raise RuntimeError(f"lz4: timed call lengths {sorted(set(lens_timed))} != "
                               f"warm-up length {out_len}")
        out_len = lens_timed[-1]
    else:
        out_len = got
    call_ms, match_ms = comp.timed_calls(args.steps)
    comp.set_timing(False)
    lz4_ms = dt / args.steps * 1e3
    lz4_gbs = n_total / (dt / args.steps) / 1e9
    rank_match_ms = ctx.all_ranks(sum(match_ms) / len(match_ms))
    rank_call_ms = ctx.all_ranks(sum(call_ms) / len(call_ms))
    rank_step_ms = ctx.all_ranks(t_rank / args.steps * 1e3)
    avg_match_ms = max(rank_match_ms)
    avg_call_ms = max(rank_call_ms)
    out_total = ctx.sum_over_ranks(out_len) + (1 if ctx.multi else 0)
    cs = sorted(call_ms)
    log(f"lz4: {lz4_ms:.3f} ms/step, {lz4_gbs:.1f} GB/s aggregate, lz4_tiles "
        f"{avg_match_ms:.3f} ms, call {avg_call_ms:.3f} ms, out {out_total} B; call "
        f"min/median/max {cs[0]:.3f}/{cs[len(cs) // 2]:.3f}/{cs[-1]:.3f} ms")
    per_rank = None
    if ctx.multi:
        per_rank = {
            "call_ms": [round(v, 4) for v in rank_call_ms],
            "lz4_tiles_ms": [round(v, 4) for v in rank_match_ms],
            "step_ms": [round(v, 4) for v in rank_step_ms],
            "call_ms_min_max": [round(min(rank_call_ms), 4), round(max(rank_call_ms), 4)],
            "note": "per rank: average compress call and lz4_tiles time (library HIP events) "
                    "and the rank's own step time before the closing barrier"}
        log(f"lz4 per rank: call ms {per_rank['call_ms']}, step ms {per_rank['step_ms']}")

    # decoder: this rank's blocks -> bytes, in HBM, with the
    # compressor's device-resident block offsets (no host round trip)
    ctx.phase("lz4 decode")
    nb_local = ldist.nblocks(n)
    if not ctx.multi:
        _, flen = comp.compress_device(d_in, n, d_out)
    else:
        comp.compress_async(d_in, n, d_out[1:], d_len, segment=True, final_shard=final_shard)
        flen = 1 + comp.async_length(d_len)
        d_out[0] = nb_local & 0xFF
    d_boff, _ = comp.block_offsets_device()
    d_dec = torch.empty(n + 300, dtype=torch.uint8, device=dev)
    _, got = lz4.decompress_device(d_out, flen, d_boff, nb_local, n + 300, d_out=d_dec)
    dec_ok = got == n and bool(torch.equal(d_dec[:n], d_in[:n]))
    torch.cuda.synchronize()
    dec_warm = settle(lambda: lz4.decompress_device(d_out, flen, d_boff, nb_local, n + 300,
                                                    d_out=d_dec, check=False),
                      torch.cuda.synchronize)
    ctx.barrier()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(args.steps):
        lz4.decompress_device(d_out, flen, d_boff, nb_local, n + 300, d_out=d_dec, check=False)
    e1.record(stream)
    torch.cuda.synchronize()
    ctx.barrier()
    ddt = ctx.max_over_ranks(time.perf_counter() - t0)
    dec_kern_ms = ctx.max_over_ranks(e0.elapsed_time(e1) / args.steps)
    dec_ok = ctx.sum_over_ranks(0 if dec_ok else 1) == 0
    del d_dec
    lz4_dec = {
        "metric": "LZ4 block-parallel decode GB/s (decoded bytes, stream resident in HBM)",
        "value": round(n_total / (ddt / args.steps) / 1e9, 3), "unit": "GB/s",
        "kernel": "lz4_decode_blocks", "avg_launch_ms": round(dec_kern_ms, 4),
        "roundtrip_ok": dec_ok, "offsets": "device-resident, written by lz4_emit",
        "warmup_launches": dec_warm,
        "roofline": {
            "bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS,
            "achieved": round((n + flen) / (dec_kern_ms / 1e3) / 1e9, 2),
            "frac": round((n + flen) / (dec_kern_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
            "note": "algorithmic bytes = compressed bytes read + decoded bytes written"},
    }
    log(f"lz4 decode: {dec_kern_ms:.3f} ms/launch, {lz4_dec['value']} GB/s, ok={dec_ok}")

    ctx.phase("lz4 bare-stream decode")
    # the same stream decoded from the bytes alone (LZ4_decode, LZ4.c:1038):
    # block boundaries found on the device, then the block decoder
    d_dec = torch.empty(n + 300, dtype=torch.uint8, device=dev)
    _, got = lz4.decompress_stream_device(d_out, flen, n + 300, d_out=d_dec)
    bare_ok = got == n and bool(torch.equal(d_dec[:n], d_in[:n]))
    torch.cuda.synchronize()
    bare_warm = settle(lambda: lz4.decompress_stream_device(d_out, flen, n + 300, d_out=d_dec),
                       torch.cuda.synchronize, chunk=2)
    ctx.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        lz4.decompress_stream_device(d_out, flen, n + 300, d_out=d_dec)
    torch.cuda.synchronize()
    ctx.barrier()
    bdt = ctx.max_over_ranks(time.perf_counter() - t0)
    bare_ok = ctx.sum_over_ranks(0 if bare_ok else 1) == 0
    del d_dec
    lz4_dec["bare_stream"] = {
        "metric": "LZ4 decode GB/s from the stream alone (lz4r_decompress_stream_device)",
        "value": round(n_total / (bdt / args.steps) / 1e9, 3), "unit": "GB/s",
        "call_ms": round(bdt / args.steps * 1e3, 4), "roundtrip_ok": bare_ok,
        "warmup_calls": bare_warm,
        "note": "whole synchronous call: on-device block-boundary discovery (lz4_bare_*), "
                "lz4_decode_blocks, one host read-back"}
    log(f"lz4 bare-stream decode: {bdt / args.steps * 1e3:.3f} ms/call, "
        f"{lz4_dec['bare_stream']['value']} GB/s, ok={bare_ok}")

    # N > 1: assemble the framed stream on rank 0 (RCCL gatherv over xGMI)
    gather_ms = gather_ok = None
    if ctx.multi:
        ctx.phase("lz4 gather")
        comp.compress_async(d_in, n, d_out[1:], d_len, segment=True, final_shard=final_shard)
        seg = int(d_len.item())              # raw: exchange_lengths raises on every rank
        lens, offs = ldist.exchange_lengths(seg, dev)
        torch.cuda.synchronize()
        ctx.barrier()
        g0 = time.perf_counter()
        full = ldist.gather_stream(d_out[1:], seg, ldist.nblocks(n_total), lens, offs, dst=0)
        torch.cuda.synchronize()
        ctx.barrier()
        gather_ms = ctx.max_over_ranks(time.perf_counter() - g0) * 1e3
        if rank == 0:
            # rank 0's own segment and the frame byte are where they belong
            gather_ok = (int(full[0].item()) == ldist.nblocks(n_total) & 0xFF and
                         bool(torch.equal(full[1:1 + seg], d_out[1:1 + seg])))
            del full
        log(f"lz4 gather: {gather_ms:.2f} ms for {sum(lens) + 1} B in pieces of "
            f"<= {ldist.GATHER_CHUNK} B")

    # N = 1: one GPU's share of config 4 (the 8-GPU job's rank-0 shard: the
    # first 8 GiB of the 64 GiB corpus) with the N > 1 step -- a segment
    # compress and its length read back (the all_gather of one rank is that
    # read) -- so the driver's 1 -> 8 curve has a same-work denominator
    share = None
    if not ctx.multi and not args.no_cfg4_share:
        share = run_cfg4_share(ctx, comp)

    roof_lz4 = {
        "bound": "hbm", "kernel": "lz4_tiles",
        "achieved": round(n / (avg_match_ms / 1e3) / 1e9, 2), "peak": HBM_PEAK_GBS,
        "unit": "GB/s", "frac": round(n / (avg_match_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
        "traffic": measured_traffic("lz4", n, 1 << 30),
        # HBM bytes of the whole compressor (lz4_tiles + lz4_emit) per call; the
        # call's algorithmic bytes are 1 B read + ~1.035 B written per input byte
        "pipeline_traffic": (None if measured_traffic("lz4_emit", n, 1 << 30) is None else
                             measured_traffic("lz4", n, 1 << 30) +
                             measured_traffic("lz4_emit", n, 1 << 30)),
        "binding_roof": issue_roof(n, avg_match_ms),
        "algorithmic_bytes_per_launch": n,
        "avg_launch_ms": round(avg_match_ms, 4),
        "whole_call_ms": round(avg_call_ms, 4),
        "note": "algorithmic bytes = 1 B read per input byte (SURVEY §8d: the HBM-read "
                "roofline); achieved = that / lz4_tiles time (summed over its 2^24-block "
                "launch chunks) from HIP events on its launch stream in each timed step, max "
                "over ranks; traffic = FETCH_SIZE(x2, gfx950) + WRITE_SIZE per launch from " +
                os.path.basename(_profile_json(TRAFFIC_JSON)) + "; the kernel is issue-bound "
                "(DESIGN.md), not HBM-bound",
    }
    comp.close()
    cfg = ("lz4_compress_1GiB_text_per_gpu" if not ctx.multi else
           "lz4_compress_64GiB_text_sharded_rccl_gather")
    if not ctx.multi and n != 1 << 30:
        cfg = f"lz4_compress_{n}B_text_per_gpu"
    if ctx.multi and n_total != CFG4_BYTES:
        cfg = f"lz4_compress_{n_total}B_text_sharded_rccl_gather"
    return {
        "metric": "LZ4 compress GB/s + JPEG DCT Mpixel/s at 1/2/4/8 MI355X; % HBM roofline",
        "value": round(lz4_gbs, 3), "unit": "GB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(lz4_ms, 4),
        "higher_is_better": True, "scaling": scaling, "vs_baseline": None, "dtype": "u8",
        "data": "synthetic: random_extract-style 30000-B passages of Metamorphosis.txt, "
                "newlines->spaces, glibc rand seed 1; each rank synthesises its shard in HBM",
        "config": {"workload": cfg, "bytes_per_rank": n, "bytes_total": n_total, "block": 300,
                   "parallelism": f"shard{world}", "compressed_bytes_total": out_total,
                   "step": ("compress (stream-ordered: the K calls queue back to back, each "
                            "call's length read after the timed region)" if not ctx.multi else
                            "segment compress + length read-back + all_gather of segment "
                            "lengths (a host round trip per step)")},
        "roofline": roof_lz4,
        "cpu_baseline": None,
        "lz4_gather_ms": None if gather_ms is None else round(gather_ms, 3),
        "lz4_gather_ok": gather_ok,
        "lz4_gather_chunk_bytes": ldist.GATHER_CHUNK if ctx.multi else None,
        "per_rank": per_rank,
        "value_incl_gather": (None if gather_ms is None else
                              round(n_total / ((lz4_ms + gather_ms) / 1e3) / 1e9, 3)),
        "value_per_gpu": round(lz4_gbs / world, 3),
        "cfg4_share": share,
        "lz4_decode": lz4_dec,
    }


def run_cfg4_share(ctx, comp):
    """configs[3]'s per-GPU work at 8 GPUs on this one GPU: the 8 GiB shard
    [0, 8 GiB) of the 64 GiB corpus, compressed as a segment per step."""
    torch = ctx.torch
    from lz4jpeg import dist as ldist
    from lz4jpeg import lz4, synth
    args, dev = ctx.args, ctx.dev
    world8 = 8
    lo, hi = ldist.shard_bytes(CFG4_BYTES, world8, 0)
    n = hi - lo
    d_in = torch.empty(n + 16, dtype=torch.uint8, device=dev)
    synth.random_passages_device(d_in, n, length=30000, seed=1, first=lo)
    cap = n + n // 8 + (1 << 20)
    d_out = torch.empty(cap, dtype=torch.uint8, device=dev)
    d_len = torch.zeros(1, dtype=torch.int64, device=dev)

    def step():
        comp.compress_async(d_in, n, d_out, d_len, segment=True, final_shard=False)
        return comp.async_length(d_len)

    comp.set_timing(True)                  # events made in the warm-up (two chunks here)
    for _ in range(max(1, args.warmup)):
        seg = step()
    if seg > cap:
        raise RuntimeError(f"lz4 cfg4 share: segment {seg} B exceeds {cap} B")
    torch.cuda.synchronize()
    warm = max(1, args.warmup) + settle(step, torch.cuda.synchronize, chunk=1)
    tiles = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        seg = step()
        tiles.append(comp.last_timing()[1])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    comp.set_timing(False)
    del d_in, d_out
    res = {
        "metric": "LZ4 compress GB/s of one GPU's share of configs[3] (8 GPUs)",
        "value": round(n / (dt / args.steps) / 1e9, 3), "unit": "GB/s",
        "ms_per_step": round(dt / args.steps * 1e3, 4), "steps": args.steps, "warmup": warm,
        "bytes": n, "segment_bytes": seg, "lz4_tiles_ms": round(sum(tiles) / len(tiles), 4),
        "step": "segment compress (lz4r_compress_segment_async) + length read-back",
        "note": "the 8-GPU job's rank-0 shard [0, 8 GiB) of the 64 GiB corpus; x8 is the "
                "ideal 8-GPU configs[3] value (no scaling loss)"}
    log(f"lz4 cfg4 share: {res['ms_per_step']} ms/step, {res['value']} GB/s")
    return res


def run_jpeg(ctx, total_images, scaling):
    import numpy as np
    torch = ctx.torch
    from lz4jpeg import jpeg, synth
    args, world, rank, dev = ctx.args, ctx.world, ctx.rank, ctx.dev
    stream = torch.cuda.current_stream()
    W, H = args.jpeg_w, args.jpeg_h
    i0, i1 = image_share(total_images, world, rank)
    B = i1 - i0
    px = W * H
    # images [i0, i1) of one continuous rand() stream (random_image.c:64-73):
    # image k = pixels [k W H, (k + 1) W H)
    d_img = torch.empty(4 * px * B, dtype=torch.uint8, device=dev)
    synth.rand_rgba_device(d_img, i0 * px, px * B, seed=1)
    if rank == 0 and not ctx.multi:
        ctx.host_img = synth.rand_rgba_stream(0, px, 1).reshape(H, W, 4)
    d_coef = torch.empty(B * jpeg.coef_count(W, H), dtype=torch.int16, device=dev)
    jsteps = args.jpeg_steps or (max(50, 10 * args.steps) if B == 1 else max(5, args.steps))
    for _ in range(max(args.warmup, 3)):
        jpeg.encode_device(d_img, W, H, B, d_coef)
    torch.cuda.synchronize()
    jwarm = max(args.warmup, 3) + settle(lambda: jpeg.encode_device(d_img, W, H, B, d_coef),
                                         torch.cuda.synchronize, chunk=50 if B == 1 else 1)
    ctx.barrier()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(jsteps):
        jpeg.encode_device(d_img, W, H, B, d_coef)
    ev1.record(stream)
    torch.cuda.synchronize()
    ctx.barrier()
    jdt = ctx.max_over_ranks(time.perf_counter() - t0)
    kern_ms = ctx.max_over_ranks(ev0.elapsed_time(ev1) / jsteps)
    px_total = px * total_images
    gpix = px_total / (jdt / jsteps) / 1e9
    px_rank = px * B
    tiles = ((W + 7) // 8) * ((H + 7) // 8) * B
    if not ctx.multi:
        wl = "jpeg_encode_3840x2160_rgb" if (W, H, B) == (W4K, H4K, 1) else f"jpeg_encode_{B}x{W}x{H}"
    else:
        wl = (f"jpeg_encode_{total_images}x{W}x{H}_rand_stream" if (W, H) != (W4K, H4K) or
              total_images != CFG5_IMAGES else "jpeg_encode_1024x4K_rand_stream")
    jres = {
        "metric": "JPEG DCT+quant+zigzag Gpixel/s (bit-exact int16 coefficients)",
        "value": round(gpix, 3), "unit": "Gpixel/s", "n_gpus": world, "steps": jsteps,
        "warmup": jwarm,
        "value_per_gpu": round(gpix / world, 3),
        "ms_per_step": round(jdt / jsteps * 1e3, 4), "higher_is_better": True,
        "scaling": scaling, "dtype": "f64",
        "data": "synthetic: glibc rand() RGBA noise (random_image.c) from srand(1), images "
                "drawn from one continuous stream",
        "config": {"workload": wl, "w": W, "h": H, "images_total": total_images,
                   "images_per_rank": B, "parallelism": f"images{world}"},
        "roofline": {
            "bound": "hbm", "kernel": "jpeg_strip_kernel",
            "achieved": round(8 * px_rank / (kern_ms / 1e3) / 1e9, 2), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(8 * px_rank / (kern_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
            "traffic": measured_traffic("jpeg", px_rank, W4K * H4K),
            "algorithmic_bytes_per_launch": 8 * px_rank,
            "avg_launch_ms": round(kern_ms, 4),
            "binding_roof": {
                "bound": "valu_fp64", "unit": "Tops/s",
                "achieved": round(tiles * 13312 / (kern_ms / 1e3) / 1e12, 2),
                "peak": FP64_VALU_PEAK_TOPS,
                "frac": round(tiles * 13312 / (kern_ms / 1e3) / 1e12 / FP64_VALU_PEAK_TOPS, 4),
                **at_held_clock(tiles * 13312 / (kern_ms / 1e3) / 1e12, FP64_VALU_PEAK_TOPS,
                                ["jpeg:void jpeg_strip_kernel<false>"]),
                "note": "13312 non-fused fp64 mul/add per tile in reference order "
                        "(8704 luma + 2x2304 chroma); peak = 78.6 TF fp64 vector spec / 2 at "
                        "2.4 GHz; peak_at_held_clock = the same per cycle at the clock the "
                        "kernel holds under its own load (" + os.path.basename(CLOCK_JSON) + ")",
            },
            "note": "8 B/pixel algorithmic (4 B RGBA read + 4 B int16 written); traffic "
                    "from PMC FETCH_SIZE x2 + WRITE_SIZE",
        },
    }
    log(f"jpeg: {jres['ms_per_step']} ms/step, {gpix:.2f} Gpix/s aggregate, kernel {kern_ms:.4f} ms")

    if not ctx.multi and B == 1 and not args.no_jpeg_batch:
        # config 5's per-GPU share at 8 GPUs (images 0..127 of the stream) in one
        # launch: the single-image line above pays the launch ramp and drain once
        # per 4K image
        NB = CFG5_IMAGES // 8
        d_bimg = torch.empty(4 * px * NB, dtype=torch.uint8, device=dev)
        synth.rand_rgba_device(d_bimg, 0, px * NB, seed=1)
        d_bcoef = torch.empty(NB * jpeg.coef_count(W, H), dtype=torch.int16, device=dev)
        jpeg.encode_device(d_bimg, W, H, NB, d_bcoef)
        b_ok = bool(torch.equal(d_bcoef[:jpeg.coef_count(W, H)], d_coef[:jpeg.coef_count(W, H)]))
        torch.cuda.synchronize()
        bwarm = settle(lambda: jpeg.encode_device(d_bimg, W, H, NB, d_bcoef), torch.cuda.synchronize,
                       chunk=1)
        bsteps = max(3, args.steps // 2)
        b0, b1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        b0.record(stream)
        for _ in range(bsteps):
            jpeg.encode_device(d_bimg, W, H, NB, d_bcoef)
        b1.record(stream)
        torch.cuda.synchronize()
        bms = b0.elapsed_time(b1) / bsteps
        btiles = ((W + 7) // 8) * ((H + 7) // 8) * NB
        jres["batch"] = {
            "metric": "JPEG DCT+quant+zigzag Gpixel/s, 128 images per launch",
            "value": round(px * NB / (bms / 1e3) / 1e9, 3), "unit": "Gpixel/s",
            "images": NB, "avg_launch_ms": round(bms, 4), "image0_equals_single": b_ok,
            "warmup": bwarm,
            "roofline": {
                "bound": "valu_fp64", "unit": "Tops/s", "peak": FP64_VALU_PEAK_TOPS,
                "achieved": round(btiles * 13312 / (bms / 1e3) / 1e12, 2),
                "frac": round(btiles * 13312 / (bms / 1e3) / 1e12 / FP64_VALU_PEAK_TOPS, 4),
                **at_held_clock(btiles * 13312 / (bms / 1e3) / 1e12, FP64_VALU_PEAK_TOPS,
                                ["jpeg:void jpeg_strip_kernel<false>"]),
                "hbm_frac": round(8 * px * NB / (bms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)},
            "note": "images 0..127 of the continuous rand() stream: config 5's per-GPU share "
                    "at 8 GPUs, on one GPU",
        }
        del d_bimg, d_bcoef
        log(f"jpeg batch of {NB}: {bms:.3f} ms/launch, {jres['batch']['value']} Gpix/s, "
            f"fp64 roof frac {jres['batch']['roofline']['frac']}")

    # the (f)-row stages run on this rank's first image
    d1_img = d_img[:4 * px]
    d1_coef = d_coef[:jpeg.coef_count(W, H)]
    rsteps = max(50, 10 * args.steps)
    # reconstruction: coefficients -> reconstructed RGBA
    jpeg.reconstruct_device(d1_coef, W, H, 1, d_orig=d1_img)
    torch.cuda.synchronize()
    rwarm = settle(lambda: jpeg.reconstruct_device(d1_coef, W, H, 1, d_orig=d1_img),
                   torch.cuda.synchronize, chunk=50)
    r0, r1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    r0.record(stream)
    for _ in range(rsteps):
        jpeg.reconstruct_device(d1_coef, W, H, 1, d_orig=d1_img)
    r1.record(stream)
    torch.cuda.synchronize()
    rec_ms = r0.elapsed_time(r1) / rsteps
    t1 = ((W + 7) // 8) * ((H + 7) // 8)
    jres["reconstruct"] = {
        "metric": "JPEG reconstruction (dequant + fp64 IDCT + YCbCr->RGB) Gpixel/s",
        "value": round(px / (rec_ms / 1e3) / 1e9, 3), "unit": "Gpixel/s",
        "kernel": "jpeg_recon_kernel", "avg_launch_ms": round(rec_ms, 4), "images": 1,
        "warmup": rwarm,
        "roofline": {
            "bound": "valu_fp64", "unit": "Tops/s", "peak": FP64_VALU_PEAK_TOPS,
            "achieved": round(t1 * 13568 / (rec_ms / 1e3) / 1e12, 2),
            "frac": round(t1 * 13568 / (rec_ms / 1e3) / 1e12 / FP64_VALU_PEAK_TOPS, 4),
            "hbm_gbs": round(8 * px / (rec_ms / 1e3) / 1e9, 2),
            "note": "13568 non-fused fp64 mul/add per tile (dequant x alpha 2x128, luma 8x(64 + "
                    "1024), chroma 2x8x(32 + 256)); 8 B/px algorithmic HBM "
                    "(4 B int16 read + 4 B RGBA written)"},
    }
    log(f"jpeg reconstruct: {rec_ms:.4f} ms, {jres['reconstruct']['value']} Gpix/s")

    # entropy stage: RLE + per-stream Huffman + bits, and back
    ent = jpeg.Entropy(t1, device=dev)
    ent.encode(d1_coef)
    d_back = torch.empty_like(d1_coef)
    ent.decode(d_back)
    torch.cuda.synchronize()
    ent_ok = bool(torch.equal(d_back, d1_coef)) and int(ent.status[0].item()) == 0 \
        and int(ent.status[1].item()) == 0
    meta = ent.meta.to(torch.int64) & 0xFFFFFFFF
    sum_bits = int((meta & 0xFFFF).sum().item())
    sum_codes = int((meta >> 24).sum().item())

    def ent_pair():
        ent.encode(d1_coef)
        ent.decode(d_back)
    ewarm = settle(ent_pair, torch.cuda.synchronize, chunk=20)
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    e0.record(stream)
    for _ in range(rsteps):
        ent.encode(d1_coef)
    e1.record(stream)
    for _ in range(rsteps):
        ent.decode(d_back)
    e2.record(stream)
    torch.cuda.synchronize()
    enc_ms, dec_ms = e0.elapsed_time(e1) / rsteps, e1.elapsed_time(e2) / rsteps
    # algorithmic bytes: coefficients (256 B/tile) + bits + table + meta
    ebytes = 256 * t1 + sum_bits // 8 + 4 * sum_codes + 12 * t1
    jres["entropy"] = {
        "metric": "JPEG entropy stage (RLE + per-block Huffman, JPEG.c:767-1097) Gpixel/s",
        "value": round(px / (enc_ms / 1e3) / 1e9, 3), "unit": "Gpixel/s", "images": 1,
        "encode_ms": round(enc_ms, 4), "decode_ms": round(dec_ms, 4), "warmup": ewarm,
        "decode_gpix_s": round(px / (dec_ms / 1e3) / 1e9, 3),
        "kernels": ["entropy_encode_lane", "entropy_decode_kernel"],
        "bits_per_pixel": round(sum_bits / px, 4), "roundtrip_ok": ent_ok,
        "roofline": {"bound": "issue (serial per-stream integer work)", "unit": "GB/s",
                     "hbm_achieved": round(ebytes / (enc_ms / 1e3) / 1e9, 2),
                     "peak": HBM_PEAK_GBS,
                     "frac": round(ebytes / (enc_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                     "note": "one lane per (tile, channel) stream; algorithmic bytes = "
                             "256 B coefficients + bits + code table + meta per tile"},
    }
    del ent, d_back
    log(f"jpeg entropy: encode {enc_ms:.4f} ms, decode {dec_ms:.4f} ms, "
        f"{jres['entropy']['value']} Gpix/s, {sum_bits / px:.3f} bits/px, ok={ent_ok}")
    return jres


# ---------------------------------------------------------- CPU baselines
def _run_threads(fn, ranges):
    ths = [threading.Thread(target=fn, args=r) for r in ranges]
    t = time.perf_counter()
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    return time.perf_counter() - t


def cpu_baselines(text, args, img):
    """Reference-path CPU throughput on this host (rank 0, N=1 only), on
    bounded samples of the same workloads: every core the process may use,
    and one core."""
    import numpy as np
    import oracle_api
    cores = host_cpu_cores()
    o = oracle_api.load()

    # LZ4: the oracle port (kind "port": the reference LZ4.c #includes the
    # Windows-only <direct.h> (LZ4.c:17) and cannot be built here)
    def lz4_rate(threads, seconds):
        calib = min(text.size, (1 << 20) * threads) // 300 * 300
        scratch = np.empty((calib // 300 + 1) * o.L.lz4o_block_bound(), np.uint8)
        t = time.perf_counter()
        o.L.lz4o_encode_parallel(text.ctypes.data, calib, threads, scratch.ctypes.data)
        rate = calib / max(time.perf_counter() - t, 1e-6)
        sample = int(min(text.size, max(calib, rate * seconds)))
        sample -= sample % 300
        scratch = np.empty((sample // 300 + 1) * o.L.lz4o_block_bound(), np.uint8)
        t = time.perf_counter()
        o.L.lz4o_encode_parallel(text.ctypes.data, sample, threads, scratch.ctypes.data)
        dt = time.perf_counter() - t
        return sample, dt

    s_all, dt_all = lz4_rate(cores, args.cpu_seconds)
    s_one, dt_one = lz4_rate(1, min(5.0, args.cpu_seconds / 2))
    cpu_lz4 = {"value": round(s_all / dt_all / 1e9, 5), "unit": "GB/s", "cores": cores,
               "kind": "port",
               "value_1core": round(s_one / dt_one / 1e9, 6),
               "sample": f"first {s_all} B of the 1 GiB corpus on {cores} pthreads over "
                         f"contiguous 300-B block ranges ({dt_all:.2f} s); 1 core: first {s_one} B "
                         f"({dt_one:.2f} s)",
               "note": "the oracle's restatement of LZ4.c (bit-identical); the reference LZ4.c "
                       "#includes the Windows-only <direct.h> (LZ4.c:17) and cannot be built"}
    log(f"cpu lz4: {cpu_lz4}")
    cpu_jpeg = None
    if img is not None:
        h, w = img.shape[:2]
        ref = oracle_api.ref_jpeg()

        def encode_rows(y0, y1, out):
            sub = np.ascontiguousarray(img[y0:y1])
            o_sub = np.empty(((w + 7) // 8) * ((y1 - y0 + 7) // 8) * 128, np.int16)
            if ref is not None:
                ref.ref_jpeg_encode_image(sub.ctypes.data, w, y1 - y0, o_sub.ctypes.data)
            else:
                o.L.jo_encode_image(sub.ctypes.data, w, y1 - y0, o_sub.ctypes.data)
            out[(y0 // 8) * ((w + 7) // 8) * 128:][:o_sub.size] = o_sub

        out = np.empty(((w + 7) // 8) * ((h + 7) // 8) * 128, np.int16)
        band = 8 * ((h // 8 + cores - 1) // cores)
        bands = [(y, min(h, y + band), out) for y in range(0, h, band)]
        dt_all = _run_threads(encode_rows, bands)
        # one core: the first 1/16 of the image's tile rows
        rows1 = max(8, (h // 16) // 8 * 8)
        dt_one = _run_threads(encode_rows, [(0, rows1, out)])
        kind = "reference" if ref is not None else "port"
        cpu_jpeg = {"value": round(w * h / dt_all / 1e9, 6), "unit": "Gpixel/s",
                    "cores": len(bands), "kind": kind,
                    "value_1core": round(w * rows1 / dt_one / 1e9, 7),
                    "sample": f"one {w}x{h} image in {len(bands)} tile-row bands on "
                              f"{len(bands)} threads ({dt_all:.2f} s); 1 core: its first "
                              f"{rows1} rows ({dt_one:.2f} s)" +
                              (" (reference JPEG.c built from its sources, oracle/_ref)"
                               if ref is not None else " (oracle port)")}
        log(f"cpu jpeg: {cpu_jpeg}")
    return cpu_lz4, cpu_jpeg


if __name__ == "__main__":
    main()
