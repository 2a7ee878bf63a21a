"""Per-basic-block dynamic instruction counts of lz4_tiles (tools only).

The roof of an issue-bound kernel needs the dynamic count of every opcode, not
only the SQ_INSTS_* totals, because gfx950 VALU opcodes do not cost the same
(profiles/r03_valu_rate.log: v_add/and/or/xor ~2.3 cycles per wave-instruction
per SIMD, VOP3-only / SGPR-operand / DPP / VOPC ~4, 64-bit shifts ~5.6).

  build   compile csrc/lz4r.hip with the product's HIPFLAGS to assembly, insert
          after every basic-block label of lz4_tiles<true> (and the inline-asm
          walk loop's local label) a counter bump -- EXEC saved to s[80:81],
          EXEC = lane 0, one vector global_atomic_add of 1 into
          lz4r_bb_acc[bb], EXEC restored -- so a block entered with EXEC = 0
          still counts (its VALU instructions still issue), assemble the code
          object (tools/ab/bbcnt.co) and write the static opcode list of every
          basic block of the UNinstrumented code (tools/ab/bb_static.json).
          The compiled kernel uses v0..v46 and s0..s31, so v60..v62 and
          s[80:81] are free; the descriptor is raised to cover them.
  run     (GPU box) load the code object as a module, compress the bench
          corpus (1 GiB, synthesised on the device) with it once, read the
          counters -> <out>/bbcounts.json.
  report  counts x static opcode lists -> dynamic opcodes per 300-B block,
          the cost-weighted VALU cycles (tools/valu_cost.py classes) and the
          per-pipe roof, optionally against a PMC summary.
"""
import collections
import ctypes
import json
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "tools", "ab")
LLVM = "/opt/rocm/lib/llvm/bin"
KERNEL = "_ZN12_GLOBAL__N_19lz4_tilesILb1EE"      # (a prefix: signatures change)
NCNT = 1024
LABEL = re.compile(r"^(\.LBB\d+_\d+):|^; (%bb\.\d+):|^\s*(1):\s*$")


def hipflags():
    out = []
    for v in ("HIPFLAGS", "LZ4R_HIPFLAGS"):        # lz4r.o's flags
        out += subprocess.run(["make", "-s", "-C", REPO, f"print-{v}"], check=True,
                              capture_output=True, text=True).stdout.split()
    return [f for f in out if f not in ("-fPIC",)]


def compile_asm(src, extra=(), flags=None):
    os.makedirs(OUT, exist_ok=True)
    s = os.path.join(OUT, "bb_src.s")
    subprocess.run(["/opt/rocm/bin/hipcc", *(flags or hipflags()), *extra, "--cuda-device-only",
                    "-S", src, "-o", s], check=True, stderr=subprocess.DEVNULL)
    return open(s).read().splitlines()


def kernel_range(L, name=KERNEL):
    st = next(i for i, l in enumerate(L) if re.match(re.escape(name) + r"\S*:\s*(;.*)?$", l))
    en = next(i for i in range(st, len(L)) if L[i].startswith(".Lfunc_end"))
    return st, en


def opcode(line):
    """The instruction text (opcode and operands) of an assembly line, or None."""
    t = line.split(";")[0].strip()
    if not t or t.startswith(".") or t.endswith(":") or t.startswith("//"):
        return None
    return " ".join(t.split())


def basic_blocks(L, st, en):
    """[(label, [opcodes])] of the function body: the entry block, then one
    per label (LLVM labels, fallthrough %bb comments, the asm loop's 1:)."""
    bbs = [("entry", [])]
    for i in range(st + 1, en):
        m = LABEL.match(L[i])
        if m:
            bbs.append((next(g for g in m.groups() if g), []))
            continue
        op = opcode(L[i])
        if op:
            bbs[-1][1].append(op)
    return bbs


# (registers {v}, {v1}, {v2} and s[{s}:{s1}] above every one the kernel uses)
BUMP = ["\ts_mov_b64 s[{s}:{s1}], exec",
        "\ts_mov_b64 exec, 1",
        "\ts_nop 1",
        "\tglobal_atomic_add v[{v}:{v1}], v{v2}, off offset:{off}",
        "\ts_mov_b64 exec, s[{s}:{s1}]",
        "\ts_nop 1"]
PROLOGUE = ["\ts_getpc_b64 s[{s}:{s1}]",
            "\ts_add_u32 s{s}, s{s}, lz4r_bb_acc@rel32@lo+4",
            "\ts_addc_u32 s{s1}, s{s1}, lz4r_bb_acc@rel32@hi+12",
            "\tv_mov_b32 v{v}, s{s}",
            "\tv_mov_b32 v{v1}, s{s1}",
            "\tv_mov_b32 v{v2}, 1"]


# a kernel with no free SGPR pair (lz4_decode_blocks uses s0..s98): EXEC saved
# in two lanes of a spare VGPR, the prologue's PC in VCC (unset at entry)
BUMP_V = ["\tv_writelane_b32 v{v3}, vcc_lo, 0",      # VCC parked in a spare VGPR,
          "\tv_writelane_b32 v{v3}, vcc_hi, 1",      # EXEC parked in VCC
          "\ts_mov_b64 vcc, exec",
          "\ts_mov_b64 exec, 1",
          "\ts_nop 1",
          "\tglobal_atomic_add v[{v}:{v1}], v{v2}, off offset:{off}",
          "\ts_mov_b64 exec, vcc",
          "\tv_readlane_b32 vcc_lo, v{v3}, 0",
          "\tv_readlane_b32 vcc_hi, v{v3}, 1",
          "\ts_nop 5"]
PROLOGUE_V = ["\ts_getpc_b64 vcc",
              "\ts_add_u32 vcc_lo, vcc_lo, lz4r_bb_acc@rel32@lo+4",
              "\ts_addc_u32 vcc_hi, vcc_hi, lz4r_bb_acc@rel32@hi+12",
              "\tv_mov_b32 v{v}, vcc_lo",
              "\tv_mov_b32 v{v1}, vcc_hi",
              "\tv_mov_b32 v{v2}, 1"]


def instrument(L, st, en, kname):
    body = L[st:en]
    used = set()
    for l in body:
        t = l.split(";")[0]
        for r in re.findall(r"\bv\[?(\d+)", t):
            used.add(("v", int(r)))
        for a, b in re.findall(r"\bv\[(\d+):(\d+)\]", t):
            used.update(("v", k) for k in range(int(a), int(b) + 1))
        for a, b in re.findall(r"\bs\[(\d+):(\d+)\]", t):
            used.update(("s", k) for k in range(int(a), int(b) + 1))
        for r in re.findall(r"\bs(\d+)\b", t):
            used.add(("s", int(r)))
    vb = (max(k for t, k in used if t == "v") + 2) & ~1
    sb = (max(k for t, k in used if t == "s") + 2) & ~1
    R = dict(v=vb, v1=vb + 1, v2=vb + 2, v3=vb + 3, s=sb, s1=sb + 1)
    vmode = sb + 2 > 100                                  # no free SGPR pair
    assert vb + 4 <= 256
    bump, pro = (BUMP_V, PROLOGUE_V) if vmode else (BUMP, PROLOGUE)
    out = list(L[:st + 1]) + [x.format(**R) for x in pro]
    k = 0
    off = lambda k: f"{4 * k}"
    out += [b.format(off=off(k), **R) for b in bump]      # entry block
    k += 1
    for i in range(st + 1, en):
        out.append(L[i])
        if LABEL.match(L[i]):
            out += [b.format(off=off(k), **R) for b in bump]
            k += 1
    assert k <= NCNT and 4 * k < 4096
    out += L[en:]
    txt = "\n".join(out)
    # descriptor / metadata: cover v60..v62 and s80..s81
    txt = re.sub(r"(\.amdhsa_kernel " + kname + r"\n(?:.*\n)*?\s*\.amdhsa_next_free_vgpr )\d+",
                 rf"\g<1>{(vb + 4 + 3) & ~3}", txt)
    txt = re.sub(r"(\.amdhsa_kernel " + kname + r"\n(?:.*\n)*?\s*\.amdhsa_accum_offset )\d+",
                 rf"\g<1>{(vb + 4 + 3) & ~3}", txt)
    if not vmode:
        txt = re.sub(r"(\.amdhsa_kernel " + kname + r"\n(?:.*\n)*?\s*\.amdhsa_next_free_sgpr )\d+",
                     rf"\g<1>{sb + 2}", txt)
    txt += ("\n\t.type\tlz4r_bb_acc,@object\n\t.section\t.bss.lz4r_bb_acc,\"aw\",@nobits\n"
            "\t.globl\tlz4r_bb_acc\n\t.protected\tlz4r_bb_acc\n\t.p2align\t8\nlz4r_bb_acc:\n\t.zero\t4096\n"
            "\t.size\tlz4r_bb_acc, 4096\n")
    return txt, k


EMIT = "_ZN12_GLOBAL__N_18lz4_emit"
DEC = "_ZN12_GLOBAL__N_117lz4_decode_blocks"
ENC = "_ZN12_GLOBAL__N_119entropy_encode_laneILb"   # + "1EE" (luma) / "0EE" (chroma)


def dec_flags():
    """lz4r_gpudec.o's flags: HIPFLAGS + its scheduler (the Makefile's target rule)."""
    base = subprocess.run(["make", "-s", "-C", REPO, "print-HIPFLAGS"], check=True,
                          capture_output=True, text=True).stdout.split()
    mk = open(os.path.join(REPO, "Makefile")).read()
    m = re.search(r"^\$\(B\)/lz4r_gpudec\.o: HIPFLAGS \+= (.*)$", mk, re.M)
    return [f for f in base if f != "-fPIC"] + (m.group(1).split() if m else [])


def build(src=None, name="prod", kernel=KERNEL):
    """kernel: KERNEL (lz4_tiles<true>), EMIT (lz4_emit; name gets an "emit_"
    prefix) or DEC (lz4_decode_blocks of lz4r_gpudec.hip; "dec_")."""
    if kernel == DEC:
        src = src or os.path.join(REPO, "lz4-jpeg_amd", "csrc", "lz4r_gpudec.hip")
        name = "dec_" + name
        L = compile_asm(src, ("-I", os.path.join(REPO, "include")), flags=dec_flags())
    elif kernel.startswith(ENC):
        src = src or os.path.join(REPO, "lz4-jpeg_amd", "csrc", "jpegr_entropy.hip")
        name = ("enc1_" if kernel.endswith("1EE") else "enc0_") + name
        base = subprocess.run(["make", "-s", "-C", REPO, "print-HIPFLAGS"], check=True,
                              capture_output=True, text=True).stdout.split()
        L = compile_asm(src, ("-I", os.path.join(REPO, "include")),
                        flags=[f for f in base if f != "-fPIC"])
    else:
        src = src or os.path.join(REPO, "lz4-jpeg_amd", "csrc", "lz4r.hip")
        if kernel == EMIT:
            name = "emit_" + name
        L = compile_asm(src)
    st, en = kernel_range(L, kernel)
    bbs = basic_blocks(L, st, en)
    kname = L[st].split(":")[0]
    txt, k = instrument(L, st, en, kname)
    assert k == len(bbs), (k, len(bbs))
    s = os.path.join(OUT, f"bbcnt_{name}.s")
    open(s, "w").write(txt)
    o = os.path.join(OUT, f"bbcnt_{name}.o")
    subprocess.run([f"{LLVM}/clang", "-target", "amdgcn-amd-amdhsa", "-mcpu=gfx950", "-c", s,
                    "-o", o], check=True)
    subprocess.run([f"{LLVM}/ld.lld", "-shared", o, "-o", os.path.join(OUT, f"bbcnt_{name}.co")],
                   check=True)
    json.dump({"kernel": kname, "bbs": bbs},
              open(os.path.join(OUT, f"bb_static_{name}.json"), "w"))
    print(f"{len(bbs)} basic blocks, {sum(len(b) for _, b in bbs)} static instructions")


def _launch(hip, fn, grid, block, args):
    params = (ctypes.c_void_p * len(args))(*[ctypes.cast(ctypes.pointer(a), ctypes.c_void_p)
                                              for a in args])
    assert hip.hipModuleLaunchKernel(fn, grid, 1, 1, block, 1, 1, 0, None, params, None) == 0


def run_emit(outdir, name="prod", nbytes=1 << 30):
    """The whole compressor from the module (lz4_tiles, the scans, the
    instrumented lz4_emit) on the bench corpus; the stream must equal the
    product library's."""
    import hashlib
    sys.path.insert(0, os.path.join(REPO, "lz4-jpeg_amd"))
    import torch
    from lz4jpeg import lz4, synth
    hip = ctypes.CDLL("libamdhip64.so")
    torch.cuda.init()
    dev = torch.device("cuda", 0)
    n = nbytes
    d_in = torch.empty(n + 16, dtype=torch.uint8, device=dev)
    synth.random_passages_device(d_in, n, length=30000, seed=1, first=0)
    nb = (n + 299) // 300
    last_n = n - (nb - 1) * 300
    slots = torch.empty(nb * (96 + 400), dtype=torch.uint8, device=dev)
    tsz = torch.empty(nb, dtype=torch.int32, device=dev)
    bsz = torch.empty(nb, dtype=torch.int16, device=dev)
    status = torch.zeros(4, dtype=torch.int64, device=dev)
    npart = (nb + 4095) // 4096
    gsum = torch.empty((nb + 63) // 64, dtype=torch.int32, device=dev)
    part = torch.empty(npart, dtype=torch.int64, device=dev)
    cap = 1 + nb * 548
    out = torch.empty(cap, dtype=torch.uint8, device=dev)
    boff = torch.empty(nb, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    mod = ctypes.c_void_p()
    assert hip.hipModuleLoad(ctypes.byref(mod),
                             os.path.join(OUT, f"bbcnt_emit_{name}.co").encode()) == 0
    S = json.load(open(os.path.join(OUT, f"bb_static_emit_{name}.json")))
    L = open(os.path.join(OUT, f"bbcnt_emit_{name}.s")).read()
    fns = {}
    for k in ("lz4_tilesILb1EE", "lz4_scan_reduce", "lz4_scan_partials", "lz4_emit"):
        mangled = re.search(r"^(_ZN12_GLOBAL__N_1\d+" + k + r"\S*?):", L, re.M).group(1)
        f = ctypes.c_void_p()
        assert hip.hipModuleGetFunction(ctypes.byref(f), mod, mangled.encode()) == 0, k
        fns[k] = f
    acc, accsz = ctypes.c_void_p(), ctypes.c_size_t()
    assert hip.hipModuleGetGlobal(ctypes.byref(acc), ctypes.byref(accsz), mod,
                                  b"lz4r_bb_acc") == 0
    assert hip.hipMemset(acc, 0, ctypes.c_size_t(4 * NCNT)) == 0
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    U32, U64, I32 = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int32
    per = (nb + 7) // 8
    heads, ovfs = P(slots), ctypes.c_void_p(slots.data_ptr() + nb * 96)
    _launch(hip, fns["lz4_tilesILb1EE"], 8 * per, 64,
            [P(d_in), U32(nb), U32(per), U32(last_n), heads, ovfs, P(tsz), P(bsz), P(status)])
    _launch(hip, fns["lz4_scan_reduce"], npart, 256, [P(tsz), U64(nb), U64(0), P(gsum), P(part)])
    lenp = ctypes.c_void_p(status.data_ptr() + 8)
    verd = ctypes.c_void_p(status.data_ptr() + 16)
    _launch(hip, fns["lz4_scan_partials"], 1, 1024,
            [P(part), U64(npart), U64(1), I32(1), I32(1), P(status), lenp, verd])
    ng = (nb + 63) // 64
    _launch(hip, fns["lz4_emit"], ng * 2, 512,
            [P(d_in), heads, ovfs, U64(0), P(tsz), U64(nb), U64(0), P(gsum), P(part), P(out),
             U64(cap), I32(1), U64(nb), U32(last_n), P(boff)])
    assert hip.hipDeviceSynchronize() == 0
    host = (ctypes.c_uint32 * NCNT)()
    assert hip.hipMemcpy(host, acc, ctypes.c_size_t(4 * NCNT), 2) == 0
    got = int(status[1].item())
    comp = lz4.Compressor()
    ref, rlen = comp.compress_device(d_in, n)
    same = rlen == got and bool(torch.equal(ref[:rlen], out[:got]))
    os.makedirs(outdir, exist_ok=True)
    res = {"bytes": n, "blocks": nb, "workgroups": ng * 2, "stream_equal_product": same,
           "counts": list(host)}
    json.dump(res, open(os.path.join(outdir, f"bbcounts_emit_{name}.json"), "w"))
    print(json.dumps({k: v for k, v in res.items() if k != "counts"}))


def run(outdir, name="prod", nbytes=1 << 30):
    sys.path.insert(0, os.path.join(REPO, "lz4-jpeg_amd"))
    import torch
    from lz4jpeg import synth
    hip = ctypes.CDLL("libamdhip64.so")
    torch.cuda.init()
    dev = torch.device("cuda", 0)
    n = nbytes
    d_in = torch.empty(n + 16, dtype=torch.uint8, device=dev)
    synth.random_passages_device(d_in, n, length=30000, seed=1, first=0)
    nb = (n + 299) // 300
    assert nb <= 1 << 24
    last_n = n - (nb - 1) * 300
    slots = torch.empty(nb * 640, dtype=torch.uint8, device=dev)
    usz = torch.empty(nb, dtype=torch.int32, device=dev)
    bsz = torch.empty(nb, dtype=torch.int16, device=dev)
    status = torch.zeros(2, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    mod = ctypes.c_void_p()
    assert hip.hipModuleLoad(ctypes.byref(mod),
                             os.path.join(OUT, f"bbcnt_{name}.co").encode()) == 0
    fn = ctypes.c_void_p()
    kname = json.load(open(os.path.join(OUT, f"bb_static_{name}.json")))["kernel"]
    assert hip.hipModuleGetFunction(ctypes.byref(fn), mod, kname.encode()) == 0
    acc, accsz = ctypes.c_void_p(), ctypes.c_size_t()
    assert hip.hipModuleGetGlobal(ctypes.byref(acc), ctypes.byref(accsz), mod,
                                  b"lz4r_bb_acc") == 0
    assert hip.hipMemset(acc, 0, ctypes.c_size_t(4 * NCNT)) == 0
    per = (nb + 7) // 8
    args = [ctypes.c_void_p(d_in.data_ptr()), ctypes.c_uint32(nb), ctypes.c_uint32(per),
            ctypes.c_uint32(last_n), ctypes.c_void_p(slots.data_ptr())]
    if "jjjPhS" in kname:             # (heads, overflow slots) since round 5
        args.append(ctypes.c_void_p(slots.data_ptr() + nb * 96))
    args += [ctypes.c_void_p(usz.data_ptr()), ctypes.c_void_p(bsz.data_ptr()),
             ctypes.c_void_p(status.data_ptr())]
    params = (ctypes.c_void_p * len(args))(*[ctypes.cast(ctypes.pointer(a), ctypes.c_void_p)
                                              for a in args])
    assert hip.hipModuleLaunchKernel(fn, 8 * per, 1, 1, 64, 1, 1, 0, None, params, None) == 0
    assert hip.hipDeviceSynchronize() == 0
    host = (ctypes.c_uint32 * NCNT)()
    assert hip.hipMemcpy(host, acc, ctypes.c_size_t(4 * NCNT), 2) == 0
    # the encoded sizes must equal the product's (the instrumentation changes no result)
    import numpy as np
    from lz4jpeg import lz4
    comp = lz4.Compressor()
    _, got = comp.compress_device(d_in, n)   # (the product library's result)
    off = comp.block_offsets(nb).astype(np.int64)
    prod = np.diff(np.append(off, got - 1))
    same = bool((prod == usz.cpu().numpy().astype(np.int64)).all())
    os.makedirs(outdir, exist_ok=True)
    res = {"bytes": n, "blocks": nb, "status": int(status[0].item()),
           "sizes_equal_product": same, "counts": list(host)}
    json.dump(res, open(os.path.join(outdir, f"bbcounts_{name}.json"), "w"))
    print(json.dumps({k: v for k, v in res.items() if k != "counts"}))


# cycles per wave-instruction per SIMD at 8 waves per SIMD (tools/valu_rate.hip;
# profiles/r03_valu_rate.log, profiles/r05_valu_rate.log)
FAST = {"v_add_u32", "v_xor_b32", "v_and_b32", "v_or_b32", "v_sub_u32", "v_mov_b32"}


def vcost(ins, table):
    op = ins.split()[0]
    base = re.sub(r"_e(32|64)$", "", op)
    args = ins.split(None, 1)[1] if " " in ins else ""
    srcs = ",".join(args.split(",")[1:])
    sgpr_src = bool(re.search(r"\bs\[?\d|\bvcc_(lo|hi)\b|\bexec|\bm0\b", srcs))
    if "_dpp" in op or " row_" in ins or "wave_sh" in ins or "quad_perm" in ins:
        return table["dpp"]
    if base in FAST:
        return table["vop2_sgpr"] if sgpr_src else table["fast"]
    for k in ("v_lshlrev_b64", "v_lshrrev_b64", "v_ashrrev_i64"):
        if base == k:
            return table["shift64"]
    if base == "v_cndmask_b32" and op.endswith("_e32"):
        return table["v_cndmask_b32_e32_vcc"]
    if base in table:
        return table[base]
    return table["default"]


def classify(ins):
    op = ins.split()[0]
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op in ("s_waitcnt", "s_nop", "s_endpgm", "s_barrier", "s_setprio", "s_sleep"):
        return op
    if op.startswith("s_"):
        return "salu"
    return "other"


def report(countsf, staticf, costf=None, pmcf=None, clock_ghz=None, ms_per_gib=None):
    C = json.load(open(countsf))
    S = json.load(open(staticf))
    nbk = C["blocks"]
    counts = C["counts"]
    bbs = S["bbs"]
    assert len(counts) >= len(bbs)
    dyn = collections.Counter()
    per_bb = []
    for (lab, ins), c in zip(bbs, counts):
        for x in ins:
            dyn[x] += c
        per_bb.append((lab, c / nbk, ins))
    cls = collections.Counter()
    ops = collections.Counter()
    for x, c in dyn.items():
        cls[classify(x)] += c / nbk
        ops[x.split()[0]] += c / nbk
    table = json.load(open(costf)) if costf else None
    out = {"blocks": nbk, "per_block": {k: round(v, 2) for k, v in sorted(cls.items())},
           "opcodes_per_block": {k: round(v, 2) for k, v in ops.most_common()}}
    if table:
        vcyc = sum(vcost(x, table) * c for x, c in dyn.items() if classify(x) == "valu") / nbk
        scyc = table["salu"] * cls["salu"]
        out["valu_cycles_per_block_per_simd"] = round(vcyc, 1)
        out["salu_cycles_per_block_per_simd"] = round(scyc, 1)
        bycost = collections.Counter()
        for x, c in dyn.items():
            if classify(x) == "valu":
                bycost[x.split()[0]] += vcost(x, table) * c / nbk
        out["valu_cycles_by_opcode"] = {k: round(v, 1) for k, v in bycost.most_common(40)}
        hot = []
        for lab, c, ins in per_bb:
            v = sum(vcost(x, table) for x in ins if classify(x) == "valu") * c
            sa = sum(1 for x in ins if classify(x) == "salu") * c * table["salu"]
            hot.append((v, lab, round(c, 3), len(ins), round(sa, 1)))
        hot.sort(reverse=True)
        out["hot_blocks"] = [{"bb": l, "execs_per_block": c, "static": n,
                              "valu_cycles": round(v, 1), "salu_cycles": sa}
                             for v, l, c, n, sa in hot[:40]]
    print(json.dumps(out, indent=1))
    return out


def run_dec(outdir, name="prod", nbytes=1 << 30):
    """The instrumented lz4_decode_blocks from the module over the product's
    compressed bench corpus (the compressor's device block offsets); the
    output must equal the input."""
    sys.path.insert(0, os.path.join(REPO, "lz4-jpeg_amd"))
    import torch
    from lz4jpeg import lz4, synth
    hip = ctypes.CDLL("libamdhip64.so")
    torch.cuda.init()
    n = nbytes
    d_in = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    synth.random_passages_device(d_in, n, length=30000, seed=1, first=0)
    comp = lz4.Compressor()
    d_stream, length = comp.compress_device(d_in, n)
    offs, nb = comp.block_offsets_device()
    out = torch.zeros(n + 300, dtype=torch.uint8, device="cuda")
    res = torch.tensor([0, -1], dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    mod = ctypes.c_void_p()
    assert hip.hipModuleLoad(ctypes.byref(mod), os.path.join(OUT, f"bbcnt_dec_{name}.co").encode()) == 0
    S = json.load(open(os.path.join(OUT, f"bb_static_dec_{name}.json")))
    f = ctypes.c_void_p()
    assert hip.hipModuleGetFunction(ctypes.byref(f), mod, S["kernel"].encode()) == 0
    acc, accsz = ctypes.c_void_p(), ctypes.c_size_t()
    assert hip.hipModuleGetGlobal(ctypes.byref(acc), ctypes.byref(accsz), mod, b"lz4r_bb_acc") == 0
    assert hip.hipMemset(acc, 0, ctypes.c_size_t(4 * NCNT)) == 0
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    U64 = ctypes.c_uint64
    grid = (nb + 31) // 32
    _launch(hip, f, grid, 64, [P(d_stream), U64(length), ctypes.c_void_p(offs), U64(nb), P(out),
                               U64(n + 300), P(res), ctypes.c_void_p(0), ctypes.c_void_p(0)])
    assert hip.hipDeviceSynchronize() == 0
    host = (ctypes.c_uint32 * NCNT)()
    assert hip.hipMemcpy(host, acc, ctypes.c_size_t(4 * NCNT), 2) == 0
    same = bool(torch.equal(out[:n], d_in[:n])) and int(res[0].item()) == n
    os.makedirs(outdir, exist_ok=True)
    r = {"bytes": n, "blocks": nb, "waves": grid, "output_equal_input": same, "counts": list(host)}
    json.dump(r, open(os.path.join(outdir, f"bbcounts_dec_{name}.json"), "w"))
    print(json.dumps({k: v for k, v in r.items() if k != "counts"}))


def run_enc(outdir, name="prod", luma="1"):
    """The instrumented entropy_encode_lane<luma> from the module over a 4K
    random image's coefficients (the product's encode_device); its bits,
    meta and table of that channel must equal the product's."""
    sys.path.insert(0, os.path.join(REPO, "lz4-jpeg_amd"))
    import torch
    from lz4jpeg import jpeg, synth
    hip = ctypes.CDLL("libamdhip64.so")
    torch.cuda.init()
    W, H = 3840, 2160
    d_img = torch.from_numpy(synth.rand_rgba(W, H, seed=1)).cuda()
    d_coef = jpeg.encode_device(d_img, W, H)
    nt = jpeg.tiles(W, H)
    ref = jpeg.Entropy(nt)
    ref.encode(d_coef)
    mine = jpeg.Entropy(nt)
    mine.scratch.zero_()
    torch.cuda.synchronize()
    tag = "enc1_" if luma == "1" else "enc0_"
    mod = ctypes.c_void_p()
    assert hip.hipModuleLoad(ctypes.byref(mod), os.path.join(OUT, f"bbcnt_{tag}{name}.co").encode()) == 0
    S = json.load(open(os.path.join(OUT, f"bb_static_{tag}{name}.json")))
    f = ctypes.c_void_p()
    assert hip.hipModuleGetFunction(ctypes.byref(f), mod, S["kernel"].encode()) == 0
    acc, accsz = ctypes.c_void_p(), ctypes.c_size_t()
    assert hip.hipModuleGetGlobal(ctypes.byref(acc), ctypes.byref(accsz), mod, b"lz4r_bb_acc") == 0
    assert hip.hipMemset(acc, 0, ctypes.c_size_t(4 * NCNT)) == 0
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    groups = (nt + 63) // 64 * (1 if luma == "1" else 2)
    deferred = ctypes.c_void_p(mine.scratch.data_ptr() + 256)
    _launch(hip, f, groups, 64, [P(d_coef), ctypes.c_uint64(nt), P(mine.bits), P(mine.meta),
                                 P(mine.table), P(mine.scratch), deferred, P(mine.status)])
    assert hip.hipDeviceSynchronize() == 0
    host = (ctypes.c_uint32 * NCNT)()
    assert hip.hipMemcpy(host, acc, ctypes.c_size_t(4 * NCNT), 2) == 0
    cs = [0] if luma == "1" else [1, 2]
    same = True
    for c in cs:
        off, n = (0, 128) if c == 0 else ((128, 64) if c == 1 else (192, 64))
        same &= bool(torch.equal(mine.meta.view(nt, 3)[:, c], ref.meta.view(nt, 3)[:, c]))
        same &= bool(torch.equal(mine.bits.view(nt, 256)[:, off:off + n], ref.bits.view(nt, 256)[:, off:off + n]))
    os.makedirs(outdir, exist_ok=True)
    r = {"tiles": nt, "waves": groups, "channel_equal_product": same, "counts": list(host)}
    json.dump(r, open(os.path.join(outdir, f"bbcounts_{tag}{name}.json"), "w"))
    print(json.dumps({k: v for k, v in r.items() if k != "counts"}))


if __name__ == "__main__":
    cmd = sys.argv[1]
    if cmd == "build_enc":          # build_enc 1|0 [src.hip name]
        build(*(sys.argv[3:5] or [None, "prod"]), kernel=ENC + sys.argv[2] + "EE")
    elif cmd == "run_enc":          # run_enc outdir 1|0 [name]
        run_enc(sys.argv[2], *(sys.argv[4:5] or ["prod"]), luma=sys.argv[3])
    elif cmd == "build_dec":
        build(*(sys.argv[2:4] or [None, "prod"]), kernel=DEC)
    elif cmd == "run_dec":
        run_dec(sys.argv[2], *sys.argv[3:4])
    elif cmd == "build":              # build [src.hip name]
        build(*sys.argv[2:4])
    elif cmd == "build_emit":       # build_emit [src.hip name]
        build(*(sys.argv[2:4] or [None, "prod"]), kernel=EMIT)
    elif cmd == "run_emit":         # run_emit outdir [name]
        run_emit(sys.argv[2], *sys.argv[3:4])
    elif cmd == "report":
        report(*sys.argv[2:5])
    elif cmd == "run":
        run(sys.argv[2], *sys.argv[3:4])   # run outdir [name]
    else:
        raise SystemExit(__doc__)
