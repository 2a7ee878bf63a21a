"""Static checks of the compressor's gfx950 code (CPU: hipcc cross-compiles).

lz4_tiles / lz4_matches drive `m0` from inline asm: it is the address base of
the ds_write_addtid_b32 stores (entries, accumulator zeroing, lcp keys) and the
lane select + counter of the greedy walk (csrc/lz4r.hip).  LLVM reserves m0
and refuses it in a clobber list ("clobbering reserved registers may lead to
undefined behaviour"), so instead of a declaration the generated code itself
is checked: no instruction outside the asm statements may read or write m0 in
these kernels, and every write of m0 that feeds an add-TID store is followed
by a wait state (the round-2 hang: the first add-TID store used the previous
block's m0 and left stale heads).

Two views of the same code, both built with the product's flags:
- the assembly of `lz4r.hip` compiled with the Makefile's own HIPFLAGS and
  LZ4R_HIPFLAGS (read from the Makefile, so a flag change there is a change
  here), where the
  compiler marks the inline asm (`;;#ASMSTART`/`;;#ASMEND`);
- the gfx950 code object extracted from the built `liblz4jpeg.so` (the bytes
  that ship), disassembled: every m0 access in it must be one of the asm
  statements' own (the same multiset as in the marked assembly), and the
  wait state must be there.
"""
import collections
import os
import re
import struct
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "lz4-jpeg_amd", "csrc", "lz4r.hip")
LIB = os.path.join(REPO, "lz4-jpeg_amd", "lz4jpeg", "liblz4jpeg.so")
HIPCC = "/opt/rocm/bin/hipcc"
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
KERNELS = ("lz4_tiles", "lz4_matches")


def _make_var(name):
    out = subprocess.run(["make", "-s", "-C", REPO, f"print-{name}"], check=True,
                         capture_output=True, text=True).stdout
    return out.split()


@pytest.fixture(scope="module")
def asm(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("no hipcc")
    flags = _make_var("HIPFLAGS") + _make_var("LZ4R_HIPFLAGS")   # lz4r.o's own additions
    assert "--offload-arch=gfx950" in flags and "-fno-strict-aliasing" in flags, flags
    out = tmp_path_factory.mktemp("isa") / "lz4r.s"
    subprocess.run([HIPCC, *flags, "--cuda-device-only", "-S", SRC, "-o", str(out)],
                   check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    return out.read_text().splitlines()


def _code_objects(path):
    """The gfx950 code objects of every offload bundle in a host binary."""
    data = open(path, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    objs, i = [], data.find(magic)
    while i >= 0:
        (n,) = struct.unpack_from("<Q", data, i + len(magic))
        o = i + len(magic) + 8
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", data, o)
            o += 24
            triple = data[o:o + tl].decode()
            o += tl
            if triple.endswith("gfx950") and size:
                objs.append(data[i + off:i + off + size])
        i = data.find(magic, i + 1)
    return objs


@pytest.fixture(scope="module")
def shipped(tmp_path_factory):
    if not os.path.exists(LIB) or not os.path.exists(OBJDUMP):
        pytest.skip("library not built")
    d = tmp_path_factory.mktemp("co")
    lines = []
    for k, co in enumerate(_code_objects(LIB)):
        p = d / f"co{k}.o"
        p.write_bytes(co)
        lines += subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", str(p)], check=True,
                                capture_output=True, text=True).stdout.splitlines()
    assert lines, "no gfx950 code object in liblz4jpeg.so"
    return lines


def _kernel_lines(lines, name):
    start = next(i for i, l in enumerate(lines) if re.match(rf"^_Z\S*{name}\S*:", l))
    end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
    return lines[start:end + 1]


def _shipped_kernels(lines, name):
    """Disassembled bodies (instruction text only) of every instance of a kernel."""
    bodies = []
    for i, l in enumerate(lines):
        if re.match(rf"^[0-9a-f]+ <_Z\S*{name}\S*>:", l):
            body = []
            for x in lines[i + 1:]:
                ins = x.split("//")[0].strip()
                if re.match(r"^[0-9a-f]+ <", x):
                    break
                if ins:
                    body.append(ins)
            bodies.append(body)
    return bodies


def _m0_ins(body):
    return [l for l in body if re.search(r"\bm0\b", l)]


def _norm(ins):
    """An m0 instruction with its registers abstracted (allocation may differ)."""
    ins = re.sub(r"\s+", " ", ins.split(";")[0].strip())
    return re.sub(r"\b[vs]\d+\b|\b[vs]\[\d+:\d+\]", "R", ins)


@pytest.mark.parametrize("kernel", KERNELS)
def test_m0_only_inside_asm(asm, kernel):
    body = _kernel_lines(asm, kernel)
    inside, outside = False, []
    for l in body:
        if ";;#ASMSTART" in l:
            inside = True
        elif ";;#ASMEND" in l:
            inside = False
        elif re.search(r"\bm0\b", l.split(";")[0]) and not inside:
            outside.append(l.strip())
    assert not outside, f"compiler-generated m0 uses in {kernel}: {outside}"


@pytest.mark.parametrize("kernel", KERNELS)
def test_m0_write_has_wait_state_before_addtid(asm, kernel):
    body = [l.strip() for l in _kernel_lines(asm, kernel)]
    n = 0
    for i, l in enumerate(body):
        if l.startswith("s_mov_b32 m0") and any("addtid" in x for x in body[i + 1:i + 4]):
            assert body[i + 1].startswith("s_nop"), body[i:i + 3]
            n += 1
    assert n >= 1


@pytest.mark.parametrize("kernel", KERNELS)
def test_shipped_m0_uses_are_the_asm_ones(asm, shipped, kernel):
    marked = collections.Counter(_norm(l) for l in _m0_ins(
        [x.split(";")[0].strip() for x in _kernel_lines(asm, kernel)]))
    bodies = _shipped_kernels(shipped, kernel)
    assert bodies, f"{kernel} not in the shipped code object"
    for body in bodies:
        got = collections.Counter(_norm(l) for l in _m0_ins(body))
        # every instance (template instantiations) uses a subset of the asm
        # statements' m0 instructions, and nothing else touches m0
        extra = got - marked
        assert not extra, f"m0 uses in the shipped {kernel} not from the asm: {extra}"


@pytest.mark.parametrize("kernel", KERNELS)
def test_shipped_m0_write_has_wait_state(shipped, kernel):
    for body in _shipped_kernels(shipped, kernel):
        n = 0
        for i, l in enumerate(body):
            if l.startswith("s_mov_b32 m0") and any("addtid" in x for x in body[i + 1:i + 4]):
                assert body[i + 1].startswith("s_nop"), body[i:i + 3]
                n += 1
        assert n >= 1, f"no add-TID m0 set found in the shipped {kernel}"
