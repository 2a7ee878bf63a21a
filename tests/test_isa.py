"""Static checks of the compressor's gfx950 code (CPU: hipcc cross-compiles).

lz4_tiles / lz4_matches drive `m0` from inline asm: it is the address base of
the ds_write_addtid_b32 stores that empty the bucket heads, and the lane
select + counter of the greedy walk (csrc/lz4r.hip).  LLVM reserves m0 and
refuses it in a clobber list ("clobbering reserved registers may lead to
undefined behaviour"), so instead of a declaration the generated code itself
is checked: no instruction outside the asm statements may read or write m0
in these kernels, and every asm write of m0 that feeds an add-TID store is
followed by a wait state (the round-2 hang: the first add-TID store used the
previous block's m0 and left stale heads).
"""
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "lz4-jpeg_amd", "csrc", "lz4r.hip")
HIPCC = "/opt/rocm/bin/hipcc"
KERNELS = ("lz4_tiles", "lz4_matches")


@pytest.fixture(scope="module")
def asm(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("no hipcc")
    out = tmp_path_factory.mktemp("isa") / "lz4r.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-std=c++17",
                    "--cuda-device-only", "-S", SRC, "-o", str(out)], check=True,
                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    return out.read_text().splitlines()


def _kernel_lines(lines, name):
    start = next(i for i, l in enumerate(lines) if re.match(rf"^_Z\S*{name}\S*:", l))
    end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
    return lines[start:end + 1]


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
    for i, l in enumerate(body):
        if l.startswith("s_mov_b32 m0") and any("addtid" in x for x in body[i + 1:i + 4]):
            assert body[i + 1].startswith("s_nop"), body[i:i + 3]
