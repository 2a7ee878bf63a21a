"""The drop-in executables (lz4-jpeg_amd/bin/{LZ4,JPEG}_{seq,par}.exe) honour
the reference's file contract: run from Experiment/ with the
reference's relative paths, exit status 0, outputs bit-exact to the oracle,
visual PNGs pixel-equal to the reference's own writers.  The reference's own
unmodified benchmark drivers (compiled from Experiment/*_experiment.c into
oracle/_ref) drive them end to end."""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

import golden_inputs
import pngdec

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "lz4-jpeg_amd", "bin")
REF = os.path.join(REPO, "oracle", "_ref")


def layout(tmp):
    """Experiment/ (cwd) beside Output-Input/ and Assets/, as in the reference."""
    for d in ("Experiment/results", "Output-Input/input", "Output-Input/out", "Output-Input/log",
              "Output-Input/Images", "Assets/Images"):
        os.makedirs(os.path.join(tmp, d), exist_ok=True)
    for exe in ("LZ4_seq.exe", "JPEG_seq.exe"):
        shutil.copy(os.path.join(BIN, exe), os.path.join(tmp, "Experiment", exe))
    shutil.copy(os.path.join(golden_inputs.GOLDEN, "Metamorphosis.txt"),
                os.path.join(tmp, "Output-Input/input/Metamorphosis.txt"))
    return os.path.join(tmp, "Experiment")


def run(cwd, cmd, timeout=120):
    env = dict(os.environ, PATH=".:" + os.environ.get("PATH", ""))
    return subprocess.run(cmd, cwd=cwd, env=env, capture_output=True, timeout=timeout)


def test_lz4_seq_file_contract(tmp_path, oracle):
    exp = layout(str(tmp_path))
    data = golden_inputs.lz4_input("text_10000")
    open(tmp_path / "Output-Input/input/input.txt", "wb").write(data)
    (tmp_path / "Output-Input/out/compressed.bin").write_bytes(b"stale")   # truncated first
    r = run(exp, ["./LZ4_seq.exe"])
    assert r.returncode == 0, r.stderr
    comp = (tmp_path / "Output-Input/out/compressed.bin").read_bytes()
    assert comp == oracle.lz4_compress(data)
    hexdump = (tmp_path / "Output-Input/out/compressed.txt").read_text()
    assert hexdump == "".join("%02X " % b for b in comp)                   # LZ4.c:101
    assert (tmp_path / "Output-Input/out/uncompressed.txt").read_bytes() == data


def test_lz4_seq_committed_golden(tmp_path):
    exp = layout(str(tmp_path))
    shutil.copy(os.path.join(golden_inputs.GOLDEN, "lz4_input.txt"),
                tmp_path / "Output-Input/input/input.txt")
    assert run(exp, ["./LZ4_seq.exe"]).returncode == 0
    ref = open(os.path.join(golden_inputs.GOLDEN, "lz4_input.compressed.bin"), "rb").read()
    assert (tmp_path / "Output-Input/out/compressed.bin").read_bytes() == ref
    # the hex dump (LZ4.c:75-107, written at :739) byte for byte against the
    # reference's own committed Output-Input/out/compressed.txt
    ref_txt = open(os.path.join(golden_inputs.GOLDEN, "lz4_input.compressed.txt"), "rb").read()
    assert (tmp_path / "Output-Input/out/compressed.txt").read_bytes() == ref_txt


def test_lz4_seq_too_small_exits_1(tmp_path):
    exp = layout(str(tmp_path))
    (tmp_path / "Output-Input/input/input.txt").write_bytes(b"y" * 299)
    r = run(exp, ["./LZ4_seq.exe"])
    assert r.returncode == 1                                               # LZ4.c:632-637
    assert b"block length is too high" in r.stdout


@pytest.mark.parametrize("w,h", [(64, 48), (37, 21), (1, 1)])
def test_jpeg_seq_file_contract(tmp_path, oracle, w, h):
    exp = layout(str(tmp_path))
    img = oracle.rand_image(w, h, seed=5)
    pngdec.write(str(tmp_path / "Assets/Images/rand_8X8.png"), img)
    r = run(exp, ["./JPEG_seq.exe"])
    assert r.returncode == 0, r.stderr
    coef = np.fromfile(tmp_path / "Output-Input/Images/coefficients.bin", dtype="<i2")
    assert np.array_equal(coef, oracle.jpeg_encode(img))
    orig = pngdec.read(str(tmp_path / "Output-Input/Images/original.png"))
    assert np.array_equal(orig, img)
    lum = pngdec.read(str(tmp_path / "Output-Input/Images/luminance.png"))
    y = np.empty((h, w), np.uint8)
    cr = np.empty((h, w), np.uint8)
    cb = np.empty((h, w), np.uint8)
    import ctypes
    oracle.L.jo_planes(np.ascontiguousarray(img).ctypes.data_as(ctypes.c_void_p), w, h,
                       y.ctypes.data_as(ctypes.c_void_p), cr.ctypes.data_as(ctypes.c_void_p),
                       cb.ctypes.data_as(ctypes.c_void_p))
    assert np.array_equal(lum[..., 0], y) and np.array_equal(lum[..., 2], y)
    for name in ("rChrominance.png", "bChrominance.png"):
        assert (tmp_path / "Output-Input/Images" / name).exists()
    import oracle_api
    rec = pngdec.read(str(tmp_path / "Output-Input/Images/reconstructed.png"))
    assert np.array_equal(rec, oracle_api.reconstruct(oracle, img))


def test_jpeg_seq_missing_image_exits_1(tmp_path):
    exp = layout(str(tmp_path))
    r = run(exp, ["./JPEG_seq.exe"])
    assert r.returncode == 1 and b"Error loading image" in r.stdout


@pytest.mark.slow
@pytest.mark.skipif(not os.path.exists(os.path.join(REF, "LZ4_sequential_experiment")),
                    reason="reference drivers not built (no /root/reference at build time)")
def test_reference_lz4_driver_runs_unchanged(tmp_path, oracle):
    """Experiment/LZ4_sequential_experiment.c, unmodified: 10 sizes x 10 runs of
    popen("LZ4_seq.exe"); it loops forever on a non-zero exit, so finishing at
    all means every run exited 0."""
    exp = layout(str(tmp_path))
    r = run(exp, [os.path.join(REF, "LZ4_sequential_experiment")], timeout=600)
    assert r.returncode == 0, r.stdout[-2000:]
    res = json.load(open(os.path.join(exp, "results", "LZ4_seq.exe_execution_times.json")))
    assert [e["text"] for e in res] == [350, 500, 1000, 2000, 5000, 10000, 15000, 20000,
                                        25000, 30000]
    data = (tmp_path / "Output-Input/input/input.txt").read_bytes()       # last extract
    assert (tmp_path / "Output-Input/out/compressed.bin").read_bytes() == oracle.lz4_compress(data)


@pytest.mark.slow
@pytest.mark.skipif(not os.path.exists(os.path.join(REF, "JPEG_sequential_experiment")),
                    reason="reference drivers not built (no /root/reference at build time)")
def test_reference_jpeg_driver_runs_unchanged(tmp_path, oracle):
    """Experiment/JPEG_sequential_experiment.c, unmodified: images 1x1 .. 2048x2048
    written by stb_image_write, 10 runs each, popen("JPEG_seq.exe")."""
    exp = layout(str(tmp_path))
    r = run(exp, [os.path.join(REF, "JPEG_sequential_experiment")], timeout=900)
    assert r.returncode == 0, r.stdout[-2000:]
    res = json.load(open(os.path.join(exp, "results", "JPEG_seq.exe_execution_times.json")))
    assert [e["image_size"] for e in res] == [2 ** i for i in range(12)]
    img = pngdec.read(str(tmp_path / "Assets/Images/rand_8X8.png"))       # last image
    coef = np.fromfile(tmp_path / "Output-Input/Images/coefficients.bin", dtype="<i2")
    assert np.array_equal(coef, oracle.jpeg_encode(img))


def _layout_par(tmp):
    exp = layout(tmp)
    for exe in ("LZ4_par.exe", "JPEG_par.exe"):
        shutil.copy(os.path.join(BIN, exe), os.path.join(exp, exe))
    return exp


def test_lz4_par_file_contract(tmp_path, oracle):
    exp = _layout_par(str(tmp_path))
    data = golden_inputs.lz4_input("text_10000")
    open(tmp_path / "Output-Input/input/input.txt", "wb").write(data)
    r = run(exp, ["./LZ4_par.exe"])
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "Output-Input/out/compressed.bin").read_bytes() == oracle.lz4_compress(data)
    assert (tmp_path / "Output-Input/out/uncompressed.txt").read_bytes() == data
    assert b"Number of cores available:" in r.stdout        # parallel LZ4.c:1246


@pytest.mark.skipif(not os.path.exists(os.path.join(REF, "LZ4_parallel_experiment")),
                    reason="reference drivers not built (no /root/reference at build time)")
def test_reference_lz4_parallel_driver_runs_unchanged(tmp_path, oracle):
    """Experiment/LZ4_parallel_experiment.c, unmodified: 10 runs of
    popen("LZ4_par.exe 2>&1") on 350-B extracts, retrying until exit 0."""
    exp = _layout_par(str(tmp_path))
    r = run(exp, [os.path.join(REF, "LZ4_parallel_experiment")], timeout=300)
    assert r.returncode == 0, r.stdout[-2000:]
    res = json.load(open(os.path.join(exp, "results", "LZ4_par.exe_execution_times.json")))
    assert [e["text"] for e in res] == [350] and len(res[0]["execution_times_sec"]) == 10
    assert r.stdout.count(b"[SUCCESS] LZ4 processing successful") == 10
    data = (tmp_path / "Output-Input/input/input.txt").read_bytes()
    assert (tmp_path / "Output-Input/out/compressed.bin").read_bytes() == oracle.lz4_compress(data)


@pytest.mark.slow
@pytest.mark.skipif(not os.path.exists(os.path.join(REF, "JPEG_parallel_experiment")),
                    reason="reference drivers not built (no /root/reference at build time)")
def test_reference_jpeg_parallel_driver_runs_unchanged(tmp_path, oracle):
    """Experiment/JPEG_parallel_experiment.c, unmodified: images 1x1 .. 2048x2048,
    10 runs each, system("JPEG_par.exe"); every run must succeed."""
    exp = _layout_par(str(tmp_path))
    r = run(exp, [os.path.join(REF, "JPEG_parallel_experiment")], timeout=900)
    assert r.returncode == 0, r.stdout[-2000:]
    assert b"[ERROR] JPEG processing failed" not in r.stdout
    assert r.stdout.count(b"[SUCCESS] JPEG processing successful") == 120
    res = json.load(open(os.path.join(exp, "results", "JPEG_par.exe_execution_times.json")))
    assert [e["image_size"] for e in res] == [2 ** i for i in range(12)]
    img = pngdec.read(str(tmp_path / "Assets/Images/rand_8X8.png"))       # last image
    coef = np.fromfile(tmp_path / "Output-Input/Images/coefficients.bin", dtype="<i2")
    assert np.array_equal(coef, oracle.jpeg_encode(img))


_VISUAL_SCRIPT = r"""
import ctypes, os, sys
import numpy as np
lib = ctypes.CDLL(sys.argv[1])
lib.ref_jpeg_visual_pngs.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
w, h = int(sys.argv[3]), int(sys.argv[4])
img = np.fromfile(sys.argv[2], dtype=np.uint8)
os.chdir(sys.argv[5])                     # OUTPUT_DIRECTORY is ../Output-Input/Images/
sys.exit(lib.ref_jpeg_visual_pngs(img.ctypes.data, w, h))
"""


@pytest.mark.skipif(not os.path.exists(os.path.join(REF, "libref_jpeg.so")),
                    reason="reference JPEG.c not built (no /root/reference at build time)")
@pytest.mark.parametrize("w,h", [(64, 48), (37, 21)])
def test_visual_pngs_equal_the_reference(tmp_path, oracle, w, h):
    """original / luminance / rChrominance / bChrominance.png decode to the
    pixels the reference's own create_*_image (JPEG.c:187-300, its
    double -> uint8_t conversions included) writes for the same image."""
    ours, ref = tmp_path / "ours", tmp_path / "ref"
    exp = layout(str(ours))
    layout(str(ref))
    img = oracle.rand_image(w, h, seed=9)
    pngdec.write(str(ours / "Assets/Images/rand_8X8.png"), img)
    assert run(exp, ["./JPEG_seq.exe"]).returncode == 0
    raw = tmp_path / "img.raw"
    np.ascontiguousarray(img).tofile(raw)
    import sys
    r = subprocess.run([sys.executable, "-c", _VISUAL_SCRIPT, os.path.join(REF, "libref_jpeg.so"),
                        str(raw), str(w), str(h), str(ref / "Experiment")],
                       capture_output=True, timeout=60)
    assert r.returncode == 0, r.stderr
    for name in ("original.png", "luminance.png", "rChrominance.png", "bChrominance.png"):
        a = pngdec.read(str(ours / "Output-Input/Images" / name))
        b = pngdec.read(str(ref / "Output-Input/Images" / name))
        assert np.array_equal(a, b), name
