"""ASan + UBSan run of the host C (lz4r_decode.c, png_io.c, synth.c) and the
oracle restatements: tests/sanitize/sanitize_main.c built by
`make sanitize`, no GPU needed."""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_host_c_and_oracle_under_asan_ubsan(tmp_path):
    subprocess.run(["make", "-C", REPO, "sanitize"], check=True, capture_output=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(REPO, "build", "sanitize_main"),
                        os.path.join(REPO, "tests", "golden"), str(tmp_path)],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "sanitize ok" in r.stdout
