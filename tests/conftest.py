import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(REPO, "lz4-jpeg_amd")
if PKG_DIR not in sys.path:
    sys.path.insert(0, PKG_DIR)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)

LIB = os.path.join(PKG_DIR, "lz4jpeg", "liblz4jpeg.so")
ORACLE = os.path.join(REPO, "oracle", "liboracle.so")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")
    config.addinivalue_line("markers", "slow: long-running (full-size) test")


def _ensure_built():
    if os.path.exists(LIB) and os.path.exists(ORACLE):
        return
    # in the build container (no prebuilt artefacts yet): build everything
    subprocess.run(["make", "-C", REPO, "-j8"], check=True,
                   stdout=subprocess.DEVNULL, stderr=subprocess.STDOUT)


_ensure_built()


@pytest.fixture(scope="session")
def oracle():
    import oracle_api
    return oracle_api.load()


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
