import os
import subprocess
import sys

import pytest

# The library reads its test hooks (CASK_SCAN_MODE, CASK_HOST_THREADS, ... : cask_amd/csrc/knobs.h)
# only under this switch, fixed when it is first used; child processes of the tests inherit it.
os.environ.setdefault("CASK_TEST_HOOKS", "1")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP extension)")


def _make(dirpath: str):
    subprocess.run(["make", "-s", "-j8"], cwd=dirpath, check=True)


@pytest.fixture(scope="session")
def oracle_lib():
    """The C oracle (test infrastructure only)."""
    import oracle_ffi
    if not os.path.exists(oracle_ffi.LIB_PATH):
        _make(os.path.join(ROOT, "oracle"))
    return oracle_ffi.load()


@pytest.fixture(scope="session")
def native():
    """The product library. Built in-tree if absent (hipcc cross-compiles without a GPU).
    CASK_TEST_LIB (tools only: checking an A/B variant build before it becomes the product) runs
    the suite on another build of the library."""
    import cask_amd
    if os.environ.get("CASK_TEST_LIB"):
        cask_amd._lib.use_library(os.environ["CASK_TEST_LIB"])
    elif not os.path.exists(cask_amd.LIB_PATH):
        _make(os.path.join(ROOT, "cask_amd"))
    return cask_amd.lib()


def golden_cases():
    return sorted(d for d in os.listdir(GOLDEN)
                  if os.path.isdir(os.path.join(GOLDEN, d)) and not d.startswith("__"))


@pytest.fixture(scope="session")
def gpu_ctx(native):
    from cask_amd import ScanContext
    return ScanContext(0)
