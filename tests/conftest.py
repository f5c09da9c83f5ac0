import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _ensure_built():
    """Build the native extension / CLI / host test binary in-tree if missing (fresh checkout)."""
    need = [os.path.join(ROOT, "bin", "mcg-cg"), os.path.join(ROOT, "build", "test_host")]
    import glob

    if not glob.glob(os.path.join(ROOT, "cuda_mpi_parallel_amd", "_C*.so")) or not all(map(os.path.exists, need)):
        subprocess.run(["make", "-C", ROOT, "-j8", f"PYTHON={sys.executable}"], check=True,
                       stdout=subprocess.DEVNULL)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run via gpurun)")
    config.addinivalue_line("markers", "slow: long-running")
    _ensure_built()


@pytest.fixture(scope="session")
def mcg():
    import cuda_mpi_parallel_amd as m

    m.native()
    return m


@pytest.fixture(scope="session")
def C(mcg):
    return mcg.native()
