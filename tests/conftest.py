import os
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


# The hot path's parity evidence (MPICH goldens, library MPI_Pack, full-size
# exact checks) runs before anything else, so that under `pytest -x` a failure
# in a transport or tool test can never hide it (round 3: one NameError in a
# fuzz script stopped the run before test_pack_gpu.py was reached).
FIRST = ("test_oracle.py", "test_pack_gpu.py", "test_fuzz_parity.py", "test_dense_gpu.py", "test_direct_gpu.py")


def pytest_collection_modifyitems(session, config, items):
    def rank(item):
        name = os.path.basename(str(item.fspath))
        return FIRST.index(name) if name in FIRST else len(FIRST)

    items[:] = sorted(items, key=rank)  # (stable: file order kept inside each group)


@pytest.fixture(scope="session")
def mpi():
    """MPI initialised (singleton) through libtempi.so for the whole session."""
    import tempi_amd

    m = tempi_amd.get_mpi()
    m.Init()
    yield m
    m.Finalize()


def _gpu_available():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu(mpi):
    """A GPU is required: fail loudly (not skip) when a gpu-marked test finds none."""
    import torch

    assert torch.cuda.is_available(), "gpu test on a machine without a GPU"
    torch.cuda.init()
    assert mpi.gpu_available(), "libtempi found no GPU at MPI_Init"
    return torch.device("cuda", 0)
