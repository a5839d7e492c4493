import os
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


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
