"""World-size-2 point-to-point through the interposer on CPU (host buffers:
TEMPI forwards to the library). Exercises MPI_Init through libtempi, the
topology allgather, MPI_Send/Recv/Isend/Irecv/Wait/Waitall/Test routing and
request handling with mixed datatypes, in two real MPI processes."""
import pytest

from tests import mpi_launch


def test_two_ranks_host_buffers():
    rc, out = mpi_launch.run(2, mpi_launch.py("p2p_world.py"), timeout=180)
    assert rc == 0 and "RESULT errors=0" in out, out[-3000:]


@pytest.mark.parametrize("ranks,nnz", [(2, 2), (3, 1), (4, 3)])
def test_alltoallv_host(ranks, nnz):
    rc, out = mpi_launch.run(ranks, mpi_launch.py("alltoallv.py", "--nnz", str(nnz), "--scale", "100"), timeout=180)
    assert rc == 0 and "RESULT errors=0" in out, out[-3000:]
