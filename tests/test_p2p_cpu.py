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


@pytest.mark.parametrize("ranks", [1, 2, 3, 4])
def test_neighbor_collectives_host(ranks):
    """MPI_Neighbor_alltoallw (dist graph with self / repeated edges) and
    MPI_Neighbor_alltoallv (periodic Cartesian) through libtempi on host
    buffers, against oracle/typemap.c."""
    rc, out = mpi_launch.run(ranks, mpi_launch.py("neighbor.py"), timeout=180)
    assert rc == 0 and "RESULT errors=0" in out, out[-3000:]


@pytest.mark.parametrize("n", [1, 2])
def test_receive_status_host(n):
    """the status program on host buffers (library path end to end)"""
    rc, out = mpi_launch.run(n, mpi_launch.py("status.py"), timeout=180)
    assert rc == 0 and "RESULT errors=0" in out, out[-3000:]


@pytest.mark.parametrize("n", [1, 2])
def test_send_order_host(n):
    """the send-order program on host buffers (library path end to end)"""
    rc, out = mpi_launch.run(n, mpi_launch.py("order.py"), timeout=180)
    assert rc == 0 and "RESULT errors=0" in out, out[-3000:]


@pytest.mark.parametrize("n", [1, 2])
def test_persistent_and_send_modes_library(n):
    """persistent requests and the send modes with TEMPI inactive (no GPU):
    the library's, through the interposer unchanged"""
    rc, out = mpi_launch.run(n, mpi_launch.py("persistent.py"), timeout=180)
    assert rc == 0 and "RESULT errors=0" in out, out[-3000:]


def test_completion_family_host():
    """MPI_Testall/Testany/Waitany/Testsome/Waitsome/Request_free through the
    interposer with host buffers (library requests only)."""
    rc, out = mpi_launch.run(2, mpi_launch.py("completion.py"), timeout=180)
    assert rc == 0 and "RESULT errors=0" in out, out[-3000:]


@pytest.mark.parametrize("n,prog", [(2, ("p2p_world.py",)), (2, ("alltoallv.py", "--nnz", "2", "--scale", "100")),
                                    (1, ("neighbor.py",)), (3, ("neighbor.py",)), (1, ("status.py",)),
                                    (2, ("status.py",)), (1, ("order.py",)), (2, ("order.py",)),
                                    (2, ("completion.py",)), (1, ("probe_order.py",)), (2, ("probe_order.py",)),
                                    (1, ("persistent.py",)), (2, ("persistent.py",)),
                                    (2, ("fuzz.py", "3", "7", "--host")),
                                    (3, ("fuzz.py", "3", "11", "--modes", "--host")),
                                    (1, ("isend_self.py",)), (2, ("isend_self.py",))])
def test_tempi_host_paths_without_gpu(n, prog):
    """TEMPI's own host-side paths -- descriptor-aware host receives, the probe
    family and its held messages, send gates, host collectives -- which run
    only beside a GPU, forced on with TEMPI_TEST_HOST_ONLY (gpu.cpp) so that
    they are checked here too (probe_order at one rank is the program that
    hung on the GPU box in round 3: it relied on MPICH buffering a send to
    itself)"""
    rc, out = mpi_launch.run(n, mpi_launch.py(*prog), env={"TEMPI_TEST_HOST_ONLY": "1"}, timeout=180)
    assert rc == 0 and out.count("RESULT errors=0") >= 1 and "errors=" not in out.replace("errors=0", ""), out[-3000:]


def _torchrun(script, n, split=False):
    import os
    import socket
    import subprocess
    import sys

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(mpi_launch.ROOT, "tests", "mpi_progs", script)]
    env = dict(os.environ)
    for k in list(env):
        if k.startswith("PMI_"):
            env.pop(k)
    return subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE if split else subprocess.STDOUT,
                          text=True, timeout=240, env=env, start_new_session=True)


@pytest.mark.parametrize("n", [2, 3])
def test_bench_plumbing_under_torchrun(n):
    """bench.py's dist_setup / barrier / max-over-ranks timing reductions on
    gloo, and an MPI exchange between the torch-launched ranks it wires up;
    stdout, which carries the bench line, holds nothing of the setup's (gloo
    prints its connection messages there)"""
    r = _torchrun("torchrun_bench.py", n, split=True)
    assert r.returncode == 0 and r.stdout.count("RESULT ok") == n, (r.stdout + r.stderr)[-3000:]
    assert [l for l in r.stdout.splitlines() if l.strip() and not l.startswith("RESULT ok")] == [], r.stdout[-3000:]


def test_mpi_under_torchrun():
    """bench.py's multi-GPU launch is torch.distributed.run, not mpiexec: the
    ranks are wired into one MPI job by tempi_amd.pmi (PMI-1 server)."""
    import os
    import socket
    import subprocess
    import sys

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(mpi_launch.ROOT, "tests", "mpi_progs", "torchrun_mpi.py")]
    env = dict(os.environ)
    for k in list(env):
        if k.startswith("PMI_"):
            env.pop(k)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=240, env=env,
                       start_new_session=True)
    assert r.returncode == 0 and r.stdout.count("RESULT ok") == 2, r.stdout[-3000:]


@pytest.mark.parametrize("n,required,expect,env,extra", [
    (1, "SERIALIZED", "SERIALIZED", {"TEMPI_TEST_HOST_ONLY": "1"}, []),
    (2, "SERIALIZED", "SERIALIZED", {"TEMPI_TEST_HOST_ONLY": "1"}, []),
    (1, "FUNNELED", "FUNNELED", {"TEMPI_TEST_HOST_ONLY": "1"}, []),
    (1, "MULTIPLE", "MULTIPLE", {"TEMPI_TEST_HOST_ONLY": "1"}, ["--concurrent"]),
    (2, "MULTIPLE", "MULTIPLE", {"TEMPI_TEST_HOST_ONLY": "1"}, ["--concurrent"]),
    (2, "MULTIPLE", "MULTIPLE", {"TEMPI_TEST_HOST_ONLY": "1"}, []),
    (2, "MULTIPLE", "MULTIPLE", {"TEMPI_DISABLE": "1"}, ["--concurrent"])])
def test_thread_level_is_truthful(n, required, expect, env, extra):
    """the level MPI_Init_thread / MPI_Query_thread report
    is one TEMPI is safe at (the reference only logs it, /root/reference/src/
    init.cpp:36-46): MPI_THREAD_MULTIPLE when asked for -- TEMPI's calls then
    run under one lock that waits and blocking library calls give up
    (core/mt.hpp) -- and at most MPI_THREAD_SERIALIZED otherwise; the
    library's level when TEMPI is disabled. Then threads x 200 content-checked
    strided Isend / Irecv rounds: serialized under one application lock, or
    (--concurrent, 3 threads) with no lock, each thread blocked in MPI_Wait
    and MPI_Recv on messages other threads send"""
    threads = "3" if "--concurrent" in extra else "2"
    rc, out = mpi_launch.run(n, mpi_launch.py("threads.py", required, expect, threads, "200", *extra), env=env,
                             timeout=180)
    assert rc == 0 and out.count("RESULT errors=0") == n, out[-3000:]


@pytest.mark.parametrize("n", [1, 2])
def test_many_requests_in_flight(n):
    """6 000 receives + 6 000 sends in flight per rank, completed in a
    scrambled order by MPI_Wait / MPI_Test, twice: the direct-mapped request
    table (core/p2p.cpp) grows past its first 4 096 slots and reuses handles,
    every handle distinct while in flight, every byte checked"""
    rc, out = mpi_launch.run(n, mpi_launch.py("manyreq.py", "6000"), env={"TEMPI_TEST_HOST_ONLY": "1"}, timeout=180)
    assert rc == 0 and out.count("RESULT errors=0") == n, out[-3000:]
