"""Multi-rank GPU transfers through libtempi.so (mpiexec, ranks share the
box's GPU(s)): every method of the strided Send/Recv/Isend/Irecv path, the
strided ping-pong app (config 3) and the 3D halo exchange app (config 4),
all with byte-exact content checks."""
import json
import os

import pytest

from tests import mpi_launch

pytestmark = pytest.mark.gpu

LIB = os.path.join(mpi_launch.ROOT, "tempi_amd", "lib")
METHODS = {
    "AUTO": {},
    "ONESHOT": {"TEMPI_DATATYPE_ONESHOT": "1"},
    "STAGED": {"TEMPI_DATATYPE_STAGED": "1"},
    "IPC": {"TEMPI_DATATYPE_IPC": "1"},
    "DEVICE": {"TEMPI_DATATYPE_DEVICE": "1"},  # no GPU-aware MPI here: IPC intra-node
    # IPC whose peer mapping fails (fault injection): NACK -> host re-send
    "IPC_FAULT": {"TEMPI_DATATYPE_IPC": "1", "TEMPI_FAULT_IPC_OPEN": "1"},
    # IPC COPY for every size and row width (the receiver copies out of the sender's object)
    "XCOPY": {"TEMPI_DATATYPE_IPC": "1", "TEMPI_IPC_COPY_MIN_BYTES": "1", "TEMPI_IPC_COPY_MIN_BLOCK": "1"},
}


def _kv_line(out, prefix):
    """(line, {key: value}) of the key=value line a rank printed after `prefix`;
    the pairs end at the first token without '=' (another rank's output can
    land on the same line before its newline)"""
    line = next(l for l in out.splitlines() if l.startswith(prefix))
    kv = {}
    for tok in line[len(prefix):].split():
        if "=" not in tok:
            break
        k, v = tok.split("=", 1)
        kv[k] = v
    return line, kv


def _json_line(out):
    for line in out.splitlines():
        if line.startswith("{"):
            return json.loads(line)
    raise AssertionError(out[-3000:])


@pytest.mark.parametrize("method", list(METHODS))
def test_p2p_world_device(gpu, method):
    rc, out = mpi_launch.run(2, mpi_launch.py("p2p_world.py", "--device"), env=METHODS[method], timeout=240)
    assert rc == 0 and "RESULT errors=0" in out, out[-4000:]


@pytest.mark.parametrize("method", list(METHODS))
@pytest.mark.parametrize("total,block", [(1024, 1), (1024, 8), (1 << 20, 1), (1 << 20, 16), (4 << 20, 256),
                                         (4 << 20, 512)])
def test_pingpong_nd(gpu, method, total, block):
    rc, out = mpi_launch.run(2, [os.path.join(LIB, "pingpong_nd"), "5", str(total), str(block), "--check"],
                             env=METHODS[method], timeout=240)
    r = _json_line(out)
    assert rc == 0 and r["errors"] == 0, out[-3000:]


@pytest.mark.parametrize("ranks,grid,env,extra", [
    (1, "48", {}, []), (2, "48", {}, []), (4, "40", {}, []), (3, "30", {}, []), (1, "128", {}, []),
    (1, "48", {"TEMPI_NO_SELF_CHANNEL": "1"}, []), (2, "48", {"TEMPI_NO_SELF_CHANNEL": "1"}, []),
    (1, "48", {"TEMPI_NO_DIRECT": "1"}, []), (2, "40", {"TEMPI_FAULT_IPC_OPEN": "1"}, []),
    (4, "32", {"TEMPI_DATATYPE_ONESHOT": "1"}, []),
    (1, "48", {}, ["--neighbor"]), (2, "40", {}, ["--neighbor"]), (4, "32", {}, ["--neighbor"]),
    (3, "30", {}, ["--neighbor"]),
    # x split (the 24-byte faces cross ranks, as at 8 ranks on (2, 2, 2))
    (2, "64 16 16", {}, []), (4, "64 64 16", {}, []), (4, "64 64 16", {}, ["--neighbor"]),
    (4, "64 64 16", {"TEMPI_DATATYPE_STAGED": "1"}, []),
    # ranks sharing this box's one GPU get one stream lane; force the
    # multi-lane configuration of one rank per GPU (scatters on lanes 1-3)
    (2, "40", {"TEMPI_STREAMS": "4"}, []), (4, "64 64 16", {"TEMPI_STREAMS": "3"}, []),
    (4, "32", {"TEMPI_STREAMS": "3"}, ["--neighbor"]), (2, "40", {"TEMPI_STREAMS": "3", "TEMPI_NO_DIRECT": "1"}, []),
    (1, "48", {"TEMPI_STREAMS": "1"}, []),
    # IPC COPY: wide rows only (the default row limit), every row, with lanes, unmappable
    (2, "40", {"TEMPI_IPC_COPY_MIN_BYTES": "1"}, []),
    (4, "64 64 16", {"TEMPI_IPC_COPY_MIN_BYTES": "1", "TEMPI_IPC_COPY_MIN_BLOCK": "1"}, []),
    (2, "40", {"TEMPI_IPC_COPY_MIN_BYTES": "1", "TEMPI_IPC_COPY_MIN_BLOCK": "1", "TEMPI_STREAMS": "3"}, []),
    (2, "40", {"TEMPI_IPC_COPY_MIN_BYTES": "1", "TEMPI_FAULT_IPC_OPEN": "1"}, []),
    (4, "32", {"TEMPI_IPC_COPY_MIN_BYTES": "1", "TEMPI_IPC_COPY_MIN_BLOCK": "1"}, ["--neighbor"]),
    # 8 ranks on (2, 2, 2), the decomposition of the driver's 8-GPU node, with
    # the stream lanes one rank per GPU gets (3)
    (8, "64", {}, []), (8, "64", {}, ["--neighbor"]), (8, "64", {"TEMPI_STREAMS": "3"}, []),
    (8, "48", {"TEMPI_STREAMS": "3"}, ["--neighbor"]),
    (8, "64", {"TEMPI_IPC_COPY_MIN_BYTES": "1", "TEMPI_IPC_COPY_MIN_BLOCK": "1", "TEMPI_STREAMS": "3"}, []),
    # every rank sees the GPU under an identity of its own: the cross-GPU
    # paths (system-scope loads, first-contact canary) between ranks of one GPU
    (4, "64 64 16", {"TEMPI_FAKE_FOREIGN_GPU": "1"}, []),
    (8, "64", {"TEMPI_FAKE_FOREIGN_GPU": "1", "TEMPI_STREAMS": "3"}, []),
    (2, "40", {"TEMPI_FAKE_FOREIGN_GPU": "1", "TEMPI_IPC_COPY_MIN_BYTES": "1", "TEMPI_IPC_COPY_MIN_BLOCK": "1"}, []),
    (4, "64 64 16", {"TEMPI_FAKE_FOREIGN_GPU": "1", "TEMPI_FAULT_CANARY": "1"}, []),
    # rank placement (MPI_Dist_graph_create_adjacent, reorder = 1) over two
    # fake nodes: every rank plays the rank it is given
    (8, "48", {"TEMPI_PLACEMENT_KAHIP": "", "TEMPI_FAKE_NODE_SIZE": "4"}, ["--reorder"]),
    (8, "48", {"TEMPI_PLACEMENT_KAHIP": "", "TEMPI_FAKE_NODE_SIZE": "4", "TEMPI_STREAMS": "3"},
     ["--reorder", "--neighbor"]),
    (4, "64 64 16", {"TEMPI_PLACEMENT_RANDOM": "", "TEMPI_FAKE_NODE_SIZE": "2"}, ["--reorder"])])
def test_halo_exchange_content(gpu, ranks, grid, env, extra):
    rc, out = mpi_launch.run(ranks, [os.path.join(LIB, "halo_exchange"), "2"] + grid.split() + ["--quants", "2", "--check"] + extra,
                             env=env, timeout=300)
    r = _json_line(out)
    assert rc == 0 and r["checked"] and r["errors"] == 0, out[-3000:]


@pytest.mark.parametrize("ranks,env", [(1, {}), (2, {}), (4, {"TEMPI_FAKE_FOREIGN_GPU": "1"}),
                                       (8, {"TEMPI_STREAMS": "3"})])
def test_halo_exchange_512_full_check(gpu, ranks, env):
    """config 4 at its full size, 8 quantities: every cell of every quantity
    checked (on the GPU), at 1 rank and in the 2-, 4- and 8-rank
    decompositions (the full-size faces through IPC COPY, slabs and the
    cross-GPU load path)"""
    rc, out = mpi_launch.run(ranks, [os.path.join(LIB, "halo_exchange"), "2", "512", "--check"], env=env,
                             timeout=240)
    r = _json_line(out)
    assert rc == 0 and r["checked"] and r["errors"] == 0 and r["global"] == [512, 512, 512], out[-3000:]
    # the GPU's busy time by TEMPI's account (counters.ns_gpu_inflight): some
    # of every iteration, never more than the iteration
    busy = r["rank0_us_per_iter"]["gpu_inflight"]
    assert 0 < busy <= r["us_per_iter"] * 1.05, r


def test_halo_check_finds_a_planted_error(gpu):
    """negative control: the GPU check counts one corrupted halo cell"""
    rc, out = mpi_launch.run(2, [os.path.join(LIB, "halo_exchange"), "1", "32", "--quants", "2", "--check-control"],
                             timeout=120)
    r = _json_line(out)
    assert r["checked"] and r["errors"] == 1, out[-3000:]


A2AV = {"AUTO": {}, "STAGED": {"TEMPI_ALLTOALLV_STAGED": "1"}, "ISIR_STAGED": {"TEMPI_ALLTOALLV_ISIR_STAGED": "1"},
        "ISIR_REMOTE_STAGED": {"TEMPI_ALLTOALLV_ISIR_REMOTE_STAGED": "1"}}


@pytest.mark.parametrize("method", list(A2AV))
@pytest.mark.parametrize("ranks,scale,nnz", [(2, 100000, 2), (4, 1000, 3), (3, 10, 1)])
def test_alltoallv_device(gpu, method, ranks, scale, nnz):
    rc, out = mpi_launch.run(ranks, mpi_launch.py("alltoallv.py", "--device", "--scale", str(scale), "--nnz",
                                                  str(nnz)), env=A2AV[method], timeout=240)
    assert rc == 0 and "RESULT errors=0" in out, out[-3000:]


@pytest.mark.parametrize("mixed", ["alt", "hostrank"])
@pytest.mark.parametrize("ranks,scale", [(2, 100000), (3, 1000), (4, 10)])
def test_alltoallv_mixed_host_device(gpu, mixed, ranks, scale):
    """ranks whose blocks are in different memories (host / device) still
    meet: every rank takes TEMPI's route, host receives land descriptors"""
    rc, out = mpi_launch.run(ranks, mpi_launch.py("alltoallv.py", "--device", "--scale", str(scale), "--nnz", "3",
                                                  "--mixed", mixed), timeout=240)
    assert rc == 0 and "RESULT errors=0" in out, out[-3000:]


@pytest.mark.parametrize("n,method", [(2, "AUTO"), (1, "AUTO"), (2, "XCOPY"), (2, "IPC"), (2, "ONESHOT"),
                                      (2, "STAGED"), (1, "NO_DIRECT"), (2, "IPC_FAULT")])
def test_every_receive_sees_payload(gpu, n, method):
    """a device strided send (ONESHOT / IPC slab / IPC COPY / DIRECT) received
    by host MPI_Irecv, MPI_Probe + MPI_Recv, MPI_Iprobe, MPI_Mprobe + MPI_Mrecv
    (host and device), MPI_Improbe + MPI_Imrecv, MPI_Sendrecv: payload bytes
    and counts exact; then MPI_ERR_TRUNCATE from every receive kind"""
    env = dict(METHODS.get(method, {}))
    if method == "NO_DIRECT":
        env["TEMPI_NO_DIRECT"] = "1"
    rc, out = mpi_launch.run(n, mpi_launch.py("anyrecv.py"), env=env, timeout=240)
    assert rc == 0 and "RESULT errors=0" in out, out[-4000:]
    if n == 2 and method == "AUTO":  # the routes the cases are named for were taken
        line, c = _kv_line(out, "rank 0 counters")
        assert int(c["ipc"]) > 0 and int(c["ipc_copy"]) > 0 and int(c["oneshot"]) > 0, line


@pytest.mark.parametrize("n,device", [(1, False), (2, False), (1, True), (2, True)])
def test_probe_keeps_non_overtaking(gpu, n, device):
    """a probe that must receive a descriptor-sized message to look at it
    keeps the sender's earlier messages too, so a later MPI_ANY_TAG receive
    still gets them in send order; MPI_Improbe / MPI_Mrecv and
    MPI_Sendrecv_replace after a probe likewise"""
    rc, out = mpi_launch.run(n, mpi_launch.py("probe_order.py", *(["--device"] if device else [])), timeout=180)
    assert rc == 0 and "RESULT errors=0" in out, out[-3000:]


@pytest.mark.parametrize("fault", [False, True])
@pytest.mark.parametrize("method", ["AUTO", "XCOPY"])
def test_cross_gpu_first_contact_canary(gpu, method, fault):
    """a peer that looks like another GPU (TEMPI_FAKE_FOREIGN_GPU) is read
    through the remote-load kernel only after its first descriptor's bytes
    read back the same through that kernel and through DMA; a mismatch
    (TEMPI_FAULT_CANARY) turns IPC with it off and the bytes still arrive"""
    env = dict(METHODS[method], TEMPI_FAKE_FOREIGN_GPU="1")
    if fault:
        env["TEMPI_FAULT_CANARY"] = "1"
    rc, out = mpi_launch.run(2, mpi_launch.py("anyrecv.py"), env=env, timeout=240)
    assert rc == 0 and "RESULT errors=0" in out, out[-4000:]
    line, c = _kv_line(out, "rank 1 counters")
    assert (int(c["canary_ok"]), int(c["canary_fail"])) == ((0, 1) if fault else (1, 0)), line


@pytest.mark.parametrize("ranks,env", [(1, {}), (2, {}), (3, {}), (4, {}), (2, {"TEMPI_DATATYPE_ONESHOT": "1"}),
                                       (3, {"TEMPI_NO_DIRECT": "1"})])
def test_neighbor_collectives_device(gpu, ranks, env):
    """MPI_Neighbor_alltoallw / _alltoallv on device buffers: TEMPI's per-edge
    route, checked against the oracle and the library's own result on host
    copies."""
    rc, out = mpi_launch.run(ranks, mpi_launch.py("neighbor.py", "--device"), env=env, timeout=240)
    assert rc == 0 and "RESULT errors=0" in out, out[-3000:]


@pytest.mark.parametrize("ranks,scale,density,env", [
    (2, 100000, 1.0, {}), (3, 1000, 0.5, {}), (4, 10, 1.0, {}), (4, 100000, 0.25, {}), (2, 1000000, 1.0, {}),
    (3, 10000, 1.0, {}),
    # 8 ranks, config 5's own rank count: the reference's scales x densities
    # (bench_alltoallv_random_sparse.cpp:140-222), and the 3 lanes of one rank per GPU
    (8, 1, 1.0, {}), (8, 100, 0.5, {}), (8, 10000, 0.125, {}), (8, 100000, 0.05, {}), (8, 1000000, 0.25, {}),
    (8, 10, 1.0, {"TEMPI_STREAMS": "3"}), (8, 100000, 0.5, {"TEMPI_STREAMS": "3"}),
    (8, 1000000, 1.0, {"TEMPI_STREAMS": "3"})])
def test_alltoallv_sparse_app(gpu, ranks, scale, density, env):
    """config 5 app: the reference's random sparse matrices, every byte checked"""
    rc, out = mpi_launch.run(ranks, [os.path.join(LIB, "alltoallv_sparse"), "3", "--scale", str(scale), "--density",
                                     str(density), "--check"], env=env, timeout=240)
    r = _json_line(out)
    assert rc == 0 and r["checked"] and r["errors"] == 0, out[-3000:]


@pytest.mark.parametrize("ranks,env", [(2, {}), (4, {}), (2, {"TEMPI_CONTIGUOUS_STAGED": "1"}), (4, METHODS["XCOPY"]),
                                       (2, {"TEMPI_DATATYPE_ONESHOT": "1"}), (8, {"TEMPI_STREAMS": "3"})])
def test_pingpong_1d_app(gpu, ranks, env):
    """the reference's bench_mpi_pingpong_1d on device buffers (MPI_BYTE,
    all pairs at once), every byte checked, small and large"""
    rc, out = mpi_launch.run(ranks, [os.path.join(LIB, "pingpong_1d"), "3", "1", "4096", str(1 << 21), str(1 << 24),
                                     "--check"], env=env, timeout=240)
    recs = [json.loads(l) for l in out.splitlines() if l.startswith("{")]
    assert rc == 0 and len(recs) == 4 and all(r["errors"] == 0 and r["buffers"] == "device" for r in recs), out[-3000:]


@pytest.mark.parametrize("env", [{}, {"TEMPI_CONTIGUOUS_STAGED": "1"}, METHODS["XCOPY"], {"TEMPI_DATATYPE_ONESHOT": "1"}])
def test_mpi_isend_app(gpu, env):
    """the reference's bench_mpi_isend on device buffers: 10 overlapping
    contiguous messages each way, 1 B to 1 MiB, every byte checked"""
    rc, out = mpi_launch.run(2, [os.path.join(LIB, "mpi_isend"), "3", "1", "64", "4096", "65536", str(1 << 20),
                                 "--check"], env=env, timeout=240)
    recs = [json.loads(l) for l in out.splitlines() if l.startswith("{")]
    assert rc == 0 and len(recs) == 5 and all(r["errors"] == 0 and r["buffers"] == "device" for r in recs), out[-3000:]


@pytest.mark.parametrize("ranks,scale,density,env", [
    (2, 100000, 1.0, {}), (4, 1000, 0.5, {}), (3, 10, 1.0, {"TEMPI_DATATYPE_ONESHOT": "1"}),
    (8, 1, 1.0, {}), (8, 100000, 0.5, {}), (8, 1000000, 0.125, {"TEMPI_STREAMS": "3"}),
    # the reference's KaHIP remapping, over two fake nodes of 4 ranks
    (8, 1000, 0.5, {"TEMPI_PLACEMENT_KAHIP": "", "TEMPI_FAKE_NODE_SIZE": "4"}),
    (8, 100000, 1.0, {"TEMPI_PLACEMENT_METIS": "", "TEMPI_FAKE_NODE_SIZE": "2", "TEMPI_FAKE_FOREIGN_GPU": "1"})])
def test_nbr_alltoallv_sparse_app(gpu, ranks, scale, density, env):
    """config 5's neighbourhood form (bench_nbr_alltoallv_random_sparse.cpp:
    distributed graph with reorder = 1, MPI_Neighbor_alltoallv of device
    buffers), every byte checked"""
    rc, out = mpi_launch.run(ranks, [os.path.join(LIB, "alltoallv_sparse"), "3", "--scale", str(scale), "--density",
                                     str(density), "--check", "--neighbor"], env=env, timeout=240)
    r = _json_line(out)
    assert rc == 0 and r["checked"] and r["errors"] == 0 and r["buffers"] == "device", out[-3000:]


@pytest.mark.parametrize("n", [1, 2])
@pytest.mark.parametrize("method", ["AUTO", "ONESHOT", "STAGED"])
def test_isend_self_reference(gpu, n, method):
    """the reference's isend.cu / isend_contiguous.cu: send to self, then
    receive, waiting on the send first; host and device, bytes checked"""
    rc, out = mpi_launch.run(n, mpi_launch.py("isend_self.py", "--device"), env=METHODS[method], timeout=180)
    assert rc == 0 and "RESULT errors=0" in out, out[-3000:]


@pytest.mark.parametrize("method", ["AUTO", "ONESHOT", "IPC", "STAGED", "XCOPY"])
def test_completion_family_device(gpu, method):
    """TEMPI device requests mixed with library requests through
    MPI_Testall / Testany / Waitany / Testsome / Waitsome / Request_free"""
    rc, out = mpi_launch.run(2, mpi_launch.py("completion.py", "--device"), env=METHODS[method], timeout=240)
    assert rc == 0 and "RESULT errors=0" in out, out[-3000:]


@pytest.mark.parametrize("env", [METHODS["XCOPY"], dict(METHODS["XCOPY"], TEMPI_FAULT_IPC_OPEN="1"),
                                 dict(METHODS["XCOPY"], TEMPI_STREAMS="3"),
                                 dict(METHODS["XCOPY"], TEMPI_FAKE_FOREIGN_GPU="1")],
                         ids=["copy", "unmapped", "lanes", "foreign"])
def test_ipc_copy_receivers(gpu, env):
    """IPC COPY against every receiver: same and other strided shapes (copy
    kernel), a receive type too deep for it and a host receive (the sender
    gathers and re-sends through the host), a blocking receive, and one send
    buffer rewritten and re-sent (no stale bytes through the peer mapping)"""
    rc, out = mpi_launch.run(2, mpi_launch.py("xcopy.py"), env=env, timeout=120)
    assert rc == 0 and "RESULT errors=0" in out, out[-3000:]
    if "TEMPI_FAULT_IPC_OPEN" not in env:
        assert "rank 0 counters ipc_copy=16 resends=2" in out, out[-3000:]


@pytest.mark.parametrize("n,method", [(2, "AUTO"), (2, "ONESHOT"), (2, "IPC"), (2, "STAGED"), (1, "AUTO"),
                                      (1, "NO_DIRECT"), (2, "XCOPY")])
def test_receive_status_and_freed_types(gpu, n, method):
    """MPI_Status source / tag / MPI_Get_count of device receives (fewer
    elements than allowed), with both datatypes freed before the wait"""
    env = dict(METHODS.get(method, {}))
    if method == "NO_DIRECT":
        env["TEMPI_NO_DIRECT"] = "1"
    rc, out = mpi_launch.run(n, mpi_launch.py("status.py", "--device"), env=env, timeout=240)
    assert rc == 0 and "RESULT errors=0" in out, out[-3000:]


@pytest.mark.parametrize("n,method", [(2, "AUTO"), (2, "ONESHOT"), (2, "IPC"), (2, "STAGED"), (1, "AUTO"),
                                      (1, "NO_DIRECT"), (2, "LANES"), (2, "XCOPY")])
def test_send_order_across_routes(gpu, n, method):
    """MPI non-overtaking: a gathered strided send, a host send, a
    library-packed irregular send and another strided send to one peer with
    one tag are matched in call order (a blocking host send behind them too)"""
    env = dict(METHODS.get(method, {}))
    if method == "NO_DIRECT":
        env["TEMPI_NO_DIRECT"] = "1"
    if method == "LANES":
        env["TEMPI_STREAMS"] = "3"
    rc, out = mpi_launch.run(n, mpi_launch.py("order.py", "--device"), env=env, timeout=240)
    assert rc == 0 and "RESULT errors=0" in out, out[-3000:]


@pytest.mark.parametrize("n,env", [(1, {}), (2, {}), (1, {"TEMPI_NO_SELF_CHANNEL": "1"}), (1, {"TEMPI_NO_DIRECT": "1"}),
                                   (1, {"TEMPI_STREAMS": "3"})])
def test_self_channel(gpu, n, env):
    """messages of a process to itself matched inside TEMPI: earliest send /
    earliest receive / MPI_ANY_TAG, and the spill to the library on a host
    send, an MPI_ANY_SOURCE receive, a probe, an MPI_Issend, a cancel"""
    rc, out = mpi_launch.run(n, mpi_launch.py("selfchan.py"), env=env, timeout=200)
    assert rc == 0 and "RESULT errors=0" in out, out[-4000:]


@pytest.mark.parametrize("n,seed,env", [(1, 7, {}), (2, 7, {}), (3, 11, {}), (4, 5, {}),
                                        (1, 23, {"TEMPI_NO_SELF_CHANNEL": "1"}), (2, 29, {"TEMPI_NO_SELF_CHANNEL": "1"}),
                                        (3, 13, {"TEMPI_STREAMS": "3"}), (2, 17, {"TEMPI_NO_IPC_COPY": "1"}),
                                        (2, 19, {"TEMPI_NO_DIRECT": "1"})])
def test_transport_fuzz(gpu, n, seed, env):
    """random mixes of every route (direct, IPC slab, IPC COPY, ONESHOT,
    library-packed, host) between all pairs incl. self, tags reused so MPI
    order matters, random posting interleavings; every byte checked"""
    rc, out = mpi_launch.run(n, mpi_launch.py("fuzz.py", "5", str(seed)), env=env, timeout=200)
    assert rc == 0 and "RESULT errors=0" in out, out[-3000:]


@pytest.mark.parametrize("method", ["TEMPI_PLACEMENT_KAHIP", "TEMPI_PLACEMENT_RANDOM"])
def test_placement_device(gpu, method):
    """the placement program with a strided device type along every edge of
    the placed communicator (TEMPI's transport), bytes against the oracle"""
    rc, out = mpi_launch.run(8, mpi_launch.py("placement.py", "--device"),
                             env={method: "", "TEMPI_FAKE_NODE_SIZE": "4"}, timeout=240)
    assert rc == 0 and "RESULT errors=0" in out, out[-3000:]


@pytest.mark.parametrize("n,method", [(1, "AUTO"), (2, "AUTO"), (2, "ONESHOT")])
def test_serialized_threads_device(gpu, n, method):
    """MPI_Init_thread(SERIALIZED) under TEMPI: two application threads take
    turns with strided device-object Isend / Irecv / Test (each thread's
    requests in flight while the other thread calls in), 300 rounds each,
    every byte checked"""
    rc, out = mpi_launch.run(n, mpi_launch.py("threads.py", "SERIALIZED", "SERIALIZED", "2", "300", "--device"),
                             env=METHODS[method], timeout=240)
    assert rc == 0 and out.count("RESULT errors=0") == n, out[-3000:]


@pytest.mark.parametrize("n,method", [(1, "AUTO"), (2, "AUTO"), (2, "ONESHOT"), (2, "IPC")])
def test_multiple_threads_device(gpu, n, method):
    """MPI_Init_thread(MULTIPLE) under TEMPI provides MPI_THREAD_MULTIPLE
    (core/mt.hpp): three threads with no application lock, each blocking in
    MPI_Wait on a strided device message another thread sends and in a host
    MPI_Recv, 200 rounds each, every byte checked -- a lock kept through a
    wait would deadlock (the test's timeout)"""
    rc, out = mpi_launch.run(n, mpi_launch.py("threads.py", "MULTIPLE", "MULTIPLE", "3", "200", "--device",
                                              "--concurrent"), env=METHODS[method], timeout=240)
    assert rc == 0 and out.count("RESULT errors=0") == n, out[-3000:]


def test_measure_system_writes_a_model_auto_uses(gpu, tmp_path):
    """VERDICT r04 next 2 (row a12): apps/measure_system --quick at 2 ranks
    (the perf.json writer, /root/reference/src/internal/measure_system.cu:
    377-606) writes the reference's schema with finite, positive, IID-flagged
    times -- d2h / h2d / both intra-node ping-pongs over 2^0 .. 2^20 bytes,
    packDevice / unpackDevice / packHost / unpackHost rows of 2^(2i+6) bytes x
    2^j-byte blocks, the launch time with sub-microsecond digits -- and a
    fresh process given that TEMPI_CACHE_DIR loads it and has AUTO price
    blocking sends with it"""
    from tests import perf_json_check

    out = tmp_path / "perf.json"
    rc, log = mpi_launch.run(2, [os.path.join(LIB, "measure_system"), "--quick", "--out", str(out)], timeout=240)
    assert rc == 0 and '"gpu": true' in log, log[-3000:]
    doc, bad = perf_json_check.check(str(out), gpu=True)
    assert not bad, bad[:10]
    rc, log = mpi_launch.run(1, mpi_launch.py("perf_pick.py"), env={"TEMPI_CACHE_DIR": str(tmp_path)}, timeout=120)
    assert rc == 0, log[-3000:]
    pick = json.loads(next(l for l in log.splitlines() if l.startswith("{")))
    assert pick["loaded"] == 1 and pick["source"] == str(out), pick
    colocated = [p for p in pick["picks"] if p[1] == 1]
    assert all(fm == 1 and m in (1, 3, 4) for _, _, m, fm in colocated), pick  # ONESHOT / STAGED / IPC, priced


def test_multiple_threads_probe_holds_a_waited_message(gpu):
    """at MPI_THREAD_MULTIPLE, thread A blocks in a host
    MPI_Recv(0, tag A) while thread B's MPI_Probe(0, tag B) finds a strided
    device message (a descriptor) that rank 0 sent right behind A's message:
    the probe must receive A's message to look at B (non-overtaking) and
    keeps it, and A's receive must take it from what is kept instead of
    asking the library forever. 100 rounds, every byte checked; a hang is
    the join timing out."""
    rc, out = mpi_launch.run(2, mpi_launch.py("probe_threads.py", "100"), timeout=240)
    assert rc == 0 and out.count("RESULT errors=0") == 2, out[-3000:]
