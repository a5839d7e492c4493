"""Run under mpiexec -n 8 with TEMPI_FAKE_NODE_SIZE=4 (two "nodes" of four
ranks, for placement only) and TEMPI_PLACEMENT_KAHIP or TEMPI_PLACEMENT_RANDOM:
rank placement in MPI_Dist_graph_create_adjacent(reorder = 1)
(/root/reference/src/dist_graph_create_adjacent.cpp:55-470).

The graph: every rank has heavy edges (weight 100) to the ranks two away
(+-2: a ring over each parity) and a light edge (weight 1) to the next rank.
Library order puts ranks 0-3 on node 0 and 4-7 on node 1, cutting heavy
edges; the best split puts one parity on each node. Checked:
  1. the new ranks are a permutation, and the new communicator is in
     application order (an Allgather over it returns 0..n-1);
  2. MPI_Dist_graph_neighbors gives application rank q the edges (and
     weights) old rank q passed, as the reference's placement does;
  3. the partitioner (KAHIP) puts one parity on each fake node and lowers the
     edge cut; RANDOM keeps the nodes' sizes;
  4. messages on the new communicator reach the application ranks they name:
     MPI_Isend / MPI_Irecv along every edge and MPI_Neighbor_alltoallv, with
     host ints, and with --device a strided device type through TEMPI's
     transport, bytes checked against the oracle;
  5. reorder = 0, or one node (TEMPI_FAKE_NODE_SIZE = n), leaves ranks alone.
"""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)

import tempi_amd  # noqa: E402

device = "--device" in sys.argv
mpi = tempi_amd.get_mpi()
if device:
    import torch

    torch.cuda.set_device(0)
mpi.Init()
rank, n = mpi.Comm_rank(), mpi.Comm_size()
method = "random" if os.environ.get("TEMPI_PLACEMENT_RANDOM") is not None else "partition"
node_size = int(os.environ["TEMPI_FAKE_NODE_SIZE"])
errors = 0


def fail(msg):
    global errors
    errors += 1
    print(f"rank {rank}: {msg}", flush=True)


def edges(r):
    """(sources, sourceweights, destinations, destweights) old rank r passes"""
    return ([(r - 2) % n, (r + 2) % n, (r - 1) % n], [100, 100, 1],
            [(r + 2) % n, (r - 2) % n, (r + 1) % n], [100, 100, 1])


def cut(app_of_process):
    """edge cut as the partitioner counts it -- every weight each rank
    passed, in-edges and out-edges alike, summed -- when process p runs
    application rank app_of_process[p] and sits on fake node p // node_size"""
    node_of_app = {a: p // node_size for p, a in enumerate(app_of_process)}
    c = 0
    for a in range(n):
        s, sw, d, dw = edges(a)
        for v, w in zip(s + d, sw + dw):
            if node_of_app[a] != node_of_app[v]:
                c += w
    return c


s, sw, d, dw = edges(rank)
g = mpi.Dist_graph_create_adjacent(s, d, reorder=True, sourceweights=sw, destweights=dw)
q = mpi.Comm_rank(g)
info = mpi.placement_info()
app = mpi.Allgather_int(q)  # world order: the application rank each process runs
if "--expect-none" in sys.argv:  # no TEMPI_PLACEMENT_*: the library's call, ranks unchanged
    if q != rank or info["placed"]:
        fail(f"placement without TEMPI_PLACEMENT_*: rank {q}, info {info}")
    mpi.Comm_free(g)
    mpi.Finalize()
    print(f"RESULT errors={errors}", flush=True)
    sys.exit(1 if errors else 0)

# 1. a permutation, and the communicator is in application order
if sorted(app) != list(range(n)):
    fail(f"new ranks {app} are not a permutation")
if mpi.Allgather_int(q, comm=g) != list(range(n)):
    fail("the placed communicator is not in application rank order")
if not info["placed"] or info["app_rank"] != q or info["nodes"] != n // node_size:
    fail(f"placement info {info}")

# 2. application rank q has old rank q's edges
gs, gd, gsw, gdw = mpi.Dist_graph_neighbors(g, 3, 3, weights=True)
es, esw, ed, edw = edges(q)
if (gs, gd, gsw, gdw) != (es, ed, esw, edw):
    fail(f"neighbours of {q}: {gs} {gd} {gsw} {gdw}, expected {es} {ed} {esw} {edw}")

# 3. the placement itself
if method == "partition":
    parities = [a % 2 for a in app]
    for k in range(n // node_size):
        if len(set(parities[k * node_size:(k + 1) * node_size])) != 1:
            fail(f"node {k} holds both parities: {app}")
    identity = cut(list(range(n)))
    if info["cut_identity"] != identity or info["cut_placed"] != cut(app) or not cut(app) < identity:
        fail(f"cuts {info}, expected identity {identity} placed {cut(app)}")
elif rank == 0:
    print(f"random placement: {app}", flush=True)

# 4a. Isend / Irecv along every edge (tag = edge index), host ints
sendv = np.array([q * 100 + i for i in range(3)], dtype=np.int32)
recvv = np.full(3, -1, dtype=np.int32)
reqs = [mpi.Irecv(recvv[i:].ctypes.data, 1, mpi.INT, gs[i], i, g) for i in range(3)]
# the sender's out-edge j toward d reaches d as its in-edge i with the same offset class:
# out-edge 0 (+2) is in-edge 0 of the receiver (from -2), 1 <-> 1, 2 (+1) <-> 2 (from -1)
reqs += [mpi.Isend(sendv[j:].ctypes.data, 1, mpi.INT, gd[j], j, g) for j in range(3)]
mpi.Waitall(reqs)
want = [gs[i] * 100 + i for i in range(3)]
if list(recvv) != want:
    fail(f"Isend/Irecv on the placed communicator: {list(recvv)}, expected {want}")

# 4b. MPI_Neighbor_alltoallv, host ints
nb_s = np.array([q * 1000 + j for j in range(3)], dtype=np.int32)
nb_r = np.full(3, -1, dtype=np.int32)
mpi.Neighbor_alltoallv(nb_s.ctypes.data, [1, 1, 1], [0, 1, 2], mpi.INT, nb_r.ctypes.data, [1, 1, 1], [0, 1, 2],
                       mpi.INT, g)
if list(nb_r) != [gs[i] * 1000 + i for i in range(3)]:
    fail(f"Neighbor_alltoallv on the placed communicator: {list(nb_r)}")

# 4c. --device: a strided device type along every edge through TEMPI
if device:
    from oracle import pyoracle
    from tests import typezoo

    RECIPE = "subarray(C,[16,24,256],[8,12,96],[2,3,64],byte)"
    tm = pyoracle.TypeMap(RECIPE)
    origin, buflen = tm.geometry(1)
    T, temps, basic = typezoo.build(mpi, RECIPE)
    src_h = [np.random.default_rng(1000 * q + j).integers(0, 256, buflen, dtype=np.uint8) for j in range(3)]
    dst_h = [np.random.default_rng(5000 + 1000 * q + i).integers(0, 256, buflen, dtype=np.uint8) for i in range(3)]
    src = [torch.from_numpy(h).cuda() for h in src_h]
    dst = [torch.from_numpy(h).cuda() for h in dst_h]
    torch.cuda.synchronize()
    c0 = mpi.counters()["isends"]
    reqs = [mpi.Irecv(dst[i].data_ptr() + origin, 1, T, gs[i], 10 + i, g) for i in range(3)]
    reqs += [mpi.Isend(src[j].data_ptr() + origin, 1, T, gd[j], 10 + j, g) for j in range(3)]
    mpi.Waitall(reqs)
    torch.cuda.synchronize()
    if mpi.counters()["isends"] - c0 != 3:
        fail("device sends did not go through TEMPI")
    for i in range(3):
        peer = gs[i]
        peer_src = np.random.default_rng(1000 * peer + i).integers(0, 256, buflen, dtype=np.uint8)
        e = dst_h[i].copy()
        tm.unpack(tm.pack(peer_src, origin, 1), e, origin, 1)
        if not np.array_equal(dst[i].cpu().numpy(), e):
            fail(f"device edge {i} from {peer}: bytes differ")
    typezoo.free(mpi, T, temps, basic)
mpi.Comm_free(g)

# 5. reorder = 0, and a single node: no placement
before = mpi.placement_info()
g0 = mpi.Dist_graph_create_adjacent(s, d, reorder=False, sourceweights=sw, destweights=dw)
if mpi.Comm_rank(g0) != rank or mpi.placement_info() != before:
    fail("reorder = 0 moved ranks")
mpi.Comm_free(g0)
os.environ["TEMPI_FAKE_NODE_SIZE"] = str(n)  # read at the call
g1 = mpi.Dist_graph_create_adjacent(s, d, reorder=True, sourceweights=sw, destweights=dw)
if mpi.Comm_rank(g1) != rank or mpi.placement_info() != before:
    fail("one node: placement moved ranks (the reference's guard leaves them)")
mpi.Comm_free(g1)

mpi.Finalize()
print(f"RESULT errors={errors}", flush=True)
sys.exit(1 if errors else 0)
