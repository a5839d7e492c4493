"""Run under mpiexec -n N (N even) with TEMPI_FAKE_NODE_SIZE and a
TEMPI_PLACEMENT_* method: the reference's dist_graph_create_adjacent test
(/root/reference/test/dist_graph_create_adjacent.cpp:17-49) -- every rank
pairs with rank + N/2 (mod N), one in-edge and one out-edge of weight 1,
MPI_Dist_graph_create_adjacent with reorder = 1 under METIS placement, then
MPI_Comm_free. The reference only checks that the calls return; here the
graph communicator must also give each application rank its partner back
(MPI_Dist_graph_neighbors), carry a message to it, and free cleanly, and the
pairs must not be cut by the placement when a pair fits on a node."""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)

import tempi_amd  # noqa: E402

mpi = tempi_amd.get_mpi()
mpi.Init()
rank, n = mpi.Comm_rank(), mpi.Comm_size()
node_size = int(os.environ.get("TEMPI_FAKE_NODE_SIZE", str(n)))
errors = 0


def fail(msg):
    global errors
    errors += 1
    print(f"rank {rank}: {msg}", flush=True)


partner = (rank + n // 2) % n
g = mpi.Dist_graph_create_adjacent([partner], [partner], reorder=True, sourceweights=[1], destweights=[1])
q = mpi.Comm_rank(g)  # the application rank this process now runs
if mpi.Allgather_int(q, comm=g) != list(range(n)):
    fail("the graph communicator is not in application order")
want = (q + n // 2) % n
gs, gd = mpi.Dist_graph_neighbors(g, 1, 1)
if list(gs) != [want] or list(gd) != [want]:
    fail(f"neighbours {gs} {gd}, expected [{want}]")
# a message along the edge reaches the application rank it names
sendv = np.array([1000 + q], dtype=np.int32)
recvv = np.zeros(1, dtype=np.int32)
reqs = [mpi.Irecv(recvv.ctypes.data, 1, mpi.INT, gs[0], 5, g), mpi.Isend(sendv.ctypes.data, 1, mpi.INT, gd[0], 5, g)]
mpi.Waitall(reqs)
if int(recvv[0]) != 1000 + want:
    fail(f"received {int(recvv[0])}, expected {1000 + want}")
# a pair that fits on one node is kept together by the partitioner (the
# random rule promises nothing about cuts)
if node_size >= 2 and os.environ.get("TEMPI_PLACEMENT_RANDOM") is None:
    app = mpi.Allgather_int(q)  # world order: application rank of each process
    node_of_app = {a: p // node_size for p, a in enumerate(app)}
    if node_of_app[q] != node_of_app[want]:
        fail(f"application ranks {q} and {want} were split across nodes")
mpi.Comm_free(g)
total = mpi.Allreduce_double(float(errors), op=mpi.SUM)
if rank == 0:
    print(f"RESULT errors={int(total)}", flush=True)
mpi.Finalize()
sys.exit(1 if total else 0)
