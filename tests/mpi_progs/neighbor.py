"""Run under mpiexec -n N: MPI_Neighbor_alltoallw / MPI_Neighbor_alltoallv
through libtempi.so on a distributed graph (random edges, self-edges and
repeated edges included) and on a periodic Cartesian grid, with strided
datatypes whose send and receive shapes differ (equal sizes).

Two oracles: (1) oracle/typemap.c -- every receive block equals
unpack(recv type, pack(send type, the sender's block)) over an untouched
canvas, edges between the same pair matched in edge order; (2) the MPI
library's own neighbourhood collective run on host copies of the same buffers
(the reference's parity oracle is the library, test/pack_unpack.cpp:61-97).
--device puts the buffers on the GPU (TEMPI's per-edge route); without it the
host buffers go to the library (passthrough) and only oracle (1) applies.
"""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)

import tempi_amd  # noqa: E402
from oracle import pyoracle  # noqa: E402
from tests import typezoo  # noqa: E402

device = "--device" in sys.argv
mpi = tempi_amd.get_mpi()
if device:
    import torch

    torch.cuda.set_device(0)
mpi.Init()
rank, n = mpi.Comm_rank(), mpi.Comm_size()

# (send recipe, receive recipe): equal type sizes, different shapes
PAIRS = [
    ("vector(64,24,40,byte)", "vector(96,16,24,byte)"),
    ("subarray(C,[20,30,64],[4,12,24],[1,2,8],byte)", "contig(1152,byte)"),
    ("vector(300,3,7,byte)", "vector(100,9,11,byte)"),
    ("hvector(5,1,53,hvector(3,1,16,contig(13,byte)))", "contig(195,byte)"),
    ("subarray(C,[40,38,512],[30,3,24],[5,3,24],byte)", "subarray(C,[40,38,512],[30,3,24],[5,3,24],byte)"),
]
for a, b in PAIRS:
    assert pyoracle.TypeMap(a).size == pyoracle.TypeMap(b).size, (a, b)

grng = np.random.default_rng(5)
dests = [list(grng.integers(0, n, grng.integers(1, 5))) for _ in range(n)]
edges = [(r, int(d), k) for r in range(n) for k, d in enumerate(dests[r])]  # k-th out-edge of r
sources = [r for (r, d, k) in edges if d == rank]
in_edges = [(r, k) for (r, d, k) in edges if d == rank]


def edge_kind(r, k):
    return (r * 7 + k * 3) % len(PAIRS), 1 + (r + k) % 2  # pair index, count


types = {}


def dtype(recipe):
    if recipe not in types:
        types[recipe] = typezoo.build(mpi, recipe)
    return types[recipe][0]


def layout(recipes_counts):
    """byte displacement (of the type origin) of each block in one buffer"""
    displs, off = [], 0
    for recipe, count in recipes_counts:
        origin, buflen = pyoracle.TypeMap(recipe).geometry(count)
        displs.append(off + origin)
        off += buflen + 16
    return displs, off + 16


def block_payload(r, k, buflen):
    return np.random.default_rng(1000 * r + k).integers(0, 256, buflen, dtype=np.uint8)


def run_alltoallw(comm, out_nbrs, in_keys, label):
    send_rc = [(PAIRS[edge_kind(rank, k)[0]][0], edge_kind(rank, k)[1]) for k in range(len(out_nbrs))]
    recv_rc = [(PAIRS[edge_kind(r, k)[0]][1], edge_kind(r, k)[1]) for (r, k) in in_keys]
    sd, slen = layout(send_rc)
    rd, rlen = layout(recv_rc)
    send = np.zeros(slen, dtype=np.uint8)
    for k, ((recipe, count), d) in enumerate(zip(send_rc, sd)):
        origin, buflen = pyoracle.TypeMap(recipe).geometry(count)
        send[d - origin:d - origin + buflen] = block_payload(rank, k, buflen)
    canvas = np.random.default_rng(77 + rank).integers(0, 256, rlen, dtype=np.uint8)
    expected = canvas.copy()
    for (r, k), (recipe, count), d in zip(in_keys, recv_rc, rd):
        srecipe = PAIRS[edge_kind(r, k)[0]][0]
        stm = pyoracle.TypeMap(srecipe)
        so, sl = stm.geometry(count)
        packed = stm.pack(block_payload(r, k, sl), so, count)
        pyoracle.TypeMap(recipe).unpack(packed, expected, d, count)
    stypes = [dtype(rc[0]) for rc in send_rc]
    rtypes = [dtype(rc[0]) for rc in recv_rc]
    scounts = [rc[1] for rc in send_rc]
    rcounts = [rc[1] for rc in recv_rc]
    errs = 0
    # the library on host copies
    hrecv = canvas.copy()
    mpi.Neighbor_alltoallw(send.ctypes.data, scounts, sd, stypes, hrecv.ctypes.data, rcounts, rd, rtypes, comm)
    if not np.array_equal(hrecv, expected):
        errs += 1
        print(f"[{rank}] {label}: library result differs from the oracle", flush=True)
    if device:
        dsend = torch.from_numpy(send).cuda()
        drecv = torch.from_numpy(canvas.copy()).cuda()
        torch.cuda.synchronize()
        before = mpi.counters()["neighbor_colls"]
        mpi.Neighbor_alltoallw(dsend.data_ptr(), scounts, sd, stypes, drecv.data_ptr(), rcounts, rd, rtypes, comm)
        got = drecv.cpu().numpy()
        if mpi.counters()["neighbor_colls"] != before + 1:
            errs += 1
            print(f"[{rank}] {label}: TEMPI did not take the device call", flush=True)
        if not np.array_equal(got, expected):
            errs += 1
            bad = np.nonzero(got != expected)[0]
            print(f"[{rank}] {label}: device result differs at {bad[:8]} ({bad.size} bytes)", flush=True)
    return errs


errors = 0
g = mpi.Dist_graph_create_adjacent(sources, [int(d) for d in dests[rank]])
s_, d_ = mpi.Dist_graph_neighbors(g, len(sources), len(dests[rank]))
assert s_ == sources and d_ == [int(d) for d in dests[rank]], (s_, d_)
# the k-th edge from r to this rank is the k-th occurrence of r among the sources
errors += run_alltoallw(g, dests[rank], in_edges, "dist graph")
errors += run_alltoallw(g, dests[rank], in_edges, "dist graph (again: cached state)")

# periodic 1-D Cartesian grid, MPI_Neighbor_alltoallv with one strided type
cart = mpi.Cart_create([n], [True])
lo, hi = mpi.Cart_shift(cart, 0)
recipe, count = "vector(64,24,40,byte)", 2
tm = pyoracle.TypeMap(recipe)
t = dtype(recipe)
lb, ext = mpi.Type_get_extent(t)
origin, buflen = tm.geometry(count)
per = (buflen + ext - 1) // ext + 1  # extents per block
sdis, rdis = [0, per], [0, per]
blen = 2 * per * ext + buflen
sendv = np.random.default_rng(900 + rank).integers(0, 256, blen, dtype=np.uint8)
canv = np.random.default_rng(901 + rank).integers(0, 256, blen, dtype=np.uint8)
hr = canv.copy()
mpi.Neighbor_alltoallv(sendv.ctypes.data + origin, [count, count], sdis, t, hr.ctypes.data + origin,
                       [count, count], rdis, t, cart)
if device:
    ds, dr = torch.from_numpy(sendv).cuda(), torch.from_numpy(canv.copy()).cuda()
    torch.cuda.synchronize()
    mpi.Neighbor_alltoallv(ds.data_ptr() + origin, [count, count], sdis, t, dr.data_ptr() + origin,
                           [count, count], rdis, t, cart)
    if not np.array_equal(dr.cpu().numpy(), hr):
        errors += 1
        print(f"[{rank}] cart alltoallv: device result differs from the library's", flush=True)
if n > 2:  # neighbours are distinct ranks: check against the oracle too
    exp = canv.copy()
    for slot, src in ((0, lo), (1, hi)):
        sv = np.random.default_rng(900 + src).integers(0, 256, blen, dtype=np.uint8)
        # the source sent to me from its opposite slot
        sslot = 1 - slot
        packed = tm.pack(sv, origin + sdis[sslot] * ext, count)
        tm.unpack(packed, exp, origin + rdis[slot] * ext, count)
    if not np.array_equal(hr, exp):
        errors += 1
        print(f"[{rank}] cart alltoallv: library result differs from the oracle", flush=True)

mpi.Comm_free(cart)
mpi.Comm_free(g)
for t_, temps, basic in types.values():
    typezoo.free(mpi, t_, temps, basic)
total = mpi.Allreduce_double(float(errors), op=mpi.SUM)
if rank == 0:
    print(f"RESULT errors={int(total)}", flush=True)
mpi.Finalize()
sys.exit(1 if total else 0)
