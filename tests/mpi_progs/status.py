"""Run under mpiexec -n 1 or -n 2: the MPI_Status of receives carries the
sender and tag and, through MPI_Get_count, the number of whole elements that
arrived (fewer than the receive allowed); both sides free their datatypes
before waiting (MPI allows it), for a strided type and an irregular one.
Blocking MPI_Recv statuses too. --device puts the buffers on the GPU. Every
byte is checked against the oracle."""
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
rank, size = mpi.Comm_rank(), mpi.Comm_size()
peer = (rank + 1) % size
src_rank = (rank - 1) % size
errors = 0


def fail(msg):
    global errors
    errors += 1
    print(f"rank {rank}: {msg}", flush=True)


def buf(n, seed):
    h = np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8)
    if device:
        return h, torch.from_numpy(h).cuda()
    return h, h.copy()


def ptr(b):
    return b.data_ptr() if device else b.ctypes.data


def host(b):
    if device:
        torch.cuda.synchronize()
        return b.cpu().numpy()
    return b


RECIPES = ["subarray(C,[40,38,512],[30,3,24],[5,3,24],byte)", "hindexed([700,1100],[0,1000],byte)"]
for it, recipe in enumerate(RECIPES * 2):
    blocking = it >= len(RECIPES)
    tm = pyoracle.TypeMap(recipe)
    sent, cap = 2, 3  # elements sent; elements the receive allows
    origin, buflen = tm.geometry(cap)
    tag = 40 + it
    # the send
    s_host, s_dev = buf(buflen, 100 * it + rank)
    ts, temps, basic = typezoo.build(mpi, recipe)
    sreq = mpi.Isend(ptr(s_dev) + origin, sent, ts, peer, tag)
    typezoo.free(mpi, ts, temps, basic)  # freed while the send is in flight
    # the receive, into room for `cap` elements
    canvas, r_dev = buf(buflen, 7000 + it)
    tr, temps_r, basic_r = typezoo.build(mpi, recipe)
    probe_t, probe_temps, probe_basic = typezoo.build(mpi, recipe)  # an equivalent type for MPI_Get_count
    if blocking:
        src, got_tag, n = mpi.Recv_status(ptr(r_dev) + origin, cap, tr, src_rank, mpi.ANY_TAG)
        typezoo.free(mpi, tr, temps_r, basic_r)
        mpi.Wait(sreq)
        src_st, tag_st, n_st = src, got_tag, n
    else:
        rreq = mpi.Irecv(ptr(r_dev) + origin, cap, tr, mpi.ANY_SOURCE, mpi.ANY_TAG)
        typezoo.free(mpi, tr, temps_r, basic_r)  # freed while the receive is in flight
        mpi.Wait(sreq)
        _, (src_st, tag_st, n_st) = mpi.Wait_status(rreq, probe_t)
    if src_st != src_rank:
        fail(f"{recipe}: status source {src_st}, expected {src_rank}")
    if tag_st != tag:
        fail(f"{recipe}: status tag {tag_st}, expected {tag}")
    if n_st != sent:
        fail(f"{recipe}: MPI_Get_count {n_st}, expected {sent} ({'blocking' if blocking else 'Irecv'})")
    src_bytes = np.random.default_rng(100 * it + src_rank).integers(0, 256, buflen, dtype=np.uint8)
    exp = canvas.copy()
    tm.unpack(tm.pack(src_bytes, origin, sent), exp, origin, sent)
    if not np.array_equal(host(r_dev), exp):
        fail(f"{recipe}: received bytes differ ({'blocking' if blocking else 'Irecv'})")
    typezoo.free(mpi, probe_t, probe_temps, probe_basic)

# MPI_Sendrecv around the ring (device objects go through TEMPI), with its
# status: source, tag, and MPI_Get_count (fewer elements than allowed)
recipe = RECIPES[0]
tm = pyoracle.TypeMap(recipe)
origin, buflen = tm.geometry(3)
t, temps, basic = typezoo.build(mpi, recipe)
s_host, s_dev = buf(buflen, 51 + rank)
canvas, r_dev = buf(buflen, 52)
got = mpi.Sendrecv(ptr(s_dev) + origin, 2, t, peer, 60 + rank, ptr(r_dev) + origin, 3, t, src_rank, mpi.ANY_TAG)
if got != (src_rank, 60 + src_rank, 2):
    fail(f"MPI_Sendrecv status {got}, expected {(src_rank, 60 + src_rank, 2)}")
exp = canvas.copy()
tm.unpack(tm.pack(np.random.default_rng(51 + src_rank).integers(0, 256, buflen, dtype=np.uint8), origin, 2), exp,
          origin, 2)
if not np.array_equal(host(r_dev), exp):
    fail("MPI_Sendrecv bytes differ")
typezoo.free(mpi, t, temps, basic)

# MPI_Request_get_status leaves the request; MPI_Cancel of a receive nothing
# will match (tag 999) completes it as cancelled
recipe = RECIPES[0]
tm = pyoracle.TypeMap(recipe)
origin, buflen = tm.geometry(1)
t, temps, basic = typezoo.build(mpi, recipe)
s_host, s_dev = buf(buflen, 31 + rank)
canvas, r_dev = buf(buflen, 32)
rreq = mpi.Irecv(ptr(r_dev) + origin, 1, t, src_rank, 77)
sreq = mpi.Isend(ptr(s_dev) + origin, 1, t, peer, 77)
while True:
    flag, st = mpi.Request_get_status(rreq, t)
    if flag:
        break
if st != (src_rank, 77, 1):
    fail(f"MPI_Request_get_status gave {st}, expected {(src_rank, 77, 1)}")
_, (src_st, tag_st, n_st) = mpi.Wait_status(rreq, t)  # still a live request: the wait releases it
if (src_st, tag_st, n_st) != (src_rank, 77, 1):
    fail(f"wait after MPI_Request_get_status gave {(src_st, tag_st, n_st)}")
mpi.Wait(sreq)
exp = canvas.copy()
tm.unpack(tm.pack(np.random.default_rng(31 + src_rank).integers(0, 256, buflen, dtype=np.uint8), origin, 1), exp,
          origin, 1)
if not np.array_equal(host(r_dev), exp):
    fail("bytes after MPI_Request_get_status differ")
for obj_recipe in RECIPES:  # strided (TEMPI receive) and irregular (library-packed receive)
    ot, otemps, obasic = typezoo.build(mpi, obj_recipe)
    otm = pyoracle.TypeMap(obj_recipe)
    o_origin, o_len = otm.geometry(1)
    canvas, r_dev = buf(o_len, 33)
    creq = mpi.Irecv(ptr(r_dev) + o_origin, 1, ot, src_rank, 999)
    mpi.Cancel(creq)
    left, was_cancelled = mpi.Wait_cancelled(creq)
    if not was_cancelled:
        fail(f"{obj_recipe}: cancelled receive not reported as cancelled")
    if not np.array_equal(host(r_dev), canvas):
        fail(f"{obj_recipe}: a cancelled receive wrote its buffer")
    typezoo.free(mpi, ot, otemps, obasic)
typezoo.free(mpi, t, temps, basic)

mpi.Finalize()
print(f"RESULT errors={errors}", flush=True)
sys.exit(1 if errors else 0)
