"""Run under mpiexec -n 1 (or more: every rank runs the same cases with
itself): TEMPI's self channel, which matches a process's device messages to
itself inside TEMPI, against MPI's matching rules -- earliest matching send,
earliest matching receive, MPI_ANY_TAG -- and its spill, which hands what it
holds to the library the moment something it cannot carry touches this
rank's messages on the communicator: a host send, an MPI_ANY_SOURCE
receive, a probe, an MPI_Issend. Each case runs on a communicator of its own
(a spill is permanent per communicator). Every byte and status is checked
against the oracle; the self_matched counter shows which cases the channel
carried."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import tempi_amd  # noqa: E402
from oracle import pyoracle  # noqa: E402
from tests import typezoo  # noqa: E402

torch.cuda.set_device(0)
mpi = tempi_amd.get_mpi()
mpi.Init()
rank = mpi.Comm_rank()
errors = 0
RECIPE = "subarray(C,[20,30,512],[10,12,48],[3,4,64],byte)"  # 10 x 12 rows of 48 B
tm = pyoracle.TypeMap(RECIPE)
origin, buflen = tm.geometry(1)
T, temps, basic = typezoo.build(mpi, RECIPE)
N = tm.size
seed = [100]


def fail(msg):
    global errors
    errors += 1
    print(f"rank {rank}: {msg}", flush=True)


def new_src():
    seed[0] += 1
    h = np.random.default_rng(seed[0]).integers(0, 256, buflen, dtype=np.uint8)
    return h, torch.from_numpy(h).cuda()


def new_dst():
    seed[0] += 1
    h = np.random.default_rng(seed[0]).integers(0, 256, buflen, dtype=np.uint8)
    return h, torch.from_numpy(h).cuda()


def expect(canvas, src_host):
    e = canvas.copy()
    tm.unpack(tm.pack(src_host, origin, 1), e, origin, 1)
    return e


def check(name, dev, canvas, src_host):
    torch.cuda.synchronize()
    got = dev.cpu().numpy()
    if not np.array_equal(got, expect(canvas, src_host)):
        fail(f"{name}: bytes differ")


def isend(comm, src_dev, tag):
    return mpi.Isend(src_dev.data_ptr() + origin, 1, T, rank, tag, comm)


def irecv(comm, dst_dev, tag, source=None):
    return mpi.Irecv(dst_dev.data_ptr() + origin, 1, T, rank if source is None else source, tag, comm)


CHANNEL = not (os.environ.get("TEMPI_NO_SELF_CHANNEL") or os.environ.get("TEMPI_NO_DIRECT"))


def matched():
    return mpi.counters()["self_matched"]


torch.cuda.synchronize()

# 1. sends first: each receive takes the earliest matching send (tags 1, 2, 1;
#    receives for 1, ANY, 1 get A, B, C)
c = mpi.Comm_dup()
m0 = matched()
srcs = [new_src() for _ in range(3)]
sreqs = [isend(c, s[1], t) for s, t in zip(srcs, (1, 2, 1))]
dsts = [new_dst() for _ in range(3)]
rreqs = [irecv(c, d[1], t) for d, t in zip(dsts, (1, mpi.ANY_TAG, 1))]
for i, (r, exp_tag) in enumerate(zip(rreqs, (1, 2, 1))):
    _, st = mpi.Wait_status(r, T)
    if st != (rank, exp_tag, 1):
        fail(f"case 1 receive {i}: status {st}")
for s in sreqs:
    mpi.Wait(s)
for i, (d, s) in enumerate(zip(dsts, (srcs[0], srcs[1], srcs[2]))):
    check(f"case 1 receive {i}", d[1], d[0], s[0])
if CHANNEL and matched() - m0 != 3:
    fail(f"case 1: the self channel matched {matched() - m0} of 3")
mpi.Comm_free(c)

# 2. receives first: a send takes the earliest waiting receive that matches
c = mpi.Comm_dup()
m0 = matched()
d1, d2 = new_dst(), new_dst()
r1, r2 = irecv(c, d1[1], 5), irecv(c, d2[1], mpi.ANY_TAG)
s1, s2 = new_src(), new_src()
q1, q2 = isend(c, s1[1], 6), isend(c, s2[1], 5)  # tag 6 skips r1 (tag 5) and takes r2 (ANY)
for r, exp in ((r1, (rank, 5, 1)), (r2, (rank, 6, 1))):
    _, st = mpi.Wait_status(r, T)
    if st != exp:
        fail(f"case 2: status {st}, expected {exp}")
mpi.Wait(q1)
mpi.Wait(q2)
check("case 2 r1", d1[1], d1[0], s2[0])
check("case 2 r2", d2[1], d2[0], s1[0])
if CHANNEL and matched() - m0 != 2:
    fail(f"case 2: the self channel matched {matched() - m0} of 2")
mpi.Comm_free(c)

# 3. spill with a receive waiting: a host send to this rank reaches it
c = mpi.Comm_dup()
d = new_dst()
r = irecv(c, d[1], 7)
h_src = new_src()[0]
packed = tm.pack(h_src, origin, 1)
hreq = mpi.Isend(packed.ctypes.data, N, mpi.BYTE, rank, 7, c)
_, st = mpi.Wait_status(r, T)
mpi.Wait(hreq)
if st != (rank, 7, 1):
    fail(f"case 3: status {st}")
check("case 3", d[1], d[0], h_src)
m0 = matched()  # after the spill the channel carries nothing on this communicator
s = new_src()
d = new_dst()
q = isend(c, s[1], 8)
mpi.Wait(irecv(c, d[1], 8))
mpi.Wait(q)
check("case 3 after spill", d[1], d[0], s[0])
if matched() != m0:
    fail("case 3: the channel matched after its spill")
mpi.Comm_free(c)

# 4. spill with sends queued: order A, B (device, queued), then C (host) --
#    receives get A, B, C
c = mpi.Comm_dup()
a, b = new_src(), new_src()
qa, qb = isend(c, a[1], 3), isend(c, b[1], 3)
ch = new_src()[0]
cpk = tm.pack(ch, origin, 1)
qc = mpi.Isend(cpk.ctypes.data, N, mpi.BYTE, rank, 3, c)
da, db = new_dst(), new_dst()
ra, rb = irecv(c, da[1], 3), irecv(c, db[1], 3)
hc = np.zeros(N, dtype=np.uint8)
rc_ = mpi.Irecv(hc.ctypes.data, N, mpi.BYTE, rank, 3, c)
for x in (ra, rb, rc_, qa, qb, qc):
    mpi.Wait(x)
check("case 4 A", da[1], da[0], a[0])
check("case 4 B", db[1], db[0], b[0])
if not np.array_equal(hc, cpk):
    fail("case 4 C: bytes differ")
mpi.Comm_free(c)

# 5. an MPI_ANY_SOURCE receive spills; it matches the queued send
c = mpi.Comm_dup()
s = new_src()
q = isend(c, s[1], 9)
d = new_dst()
_, st = mpi.Wait_status(irecv(c, d[1], 9, source=mpi.ANY_SOURCE), T)
mpi.Wait(q)
if st != (rank, 9, 1):
    fail(f"case 5: status {st}")
check("case 5", d[1], d[0], s[0])
mpi.Comm_free(c)

# 6. a probe spills and reports the payload of the queued send
c = mpi.Comm_dup()
s = new_src()
q = isend(c, s[1], 10)
pst = mpi.Probe(rank, 10, T, comm=c)
if pst != (rank, 10, 1):
    fail(f"case 6: probe {pst}")
d = new_dst()
mpi.Wait(irecv(c, d[1], 10))
mpi.Wait(q)
check("case 6", d[1], d[0], s[0])
mpi.Comm_free(c)

# 7. a waiting receive cancelled: nothing written; a later send matches the
#    next receive
c = mpi.Comm_dup()
d = new_dst()
r = irecv(c, d[1], 11)
mpi.Cancel(r)
_, was = mpi.Wait_cancelled(r)
torch.cuda.synchronize()
if not was or not np.array_equal(d[1].cpu().numpy(), d[0]):
    fail("case 7: cancelled receive not reported cancelled or written")
s, d = new_src(), new_dst()
q = isend(c, s[1], 11)
mpi.Wait(irecv(c, d[1], 11))
mpi.Wait(q)
check("case 7 after cancel", d[1], d[0], s[0])
mpi.Comm_free(c)

# 8. MPI_Issend to this rank (a send mode TEMPI does not carry) spills; the
#    waiting device receive gets it
c = mpi.Comm_dup()
d = new_dst()
r = irecv(c, d[1], 12)
h_src = new_src()[0]
pk = tm.pack(h_src, origin, 1)
ireq = mpi.Request()
rcode = mpi.L.MPI_Issend(ctypes.c_void_p(pk.ctypes.data), N, mpi.h(mpi.BYTE), rank, 12, mpi.h(c), ctypes.byref(ireq))
if rcode != 0:
    fail(f"case 8: MPI_Issend rc {rcode}")
mpi.Wait(r)
mpi.Wait(ireq.value)
check("case 8", d[1], d[0], h_src)
mpi.Comm_free(c)

# 9. a send waited on before its receive exists completes alone (gather
#    fallback), and the later receive still gets it from the channel. (A
#    program MPI calls unsafe: the library route of TEMPI_NO_DIRECT may, like
#    the library itself, hold a send to this rank until its receive exists.)
c = mpi.Comm_dup()
if os.environ.get("TEMPI_NO_DIRECT"):
    mpi.Comm_free(c)
    c = None
if c is not None:
    s = new_src()
    mpi.Wait(isend(c, s[1], 13))
    d = new_dst()
    mpi.Wait(irecv(c, d[1], 13))
    check("case 9", d[1], d[0], s[0])
    mpi.Comm_free(c)

typezoo.free(mpi, T, temps, basic)
print(f"rank {rank} self_matched={mpi.counters()['self_matched']}", flush=True)
mpi.Finalize()
print(f"RESULT errors={errors}", flush=True)
sys.exit(1 if errors else 0)
