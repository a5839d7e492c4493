"""Run under mpiexec -n 1 or 2: persistent requests (MPI_Send_init /
MPI_Ssend_init / MPI_Bsend_init / MPI_Rsend_init / MPI_Recv_init, MPI_Start /
MPI_Startall) and the send modes (MPI_Ssend / MPI_Bsend / MPI_Rsend and their
I-forms), which the reference does not interpose. Each rank sends to
(rank + 1) % size and receives from (rank - 1) % size, so one rank exercises
messages to itself. Every received byte is checked against the oracle.
--device puts the strided buffers on the GPU. With TEMPI holding the
persistent requests (a GPU, or TEMPI_TEST_HOST_ONLY) it also checks that a
second MPI_Start of an active request is an error and that the starts were
counted."""
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
mpi.Comm_set_errhandler(mpi.ERRORS_RETURN)
rank, size = mpi.Comm_rank(), mpi.Comm_size()
peer, src = (rank + 1) % size, (rank - 1) % size
recipe, count = "subarray(C,[40,38,512],[30,3,24],[5,3,24],byte)", 2  # 4320 packed bytes
tm = pyoracle.TypeMap(recipe)
origin, buflen = tm.geometry(count)
t, temps, basic = typezoo.build(mpi, recipe)
packed = mpi.Pack_size(count, t)
tempi_holds = device or os.environ.get("TEMPI_TEST_HOST_ONLY") == "1"
errors = 0
mpi.Buffer_attach(8 * (packed + mpi.const("MPI_BSEND_OVERHEAD")) + 4096)
mpi.reset_counters()


def fail(msg):
    global errors
    errors += 1
    print(f"[{rank}] {msg}", flush=True)


def rand(seed):
    return np.random.default_rng(seed).integers(0, 256, buflen, dtype=np.uint8)


def buf(seed):
    h = rand(seed)
    return torch.from_numpy(h).cuda() if device else h


def ptr(b):
    return b.ctypes.data if isinstance(b, np.ndarray) else b.data_ptr()


def host(b):
    if isinstance(b, np.ndarray):  # (host receives of device sends, too)
        return b
    torch.cuda.synchronize()
    return b.cpu().numpy()


def refill(b, seed):
    h = rand(seed)
    if device:
        b.copy_(torch.from_numpy(h))
        torch.cuda.synchronize()
    else:
        b[:] = h


def check(label, rbuf, canvas_seed, src_seed):
    exp = rand(canvas_seed)
    tm.unpack(tm.pack(rand(src_seed), origin, count), exp, origin, count)
    if not np.array_equal(host(rbuf), exp):
        fail(f"{label}: wrong bytes")


# ---------------------------------------------------------------- persistent
INITS = {"send": mpi.Send_init, "ssend": mpi.Ssend_init, "bsend": mpi.Bsend_init, "rsend": mpi.Rsend_init}
for m, (mode, init) in enumerate(INITS.items()):
    tag = 20 + m
    dup = mpi.Type_dup(t)
    mpi.Type_commit(dup)
    sbuf, rbuf = buf(1), buf(2)
    rreq = mpi.Recv_init(ptr(rbuf) + origin, count, dup, src, tag)
    sreq = init(ptr(sbuf) + origin, count, dup, peer, tag)
    mpi.Type_free(dup)  # the persistent requests keep what they need
    for it in range(3):
        refill(sbuf, 1000 * rank + 10 * it + m)
        refill(rbuf, 500 + it)
        r2 = mpi.Start(rreq)
        mpi.Barrier()  # (ready mode: every receive is posted before its send starts)
        s2 = mpi.Start(sreq)
        assert r2 == rreq and s2 == sreq
        r2, (s_src, s_tag, n) = mpi.Wait_status(rreq, t)
        if r2 != rreq:
            fail(f"{mode}: the wait released the persistent receive")
        if (s_src, s_tag, n) != (src, tag, count):
            fail(f"{mode} it {it}: status {(s_src, s_tag, n)} != {(src, tag, count)}")
        if mpi.Wait(sreq) != sreq:
            fail(f"{mode}: the wait released the persistent send")
        check(f"{mode} it {it}", rbuf, 500 + it, 1000 * src + 10 * it + m)
    # inactive: completes at once, skipped by the any / some family
    flag, r2 = mpi.Test(rreq)
    if not flag or r2 != rreq:
        fail(f"{mode}: inactive test {flag} {r2}")
    flag, st = mpi.Request_get_status(rreq, t)
    if not flag:
        fail(f"{mode}: inactive get_status not complete")
    idx, flag, reqs = mpi.Testany([rreq, sreq])
    if not flag or idx != mpi.UNDEFINED or reqs != [rreq, sreq]:
        fail(f"{mode}: Testany over inactive requests gave {(idx, flag)}")
    idx, reqs = mpi.Waitany([rreq, sreq])
    if idx != mpi.UNDEFINED:
        fail(f"{mode}: Waitany over inactive requests gave {idx}")
    got, reqs = mpi.Testsome([rreq, sreq])
    if got is not None:
        fail(f"{mode}: Testsome over inactive requests gave {got}")
    flag, reqs = mpi.Testall([rreq, sreq])
    if not flag or reqs != [rreq, sreq]:
        fail(f"{mode}: Testall over inactive requests gave {flag}")
    # MPI_Startall + MPI_Waitall: the handles stay
    refill(sbuf, 77 + rank)
    refill(rbuf, 78)
    rreq, = mpi.Startall([rreq])
    mpi.Barrier()
    reqs = mpi.Startall([sreq])
    reqs = mpi.Waitall([rreq, sreq])
    if reqs != [rreq, sreq]:
        fail(f"{mode}: Waitall released persistent requests")
    check(f"{mode} startall", rbuf, 78, 77 + src)
    if mpi.Request_free(rreq) != mpi.REQUEST_NULL or mpi.Request_free(sreq) != mpi.REQUEST_NULL:
        fail(f"{mode}: Request_free did not null the handle")
    mpi.Barrier()

# a started receive nothing matches: cancelled, the handle stays
rbuf = buf(3)
rreq = mpi.Recv_init(ptr(rbuf) + origin, count, t, src, 777)
mpi.Start(rreq)
if tempi_holds and mpi.Start_rc(rreq) == 0:
    fail("a second MPI_Start of an active request succeeded")
mpi.Cancel(rreq)
r2, cancelled = mpi.Wait_cancelled(rreq)
if not cancelled or r2 != rreq:
    fail(f"cancel of a started persistent receive: cancelled={cancelled}")
mpi.Request_free(rreq)
mpi.Barrier()

# a persistent host receive of a device send (a co-located device send may
# travel as a descriptor, which the persistent receive must land)
if device:
    sbuf = buf(4)
    refill(sbuf, 4000 + rank)
    hrecv = rand(41)
    rreq = mpi.Recv_init(hrecv.ctypes.data + origin, count, t, src, 30)
    mpi.Start(rreq)
    s = mpi.Isend(ptr(sbuf) + origin, count, t, peer, 30)
    mpi.Wait(rreq)
    mpi.Wait(s)
    check("host persistent receive of a device send", hrecv, 41, 4000 + src)
    mpi.Request_free(rreq)
    mpi.Barrier()

# ---------------------------------------------------------------- send modes
for m, mode in enumerate(("ssend", "bsend", "rsend", "issend", "ibsend", "irsend")):
    tag = 40 + m
    sbuf, rbuf = buf(5), buf(6)
    refill(sbuf, 3000 + 10 * rank + m)
    r = mpi.Irecv(ptr(rbuf) + origin, count, t, src, tag)
    mpi.Barrier()  # (ready mode)
    fn = getattr(mpi, mode.capitalize())
    s = fn(ptr(sbuf) + origin, count, t, peer, tag)
    mpi.Wait(r)
    if s is not None:
        mpi.Wait(s)
    check(mode, rbuf, 6, 3000 + 10 * src + m)
    mpi.Barrier()

# buffered mode against the attached buffer: a message that does not fit is
# an error (returned: ERRORS_RETURN), not a hang -- a device object's
# MPI_Ibsend reaches the library only after its gather
bsize = 8 * (packed + mpi.const("MPI_BSEND_OVERHEAD")) + 4096
mpi.Buffer_detach()
mpi.Buffer_attach(mpi.const("MPI_BSEND_OVERHEAD") + 64)  # (MPICH refuses less than its overhead)
sbuf = buf(7)
try:
    s = mpi.Ibsend(ptr(sbuf) + origin, count, t, peer, 60)
    mpi.Wait(s)
    fail("an MPI_Ibsend larger than the attached buffer succeeded")
except tempi_amd.mpi.MPIError:
    pass
mpi.Barrier()
mpi.Buffer_detach()
mpi.Buffer_attach(bsize)
# MPI_Buffer_detach right after MPI_Ibsend: the detach waits until the message
# is the library's, and it still arrives
sbuf, rbuf = buf(8), buf(9)
refill(sbuf, 8000 + rank)
r = mpi.Irecv(ptr(rbuf) + origin, count, t, src, 61)
mpi.Barrier()
s = mpi.Ibsend(ptr(sbuf) + origin, count, t, peer, 61)
mpi.Buffer_detach()
mpi.Wait(r)
mpi.Wait(s)
check("ibsend then detach", rbuf, 9, 8000 + src)
mpi.Barrier()
mpi.Buffer_attach(bsize)

# a receive the library refuses (a source rank outside the communicator,
# ERRORS_RETURN): an error at the call or at its wait, not a hang
rbuf = buf(12)
try:
    r = mpi.Irecv(ptr(rbuf) + origin, count, t, size + 3, 63)
    mpi.Wait(r)
    fail("a receive from a rank outside the communicator succeeded")
except tempi_amd.mpi.MPIError:
    pass
mpi.Barrier()

# a host send queued behind a device send that is still
# gathering to the same peer (TEMPI's HostIsendOp) whose post the library
# refuses (a negative tag): MPI_Waitall returns MPI_ERR_IN_STATUS, the
# refused request's status carries the library's error, the device send's
# MPI_SUCCESS, and the device message still arrives. ONESHOT gathers 16 MiB
# into pinned host memory (milliseconds), so the gate is still closed when
# the host send is posted. (Two ranks or more: a send to itself may be
# matched by the self channel instead of gathering.)
if device and size >= 2:
    big_recipe = "vector(65536,256,512,byte)"
    bt, btemps, bbasic = typezoo.build(mpi, big_recipe)
    btm = pyoracle.TypeMap(big_recipe)
    borigin, blen = btm.geometry(1)
    bsrc = torch.from_numpy(np.random.default_rng(4000 + rank).integers(0, 256, blen, dtype=np.uint8)).cuda()
    bdst = torch.zeros(blen, dtype=torch.uint8, device="cuda")
    hb = np.zeros(64, dtype=np.uint8)
    torch.cuda.synchronize()
    mpi.set_datatype_method(1)  # ONESHOT
    r = mpi.Irecv(bdst.data_ptr() + borigin, 1, bt, src, 64)
    mpi.Barrier()
    c0 = mpi.counters()["lib_sends"]
    s_dev = mpi.Isend(bsrc.data_ptr() + borigin, 1, bt, peer, 64)
    try:
        s_host = mpi.Isend(hb.ctypes.data, 64, mpi.BYTE, peer, -5)
    except tempi_amd.mpi.MPIError:
        s_host = None
        fail("the host send behind a gathering send was refused at the call, not queued")
    if s_host is not None:
        rc, errs = mpi.Waitall_errors([s_dev, s_host])
        if rc != mpi.const("MPI_ERR_IN_STATUS") or errs[0] != mpi.SUCCESS or errs[1] == mpi.SUCCESS:
            fail(f"queued host send refused by the library: Waitall rc {rc}, status errors {errs}")
    mpi.Wait(r)
    exp = btm.pack(np.random.default_rng(4000 + src).integers(0, 256, blen, dtype=np.uint8), borigin, 1)
    got = btm.pack(bdst.cpu().numpy(), borigin, 1)
    if not np.array_equal(got, exp):
        fail("the device send beside a refused host send did not arrive intact")
    forced = [k for k, v in (("ONESHOT", 1), ("DEVICE", 2), ("STAGED", 3), ("IPC", 4))
              if "TEMPI_DATATYPE_" + k in os.environ]
    mpi.set_datatype_method({"ONESHOT": 1, "DEVICE": 2, "STAGED": 3, "IPC": 4}[forced[0]] if forced else 0)
    typezoo.free(mpi, bt, btemps, bbasic)
    mpi.Barrier()

# MPI_Sendrecv_replace whose receive side is MPI_PROC_NULL: the send of the
# (device) object still goes through TEMPI (it used to reach the
# library, which cannot read GPU memory), and the object is left as it was
sbuf, rbuf = buf(10), buf(11)
refill(sbuf, 9000 + rank)
r = mpi.Irecv(ptr(rbuf) + origin, count, t, src, 62)
mpi.Barrier()
mpi.Sendrecv_replace(ptr(sbuf) + origin, count, t, peer, 62, mpi.PROC_NULL, 62)
mpi.Wait(r)
check("sendrecv_replace to a peer from MPI_PROC_NULL", rbuf, 11, 9000 + src)
if not np.array_equal(host(sbuf), rand(9000 + rank)):
    fail("sendrecv_replace from MPI_PROC_NULL changed the object")
mpi.Barrier()

c = mpi.counters()
starts, sends = c["persistent_starts"], c["sends"]
if tempi_holds and starts < 4 * 4:
    fail(f"persistent_starts = {starts}")
if device and sends < 6:
    fail(f"device send modes not carried by TEMPI: sends = {sends}")
mpi.Buffer_detach()
typezoo.free(mpi, t, temps, basic)
total = mpi.Allreduce_double(float(errors), op=mpi.SUM)
if rank == 0:
    print(f"RESULT errors={int(total)} persistent_starts={starts} sends={sends}", flush=True)
mpi.Finalize()
sys.exit(1 if total else 0)
