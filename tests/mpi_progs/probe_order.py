"""Run under mpiexec -n 1 or -n 2: MPI's non-overtaking rule across a probe
that has to receive a message to look at it. Every rank sends
its successor A (1000 B, tag 1), B (128 B = a descriptor's size, tag 2) and
C (160 B, tag 1), then:
  1. MPI_Iprobe(src, tag 2) finds B; MPI_Recv(src, MPI_ANY_TAG) must still
     return A, then B, then C;
  2. the same sends; MPI_Improbe(src, tag 2) claims B; MPI_Recv(src,
     MPI_ANY_TAG) returns A then C, and MPI_Mrecv returns B;
  3. the same sends; MPI_Probe(src, tag 2); MPI_Sendrecv_replace(src,
     MPI_ANY_TAG) must return A, MPI_Recv(ANY_TAG) B, then C. (The exchange's
     outgoing message has its receive posted beforehand: at one rank it goes
     to this same process, and MPICH completes a send to itself only once a
     receive matches it, so the program would hang with the library alone.)
With --device, B is a strided device object (a real descriptor on IPC /
DIRECT routes) received into host memory."""
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
rank, size = mpi.Comm_rank(), mpi.Comm_size()
peer, src = (rank + 1) % size, (rank - 1) % size
errors = 0
vec = mpi.Type_commit(mpi.Type_vector(16, 8, 24, mpi.BYTE))  # 128 packed bytes


def fail(msg):
    global errors
    errors += 1
    print(f"rank {rank}: {msg}", flush=True)


def payload(who, tag, n):
    return ((np.arange(n, dtype=np.int64) * 7 + who * 31 + tag * 11) & 0xFF).astype(np.uint8)


def send_three(round_):
    a = payload(rank, 1 + round_ * 10, 1000)
    c = payload(rank, 3 + round_ * 10, 160)
    b = payload(rank, 2 + round_ * 10, 16 * 24)  # the vector's extent; 128 bytes travel
    keep = [a, c, b]
    reqs = [mpi.Isend(a.ctypes.data, 1000, mpi.BYTE, peer, 1)]
    if device:
        bd = torch.from_numpy(b).cuda()
        torch.cuda.synchronize()
        keep.append(bd)
        reqs.append(mpi.Isend(bd.data_ptr(), 1, vec, peer, 2))
    else:
        reqs.append(mpi.Isend(b.ctypes.data, 1, vec, peer, 2))
    reqs.append(mpi.Isend(c.ctypes.data, 160, mpi.BYTE, peer, 1))
    return reqs, keep


def expect(round_, which):
    tag = {"A": 1, "B": 2, "C": 3}[which] + round_ * 10
    if which == "B":
        full = payload(src, tag, 16 * 24)
        return 2, full.reshape(16, 24)[:, :8].reshape(-1)
    return 1, payload(src, tag, 1000 if which == "A" else 160)


def check_recv(round_, which, got_src, got_tag, n, buf):
    etag, exp = expect(round_, which)
    if (got_src, got_tag, n) != (src, etag, exp.size) or not np.array_equal(buf[:n], exp):
        fail(f"round {round_}: expected {which} (tag {etag}, {exp.size} B) got tag {got_tag}, {n} B")


for round_ in range(3):
    reqs, keep = send_three(round_)
    buf = np.zeros(4096, dtype=np.uint8)
    if round_ == 0:
        while mpi.Iprobe(src, 2, mpi.BYTE) is None:
            pass
        order = "ABC"
        for which in order:
            s, t, n = mpi.Recv_status(buf.ctypes.data, 4096, mpi.BYTE, src, mpi.ANY_TAG)
            check_recv(round_, which, s, t, n, buf)
    elif round_ == 1:
        got = None
        while got is None:
            got = mpi.Improbe(src, 2, mpi.BYTE)
        msg, (s, t, n) = got
        if (t, n) != (2, 128):
            fail(f"improbe reported tag {t}, {n} B")
        for which in "AC":
            s, t, n = mpi.Recv_status(buf.ctypes.data, 4096, mpi.BYTE, src, mpi.ANY_TAG)
            check_recv(round_, which, s, t, n, buf)
        s, t, n = mpi.Mrecv(buf.ctypes.data, 4096, mpi.BYTE, msg)
        check_recv(round_, "B", s, t, n, buf)
    else:
        mpi.Probe(src, 2, mpi.BYTE)
        # the replace buffer sends 1000 bytes to peer, whose receive is posted first
        b7 = np.zeros(1000, dtype=np.uint8)
        r7 = mpi.Irecv(b7.ctypes.data, 1000, mpi.BYTE, src, 7)
        rep = payload(rank, 99, 1000)
        s, t, n = mpi.Sendrecv_replace(rep.ctypes.data, 1000, mpi.BYTE, peer, 7, src, mpi.ANY_TAG)
        check_recv(round_, "A", s, t, n, rep)
        for which in "BC":
            s, t, n = mpi.Recv_status(buf.ctypes.data, 4096, mpi.BYTE, src, mpi.ANY_TAG)
            check_recv(round_, which, s, t, n, buf)
        _, (s, t, n) = mpi.Wait_status(r7, mpi.BYTE)
        if (s, t, n) != (src, 7, 1000) or not np.array_equal(b7, payload(src, 99, 1000)):
            fail("Sendrecv_replace's outgoing message")
    mpi.Waitall(reqs)
    mpi.Barrier()
mpi.Type_free(vec)
print(f"RESULT errors={errors}", flush=True)
mpi.Finalize()
