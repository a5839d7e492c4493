"""Run under mpiexec -n 1 or -n 2: MPI's non-overtaking rule for sends that
take different routes to one peer. Each rank sends, all with one tag, in this
order: a strided device object (gathered on the GPU first), a host buffer (the
library at once), a device object of an irregular type (library-packed), and
a second strided device object; the peer's receives, posted in the same
order, must match them in that order. With one rank the messages go to self
(run it with TEMPI_NO_DIRECT=1 so the strided sends are gathered too).
--device puts the typed buffers on the GPU. Every byte is checked against the
oracle."""
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
TAG = 7
strided = "subarray(C,[40,38,512],[30,3,24],[5,3,24],byte)"
irregular = "hindexed([700,1100],[0,1000],byte)"
errors = 0


class Obj:
    def __init__(self, recipe, count):
        self.tm = pyoracle.TypeMap(recipe)
        self.count = count
        self.origin, self.buflen = self.tm.geometry(count)
        self.t, self.temps, self.basic = typezoo.build(mpi, recipe)

    def buf(self, seed):
        h = np.random.default_rng(seed).integers(0, 256, self.buflen, dtype=np.uint8)
        if device:
            return h, torch.from_numpy(h).cuda()
        return h, h.copy()

    def expected(self, canvas, seed):
        src = np.random.default_rng(seed).integers(0, 256, self.buflen, dtype=np.uint8)
        exp = canvas.copy()
        self.tm.unpack(self.tm.pack(src, self.origin, self.count), exp, self.origin, self.count)
        return exp


def ptr(b):
    return b.data_ptr() if device else b.ctypes.data


def host(b):
    if device and not isinstance(b, np.ndarray):
        torch.cuda.synchronize()
        return b.cpu().numpy()
    return b


S = Obj(strided, 2)
I = Obj(irregular, 3)
HOSTN = 4096

for it in range(20):
    base = 1000 * it + 100 * rank
    rbase = 1000 * it + 100 * src_rank
    sends = []
    keep = []
    # sends, in order: strided, host, irregular, strided
    plan = [(S, base + 1), (None, base + 2), (I, base + 3), (S, base + 4)]
    for obj, seed in plan:
        if obj is None:
            h = np.random.default_rng(seed).integers(0, 256, HOSTN, dtype=np.uint8)
            keep.append(h)
            sends.append(mpi.Isend(h.ctypes.data, HOSTN, mpi.BYTE, peer, TAG))
        else:
            _, d = obj.buf(seed)
            keep.append(d)
            sends.append(mpi.Isend(ptr(d) + obj.origin, obj.count, obj.t, peer, TAG))
    # every few rounds, alternate a blocking host send behind the gathers
    if it % 4 == 3:
        h = np.random.default_rng(base + 5).integers(0, 256, HOSTN, dtype=np.uint8)
        keep.append(h)
    recvs, checks = [], []
    for k, (obj, _) in enumerate(plan):
        seed = rbase + k + 1
        if obj is None:
            hb = np.zeros(HOSTN, dtype=np.uint8)
            recvs.append(mpi.Irecv(hb.ctypes.data, HOSTN, mpi.BYTE, src_rank, TAG))
            checks.append((hb, lambda b, s=seed: np.random.default_rng(s).integers(0, 256, HOSTN, dtype=np.uint8),
                           "host"))
        else:
            canvas, d = obj.buf(90000 + seed)
            recvs.append(mpi.Irecv(ptr(d) + obj.origin, obj.count, obj.t, src_rank, TAG))
            checks.append((d, lambda b, o=obj, c=canvas, s=seed: o.expected(c, s), "typed"))
    if it % 4 == 3:
        hb = np.zeros(HOSTN, dtype=np.uint8)
        if size == 1:
            r = mpi.Irecv(hb.ctypes.data, HOSTN, mpi.BYTE, src_rank, TAG + 1)
            mpi.Send(keep[-1].ctypes.data, HOSTN, mpi.BYTE, peer, TAG + 1)
            mpi.Wait(r)
        else:
            mpi.Send(keep[-1].ctypes.data, HOSTN, mpi.BYTE, peer, TAG + 1)
            mpi.Recv(hb.ctypes.data, HOSTN, mpi.BYTE, src_rank, TAG + 1)
        if not np.array_equal(hb, np.random.default_rng(rbase + 5).integers(0, 256, HOSTN, dtype=np.uint8)):
            errors += 1
            print(f"rank {rank} iter {it}: blocking host message wrong", flush=True)
    mpi.Waitall(sends + recvs)
    for k, (b, exp, what) in enumerate(checks):
        got = host(b)
        if not np.array_equal(got, exp(b)):
            errors += 1
            print(f"rank {rank} iter {it}: receive {k} ({what}) matched the wrong message", flush=True)

for o in (S, I):
    typezoo.free(mpi, o.t, o.temps, o.basic)
mpi.Finalize()
print(f"RESULT errors={errors}", flush=True)
sys.exit(1 if errors else 0)
