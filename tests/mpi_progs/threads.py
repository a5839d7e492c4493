"""Run under mpiexec -n 1 or -n 2: the thread level TEMPI reports, and
several application threads calling MPI at that level.

MPI_Init_thread(REQUIRED) must report EXPECT, MPI_Query_thread the same:
MPI_THREAD_MULTIPLE when it was asked for (TEMPI's calls then run under one
process-wide lock, core/mt.hpp), at most MPI_THREAD_SERIALIZED otherwise,
and the library's own level with TEMPI_DISABLE=1.

Then THREADS threads each run ITERS content-checked rounds of strided
MPI_Isend / MPI_Irecv to the peer rank (itself at one rank):
  default       every MPI call under one Python lock -- what SERIALIZED
                allows: calls from any thread, never two at once; requests
                completed by MPI_Test polling while the other threads'
                requests are in flight;
  --concurrent  (MULTIPLE) no lock at all. Thread w sends with its own tag
                and receives the message thread w+1 sends, then blocks in
                MPI_Wait, so each wait depends on another thread getting into
                TEMPI while it waits; each round also blocks in a host
                MPI_Recv for a message another thread sends. A lock held
                through a wait deadlocks here (the run is killed by the test's
                timeout).
--device puts the strided objects on the GPU (each thread on the HIP device
it finds).
usage: threads.py REQUIRED EXPECT [THREADS ITERS] [--device] [--concurrent]"""
import os
import sys
import threading

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)

import tempi_amd  # noqa: E402
from oracle import pyoracle  # noqa: E402
from tests import typezoo  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
device = "--device" in sys.argv
concurrent = "--concurrent" in sys.argv
LEVELS = {"SINGLE": "THREAD_SINGLE", "FUNNELED": "THREAD_FUNNELED", "SERIALIZED": "THREAD_SERIALIZED",
          "MULTIPLE": "THREAD_MULTIPLE"}
mpi = tempi_amd.get_mpi()
level = {k: mpi.const("MPI_" + v) for k, v in LEVELS.items()}
required, expect = level[args[0]], level[args[1]]
threads_n = int(args[2]) if len(args) > 2 else 2
iters = int(args[3]) if len(args) > 3 else 500
if device:
    import torch

    torch.cuda.set_device(0)
provided = mpi.Init_thread(required)
rank, size = mpi.Comm_rank(), mpi.Comm_size()
errors = 0
if provided != expect:
    errors += 1
    print(f"rank {rank}: MPI_Init_thread({args[0]}) provided {provided}, expected {expect}", flush=True)
queried = mpi.Query_thread()
if queried != provided:
    errors += 1
    print(f"rank {rank}: MPI_Query_thread {queried} != provided {provided}", flush=True)

peer, src = (rank + 1) % size, (rank - 1) % size
big = threading.Lock()  # MPI_THREAD_SERIALIZED: one MPI call at a time
recipes = ["subarray(C,[40,38,64],[30,3,24],[5,3,24],byte)", "vector(64,24,96,byte)"]
types = [typezoo.build(mpi, r) for r in recipes]
maps = [pyoracle.TypeMap(r) for r in recipes]
counts = [2, 3]
werrors = [0] * threads_n
HOSTN = 256


def call(fn, *a):
    with big:
        return fn(*a)


def worker(w):
    # concurrent: this thread sends as w and receives what thread w+1 sends,
    # all threads with one shape; serialized: each thread with its own
    partner = (w + 1) % threads_n if concurrent else w
    k = 0 if concurrent else w % len(recipes)
    t, tm, count = types[k][0], maps[k], counts[k]
    origin, buflen = tm.geometry(count)
    for it in range(iters):
        seed = (w * 100003 + it) * 17
        pseed = (partner * 100003 + it) * 17
        hsend = np.random.default_rng(seed + rank).integers(0, 256, buflen, dtype=np.uint8)
        canvas = np.random.default_rng(seed + 7).integers(0, 256, buflen, dtype=np.uint8)
        if device:
            s, r = torch.from_numpy(hsend).cuda(), torch.from_numpy(canvas).cuda()
            torch.cuda.synchronize()
            sp, rp = s.data_ptr(), r.data_ptr()
        else:
            s, r = hsend, canvas.copy()
            sp, rp = s.ctypes.data, r.ctypes.data
        if concurrent:
            sq = mpi.Isend(sp + origin, count, t, peer, 100 + w)
            hs = np.random.default_rng(seed + 5 + rank).integers(0, 256, HOSTN, dtype=np.uint8)
            hq = mpi.Isend(hs.ctypes.data, HOSTN, mpi.BYTE, peer, 300 + w)
            rq = mpi.Irecv(rp + origin, count, t, src, 100 + partner)
            mpi.Wait(rq)  # blocks until thread `partner` of rank src has sent
            hr = np.zeros(HOSTN, dtype=np.uint8)
            mpi.Recv(hr.ctypes.data, HOSTN, mpi.BYTE, src, 300 + partner)  # blocking, in the library
            mpi.Wait(sq)
            mpi.Wait(hq)
            if not np.array_equal(hr, np.random.default_rng(pseed + 5 + src).integers(0, 256, HOSTN, dtype=np.uint8)):
                werrors[w] += 1
                if werrors[w] < 4:
                    print(f"rank {rank} thread {w} iter {it}: host message wrong", flush=True)
        else:
            tag = 100 + w  # one tag per thread: its messages pair up with the peer's same thread
            rq = call(mpi.Irecv, rp + origin, count, t, src, tag)
            sq = call(mpi.Isend, sp + origin, count, t, peer, tag)
            # completed by MPI_Test polling: a blocking MPI_Wait under the lock
            # would hold it while the peer's matching thread waits for this
            # process's other thread (a deadlock of the application's making)
            pending = [rq, sq] if it % 2 else [sq, rq]
            while pending:
                done, pending[0] = call(mpi.Test, pending[0])
                if done:
                    pending.pop(0)
        got = r.cpu().numpy() if device else r
        exp = canvas.copy()
        peer_src = np.random.default_rng(pseed + src).integers(0, 256, buflen, dtype=np.uint8)
        tm.unpack(tm.pack(peer_src, origin, count), exp, origin, count)
        if not np.array_equal(got, exp):
            werrors[w] += 1
            if werrors[w] < 4:
                print(f"rank {rank} thread {w} iter {it}: received object wrong", flush=True)


ths = [threading.Thread(target=worker, args=(w,)) for w in range(threads_n)]
for th in ths:
    th.start()
for th in ths:
    th.join()
errors += sum(werrors)
c = mpi.counters()
if device and os.environ.get("TEMPI_DISABLE") is None and c["isends"] < threads_n * iters:
    errors += 1
    print(f"rank {rank}: only {c['isends']} sends went through TEMPI", flush=True)
for t, temps, basic in types:
    typezoo.free(mpi, t, temps, basic)
mpi.Finalize()
print(f"RESULT errors={errors} provided={provided}", flush=True)
sys.exit(1 if errors else 0)
