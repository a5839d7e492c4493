"""Run under mpiexec -n 2: at MPI_THREAD_MULTIPLE a
blocking host MPI_Recv must see a message another thread's probe took out
of the library.

Rank 1 starts two threads each round, with no application lock:
  A  MPI_Recv(0, tag A) into host memory: TEMPI's host receive, which waits
     in a loop that hands TEMPI's lock over between passes;
  B  MPI_Probe(0, tag B), then MPI_Recv(0, tag B) into a strided device
     object.
then tells rank 0 to send, and rank 0 sends A (1000 host bytes, tag A) and
right behind it B (a strided device object: a descriptor-sized message on
TEMPI's IPC / DIRECT routes). B's probe must receive A to look at B (the
non-overtaking rule) and keeps it; A's receive must then take it from what
is kept -- before the fix its loop only asked the library again and spun
forever (a hang: the join times out) or took a later message.
Every byte is checked. usage: probe_threads.py ROUNDS -> "RESULT errors=0" """
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)
import tempi_amd  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 100
import torch  # noqa: E402

torch.cuda.set_device(0)
mpi = tempi_amd.get_mpi()
provided = mpi.Init_thread(mpi.const("MPI_THREAD_MULTIPLE"))
rank, size = mpi.Comm_rank(), mpi.Comm_size()
assert size == 2, "probe_threads.py runs at 2 ranks"
errors = 0
if provided != mpi.const("MPI_THREAD_MULTIPLE"):
    errors += 1
    print(f"rank {rank}: provided {provided}", flush=True)
vec = mpi.Type_commit(mpi.Type_vector(16, 8, 24, mpi.BYTE))  # 128 packed bytes: a descriptor's size
EXT = 16 * 24


def payload(r, tag, n):
    return ((np.arange(n, dtype=np.int64) * 13 + r * 7 + tag * 5) & 0xFF).astype(np.uint8)


def fail(msg):
    global errors
    errors += 1
    print(f"rank {rank}: {msg}", flush=True)


for r in range(rounds):
    tag_a, tag_b = 100 + 2 * (r % 50), 101 + 2 * (r % 50)
    if rank == 0:
        go = np.zeros(1, dtype=np.uint8)
        mpi.Recv(go.ctypes.data, 1, mpi.BYTE, 1, 7)
        a = payload(r, tag_a, 1000)
        b = torch.from_numpy(payload(r, tag_b, EXT)).cuda()
        torch.cuda.synchronize()
        ra = mpi.Isend(a.ctypes.data, 1000, mpi.BYTE, 1, tag_a)
        rb = mpi.Isend(b.data_ptr(), 1, vec, 1, tag_b)
        mpi.Wait(ra)
        mpi.Wait(rb)
        continue
    got_a = np.zeros(1000, dtype=np.uint8)
    got_b = torch.zeros(EXT, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()

    def thread_a():
        mpi.Recv(got_a.ctypes.data, 1000, mpi.BYTE, 0, tag_a)

    def thread_b():
        mpi.Probe(0, tag_b, mpi.BYTE)
        mpi.Recv(got_b.data_ptr(), 1, vec, 0, tag_b)

    ts = [threading.Thread(target=thread_a, daemon=True), threading.Thread(target=thread_b, daemon=True)]
    for t in ts:
        t.start()
    time.sleep(0.002)  # both threads are waiting inside TEMPI
    go = np.ones(1, dtype=np.uint8)
    mpi.Send(go.ctypes.data, 1, mpi.BYTE, 0, 7)
    for t in ts:
        t.join(60)
    if any(t.is_alive() for t in ts):
        print(f"rank 1: round {r}: a receive never completed (hang)", flush=True)
        os._exit(3)
    if not np.array_equal(got_a, payload(r, tag_a, 1000)):
        fail(f"round {r}: host message A wrong")
    exp = payload(r, tag_b, EXT)
    mask = np.zeros(EXT, dtype=bool)
    for i in range(16):
        mask[i * 24:i * 24 + 8] = True
    gb = got_b.cpu().numpy()
    if not (np.array_equal(gb[mask], exp[mask]) and not gb[~mask].any()):
        fail(f"round {r}: device message B wrong")
mpi.Type_free(vec)
mpi.Finalize()
print(f"RESULT errors={errors}", flush=True)
