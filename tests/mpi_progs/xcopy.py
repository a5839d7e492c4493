"""Run under mpiexec -n 2 with TEMPI_IPC_COPY_MIN_BYTES / _MIN_BLOCK lowered:
IPC COPY (the receiver copies straight out of the sender's object) against
every kind of receiver. Rank 0 sends, rank 1 receives, for each case:
  same      the same strided type on both sides (the copy kernel)
  reshape   another strided shape of the same size (the copy kernel)
  deep      a receive type of more dimensions than the copy kernel takes
            (NACK: the sender gathers and sends the bytes through the host)
  host      a blocking host-buffer MPI_Recv (the descriptor is landed; a
            non-blocking host receive of a TEMPI IPC message is unsupported,
            INTEGRATION.md)
  blocking  a blocking device MPI_Recv
  reuse     the same send buffer rewritten and sent again (no stale bytes)
  realloc   the send buffer freed back to HIP and a new one allocated (maybe
            at the same address) before each send: the receiver must map the
            new allocation, not reuse the old mapping
Every received byte is checked against the oracle; counters are printed."""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)

import tempi_amd  # noqa: E402
from oracle import pyoracle  # noqa: E402
from tests import typezoo  # noqa: E402

import torch  # noqa: E402

torch.cuda.set_device(0)
mpi = tempi_amd.get_mpi()
mpi.Init()
rank, size = mpi.Comm_rank(), mpi.Comm_size()
assert size == 2
errors = 0

SEND = "subarray(C,[6,20,1100],[4,16,512],[1,2,64],byte)"  # 4 x 16 rows of 512 B = 32 KiB
CASES = [
    ("same", SEND, SEND, 1),
    ("reshape", SEND, "vector(128,256,300,byte)", 1),
    ("deep", SEND, "hvector(2,1,70000,hvector(2,1,30000,hvector(2,1,9000,vector(16,256,512,byte))))", 1),
    ("host", SEND, SEND, 1),
    ("blocking", SEND, SEND, 1),
    ("reuse", SEND, SEND, 3),
    ("realloc", SEND, SEND, 8),
]


def fail(msg):
    global errors
    errors += 1
    print(f"rank {rank}: {msg}", flush=True)


stm = pyoracle.TypeMap(SEND)
so, slen = stm.geometry(1)
st, stemps, sbasic = typezoo.build(mpi, SEND)
sbuf = torch.zeros(slen, dtype=torch.uint8, device="cuda")
for ci, (name, _, rrecipe, reps) in enumerate(CASES):
    rtm = pyoracle.TypeMap(rrecipe)
    if rtm.size != stm.size:
        raise SystemExit(f"case {name}: sizes differ ({rtm.size} vs {stm.size})")
    ro, rlen = rtm.geometry(1)
    rt, rtemps, rbasic = typezoo.build(mpi, rrecipe)
    prev = None
    for rep in range(reps):
        seed = 1000 * ci + rep
        src = np.random.default_rng(seed).integers(0, 256, slen, dtype=np.uint8)
        if rank == 0:
            if name == "realloc":
                del sbuf
                torch.cuda.synchronize()
                torch.cuda.empty_cache()  # the block goes back to hipFree
                sbuf = torch.zeros(slen, dtype=torch.uint8, device="cuda")
            sbuf.copy_(torch.from_numpy(src))
            torch.cuda.synchronize()
            mpi.Wait(mpi.Isend(sbuf.data_ptr() + so, 1, st, 1, 50 + ci))
        else:
            canvas = np.random.default_rng(seed + 7).integers(0, 256, rlen, dtype=np.uint8)
            exp = canvas.copy()
            rtm.unpack(stm.pack(src, so, 1), exp, ro, 1)
            if name == "host":
                hb = canvas.copy()
                mpi.Recv(hb.ctypes.data + ro, 1, rt, 0, 50 + ci)
                got = hb
            else:
                dbuf = torch.from_numpy(canvas).cuda()
                if name == "blocking":
                    mpi.Recv(dbuf.data_ptr() + ro, 1, rt, 0, 50 + ci)
                else:
                    mpi.Wait(mpi.Irecv(dbuf.data_ptr() + ro, 1, rt, 0, 50 + ci))
                torch.cuda.synchronize()
                got = dbuf.cpu().numpy()
            if not np.array_equal(got, exp):
                stale = prev is not None and np.array_equal(rtm.pack(got, ro, 1), prev)
                diff = np.flatnonzero(got != exp)
                gp, ep = rtm.pack(got, ro, 1), rtm.pack(exp, ro, 1)
                pd = np.flatnonzero(gp != ep)
                zeros = int(np.count_nonzero(gp[pd] == 0))
                unwritten = int(np.count_nonzero(gp[pd] == rtm.pack(canvas, ro, 1)[pd]))
                fail(f"case {name} rep {rep}: received bytes differ" + (" (the previous message's)" if stale else "")
                     + f" [{diff.size} bytes, {pd.size} of the payload at packed offsets {pd[:1].tolist()}..{pd[-1:].tolist()}"
                     f": {zeros} zero, {unwritten} still the canvas; outside the payload {diff.size - pd.size}]")
            prev = stm.pack(src, so, 1)
    typezoo.free(mpi, rt, rtemps, rbasic)
typezoo.free(mpi, st, stemps, sbasic)
c = mpi.counters()
print(f"rank {rank} counters ipc_copy={c['send_ipc_copy']} resends={c['copy_resends']} ipc={c['send_ipc']} "
      f"replaced={c['ipc_maps_replaced']}",
      flush=True)
mpi.Finalize()
print(f"RESULT errors={errors}", flush=True)
sys.exit(1 if errors else 0)
