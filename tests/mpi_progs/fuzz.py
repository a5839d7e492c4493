"""Run under mpiexec -n 2..4: a randomized mix of every route through the
transport. Each round every rank draws (from a seed all ranks share) a list
of messages for every (sender, receiver) pair, the receiver included:
strided or irregular types, counts from tiny to past the 128 KiB IPC COPY
limit, narrow and wide rows, device or host buffers on either side, tags from
a small set (so MPI's non-overtaking order between messages with one tag is
exercised). With --modes, also send modes (MPI_Isend / MPI_Issend /
MPI_Ibsend, and persistent MPI_Send_init + MPI_Start), receive kinds
(MPI_Irecv, persistent MPI_Recv_init + MPI_Start) and host receives of
device sends. Every rank posts its receives and sends in a random
interleaving, waits for all with one MPI_Waitall, and checks every received
byte against the oracle. --host keeps every buffer in host memory (no GPU
needed: the CPU suite runs it under TEMPI_TEST_HOST_ONLY so that a script
that cannot start fails there, not on the GPU box).
usage: fuzz.py [rounds] [seed] [--modes] [--host]"""
import os
import random
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)

import tempi_amd  # noqa: E402
from oracle import pyoracle  # noqa: E402
from tests import typezoo  # noqa: E402

host_only = "--host" in sys.argv
if not host_only:
    import torch

    torch.cuda.set_device(0)
mpi = tempi_amd.get_mpi()
mpi.Init()
rank, size = mpi.Comm_rank(), mpi.Comm_size()
modes = "--modes" in sys.argv
if modes:
    mpi.Buffer_attach(256 << 20)  # (MPI_Ibsend: every round's buffered sends fit)
argv = [a for a in sys.argv[1:] if a not in ("--modes", "--host")]
rounds = int(argv[0]) if len(argv) > 0 else 6
seed0 = int(argv[1]) if len(argv) > 1 else 7
errors = 0

# (recipe, element bytes): narrow rows, wide rows, contiguous, irregular
RECIPES = [
    "subarray(C,[40,38,512],[30,3,24],[5,3,24],byte)",      # 24-byte rows, 2160 B
    "subarray(C,[6,20,1100],[4,16,512],[1,2,64],byte)",     # 512-byte rows, 32 KiB
    "vector(64,256,300,byte)",                              # 256-byte rows, 16 KiB
    "contig(4096,byte)",                                    # contiguous, 4 KiB
    "hindexed([700,1100],[0,1000],byte)",                   # irregular (library-packed)
]
TYPES = [typezoo.build(mpi, r) for r in RECIPES]
MAPS = [pyoracle.TypeMap(r) for r in RECIPES]


def plan(rnd, src, dst):
    """the messages src sends to dst in round rnd (same on every rank)"""
    rng = random.Random(seed0 * 1000003 + rnd * 1009 + src * 31 + dst)
    msgs = []
    for k in range(rng.choice([0, 1, 2, 3, 5])):
        ti = rng.randrange(len(RECIPES))
        count = rng.choice([1, 2, 3, 9, 40]) if ti != 3 else rng.choice([1, 8, 40])
        sdev = rng.random() < 0.85
        if modes:
            # (host receives of device sends: descriptors landed by the host receive)
            rdev = rng.random() < (0.8 if sdev else 0.5)
            smode = rng.choice(["isend", "isend", "issend", "ibsend", "persist"])
            rkind = rng.choice(["irecv", "irecv", "persist"])
        else:
            rdev = True if sdev else rng.random() < 0.5
            smode, rkind = "isend", "irecv"
        if host_only:
            sdev = rdev = False
        msgs.append(dict(ti=ti, count=count, tag=rng.choice([3, 4]), sdev=sdev, rdev=rdev,
                         seed=rng.randrange(1 << 30), smode=smode, rkind=rkind))
    return msgs


def buffer(n, seed, dev):
    h = np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8)
    return h, (torch.from_numpy(h).cuda() if dev else h.copy())


def addr(b):
    return b.ctypes.data if isinstance(b, np.ndarray) else b.data_ptr()


def sync():
    if not host_only:
        torch.cuda.synchronize()


for rnd in range(rounds):
    ops, checks, keep = [], [], []
    for dst in range(size):
        for m in plan(rnd, rank, dst):
            tm = MAPS[m["ti"]]
            origin, n = tm.geometry(m["count"])
            _, b = buffer(n, m["seed"], m["sdev"])
            keep.append(b)
            ops.append((m["smode"], addr(b) + origin, m["count"], TYPES[m["ti"]][0], dst, m["tag"]))
    recvs_by_src = []
    for src in range(size):
        for m in plan(rnd, src, rank):
            tm = MAPS[m["ti"]]
            origin, n = tm.geometry(m["count"])
            canvas, b = buffer(n, m["seed"] ^ 0x5A5A, m["rdev"])
            src_bytes = np.random.default_rng(m["seed"]).integers(0, 256, n, dtype=np.uint8)
            exp = canvas.copy()
            tm.unpack(tm.pack(src_bytes, origin, m["count"]), exp, origin, m["count"])
            keep.append(b)
            recvs_by_src.append(("recv_" + m["rkind"], addr(b) + origin, m["count"], TYPES[m["ti"]][0], src,
                                 m["tag"]))
            checks.append((b, exp, f"round {rnd} {RECIPES[m['ti']][:22]} x{m['count']} from {src} tag {m['tag']}"))
    # a random interleaving that keeps each list's own order (MPI order per
    # (peer, tag) is what the messages are matched by)
    rng = random.Random(seed0 * 7 + rnd * 13 + rank)
    seq, i, j = [], 0, 0
    while i < len(ops) or j < len(recvs_by_src):
        if j >= len(recvs_by_src) or (i < len(ops) and rng.random() < 0.5):
            seq.append(ops[i])
            i += 1
        else:
            seq.append(recvs_by_src[j])
            j += 1
    sync()
    reqs, persistent = [], []
    for kind, p, count, t, peer, tag in seq:
        if kind == "isend":
            reqs.append(mpi.Isend(p, count, t, peer, tag))
        elif kind == "issend":
            reqs.append(mpi.Issend(p, count, t, peer, tag))
        elif kind == "ibsend":
            reqs.append(mpi.Ibsend(p, count, t, peer, tag))
        elif kind == "persist":
            r = mpi.Send_init(p, count, t, peer, tag)
            persistent.append(r)
            reqs.append(mpi.Start(r))
        elif kind == "recv_persist":
            r = mpi.Recv_init(p, count, t, peer, tag)
            persistent.append(r)
            reqs.append(mpi.Start(r))
        else:
            reqs.append(mpi.Irecv(p, count, t, peer, tag))
    mpi.Waitall(reqs)
    for r in persistent:
        mpi.Request_free(r)
    sync()
    for b, exp, what in checks:
        got = b if isinstance(b, np.ndarray) else b.cpu().numpy()
        if not np.array_equal(got, exp):
            errors += 1
            print(f"rank {rank}: {what}: bytes differ", flush=True)
    mpi.Barrier()

for t in TYPES:
    typezoo.free(mpi, *t)
if modes:
    mpi.Buffer_detach()
c = mpi.counters()
print(f"rank {rank} routes: direct={c['send_direct']} ipc={c['send_ipc']} copy={c['send_ipc_copy']} "
      f"oneshot={c['send_oneshot']} lib={c['lib_sends']}", flush=True)
mpi.Finalize()
print(f"RESULT errors={errors}", flush=True)
sys.exit(1 if errors else 0)
