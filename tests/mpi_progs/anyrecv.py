"""Run under mpiexec -n 1 or -n 2: every kind of receive an application can
post sees the payload of a device strided MPI_Isend, whichever route TEMPI
took for it (AUTO: ONESHOT below 4 KiB, an IPC slab descriptor at 8 KiB, an
IPC COPY descriptor at 1 MiB; at 1 rank a DIRECT descriptor). The last rank
receives what rank 0 sends with

  host MPI_Irecv (contiguous, in place; strided, staged), MPI_Probe +
  MPI_Get_count + MPI_Recv, MPI_Iprobe + MPI_Irecv, MPI_Probe twice,
  MPI_Mprobe + MPI_Mrecv (host and device), MPI_Improbe + MPI_Imrecv,
  MPI_Probe + device MPI_Irecv, MPI_Sendrecv into host memory

and every byte is checked against the oracle (oracle/typemap.c through
pyoracle). Then, with MPI_ERRORS_RETURN, a message larger than the receive
is reported as MPI_ERR_TRUNCATE on each kind of receive, and the buffer is
left as it was. Reference wire format: /root/reference/src/internal/
sender.cpp:109,161 and async_operation.cpp:127,261 (always MPI_PACKED bytes)."""
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
rank, size = mpi.Comm_rank(), mpi.Comm_size()
SENDER, RECEIVER = 0, size - 1
errors = 0


def fail(msg):
    global errors
    errors += 1
    print(f"rank {rank}: {msg}", flush=True)


def payload_of(recipe, count, seed):
    tm = pyoracle.TypeMap(recipe)
    origin, buflen = tm.geometry(count)
    src = np.random.default_rng(seed).integers(0, 256, buflen, dtype=np.uint8)
    return tm, origin, buflen, src, tm.pack(src, origin, count)


# 256-byte rows at stride 512: 96 B is a partial row (ONESHOT), 8 KiB an IPC
# slab, 1 MiB an IPC COPY (wide rows, above the eager limit)
SIZES = {"96B": "vector(1,96,512,byte)", "8KiB": "vector(32,256,512,byte)", "1MiB": "vector(4096,256,512,byte)"}
KINDS = ["irecv_host_contig", "irecv_host_strided", "probe_recv", "iprobe_irecv", "probe_twice",
         "mprobe_mrecv_host", "mprobe_mrecv_dev", "improbe_imrecv_host", "probe_irecv_dev", "sendrecv_host"]

case = 0
for label, recipe in SIZES.items():
    for kind in KINDS:
        case += 1
        tag = 100 + case
        seed = 1000 + case
        tm, origin, buflen, src, packed = payload_of(recipe, 1, seed)
        n = packed.size
        t, temps, basic = typezoo.build(mpi, recipe)
        sreq = None
        if rank == SENDER and kind != "sendrecv_host":
            s_dev = torch.from_numpy(src).cuda()
            torch.cuda.synchronize()
            sreq = mpi.Isend(s_dev.data_ptr() + origin, 1, t, RECEIVER, tag)
        if rank == SENDER and kind == "sendrecv_host" and size > 1:
            s_dev = torch.from_numpy(src).cuda()
            torch.cuda.synchronize()
            mpi.Send(s_dev.data_ptr() + origin, 1, t, RECEIVER, tag)
        if rank == RECEIVER:
            where = f"{label} {kind}"
            print(f"case {where}", flush=True)
            got = None  # the packed bytes that arrived, or the strided canvas
            canvas = np.random.default_rng(seed + 7).integers(0, 256, buflen, dtype=np.uint8)
            exp_canvas = canvas.copy()
            tm.unpack(packed, exp_canvas, origin, 1)
            contig = np.zeros(n + 64, dtype=np.uint8)  # room beyond the payload stays zero
            if kind == "irecv_host_contig":
                _, st = mpi.Wait_status(mpi.Irecv(contig.ctypes.data, n + 64, mpi.BYTE, SENDER, tag), mpi.BYTE)
                got = contig
                if st[2] != n:
                    fail(f"{where}: MPI_Get_count {st[2]} != {n}")
            elif kind == "irecv_host_strided":
                h = canvas.copy()
                _, st = mpi.Wait_status(mpi.Irecv(h.ctypes.data + origin, 1, t, SENDER, tag), t)
                got = h
                if st[2] != 1:
                    fail(f"{where}: MPI_Get_count {st[2]} != 1")
            elif kind in ("probe_recv", "probe_twice"):
                s0, tg, cnt = mpi.Probe(mpi.ANY_SOURCE, mpi.ANY_TAG, mpi.BYTE)
                if kind == "probe_twice":
                    again = mpi.Probe(SENDER, tag, mpi.BYTE)
                    if again != (s0, tg, cnt):
                        fail(f"{where}: second probe {again} != {(s0, tg, cnt)}")
                if (s0, tg, cnt) != (SENDER, tag, n):
                    fail(f"{where}: probe {(s0, tg, cnt)} != {(SENDER, tag, n)}")
                _, _, c2 = mpi.Probe(SENDER, tag, t)  # MPI_Get_count in the sender's type
                if c2 != 1:
                    fail(f"{where}: MPI_Get_count(type) {c2} != 1")
                st = mpi.Recv_status(contig.ctypes.data, cnt, mpi.BYTE, s0, tg)
                got = contig
                if st[2] != n:
                    fail(f"{where}: received count {st[2]} != {n}")
            elif kind == "iprobe_irecv":
                st = None
                while st is None:
                    st = mpi.Iprobe(SENDER, mpi.ANY_TAG, mpi.BYTE)
                if st != (SENDER, tag, n):
                    fail(f"{where}: iprobe {st} != {(SENDER, tag, n)}")
                h = canvas.copy()
                mpi.Wait(mpi.Irecv(h.ctypes.data + origin, 1, t, SENDER, tag))
                got = h
            elif kind == "mprobe_mrecv_host":
                m, st = mpi.Mprobe(SENDER, tag, mpi.BYTE)
                if st != (SENDER, tag, n):
                    fail(f"{where}: mprobe {st} != {(SENDER, tag, n)}")
                st2 = mpi.Mrecv(contig.ctypes.data, st[2], mpi.BYTE, m)
                got = contig
                if st2[2] != n:
                    fail(f"{where}: mrecv count {st2[2]} != {n}")
            elif kind == "mprobe_mrecv_dev":
                m, st = mpi.Mprobe(mpi.ANY_SOURCE, tag, t)
                if st != (SENDER, tag, 1):
                    fail(f"{where}: mprobe {st} != {(SENDER, tag, 1)}")
                d = torch.from_numpy(canvas).cuda()
                torch.cuda.synchronize()
                st2 = mpi.Mrecv(d.data_ptr() + origin, 1, t, m)
                torch.cuda.synchronize()
                got = d.cpu().numpy()
                if st2 != (SENDER, tag, 1):
                    fail(f"{where}: mrecv status {st2}")
            elif kind == "improbe_imrecv_host":
                r = None
                while r is None:
                    r = mpi.Improbe(SENDER, tag, t)
                m, st = r
                if st != (SENDER, tag, 1):
                    fail(f"{where}: improbe {st}")
                h = canvas.copy()
                _, st2 = mpi.Wait_status(mpi.Imrecv(h.ctypes.data + origin, 1, t, m), t)
                got = h
                if st2 != (SENDER, tag, 1):
                    fail(f"{where}: imrecv status {st2}")
            elif kind == "probe_irecv_dev":
                st = mpi.Probe(SENDER, tag, mpi.BYTE)
                if st != (SENDER, tag, n):
                    fail(f"{where}: probe {st}")
                d = torch.from_numpy(canvas).cuda()
                torch.cuda.synchronize()
                mpi.Wait(mpi.Irecv(d.data_ptr() + origin, 1, t, SENDER, tag))
                torch.cuda.synchronize()
                got = d.cpu().numpy()
            elif kind == "sendrecv_host":
                # at 1 rank the device send is this call's own send side
                if size == 1:
                    s_dev = torch.from_numpy(src).cuda()
                    torch.cuda.synchronize()
                    st = mpi.Sendrecv(s_dev.data_ptr() + origin, 1, t, RECEIVER, tag, contig.ctypes.data, n + 64,
                                      mpi.BYTE, SENDER, tag)
                else:
                    st = mpi.Sendrecv(0, 0, mpi.BYTE, mpi.PROC_NULL, 0, contig.ctypes.data, n + 64, mpi.BYTE,
                                      SENDER, tag)
                got = contig
                if st != (SENDER, tag, n):
                    fail(f"{where}: sendrecv status {st}")
            if got is contig:
                if not np.array_equal(contig[:n], packed) or contig[n:].any():
                    bad = np.flatnonzero(contig[:n] != packed)
                    fail(f"{where}: packed bytes differ at {bad[:8]} (of {bad.size})")
            elif got is not None and not np.array_equal(got, exp_canvas):
                bad = np.flatnonzero(got != exp_canvas)
                fail(f"{where}: unpacked bytes differ at {bad[:8]} (of {bad.size})")
        if sreq is not None:
            mpi.Wait(sreq)
        typezoo.free(mpi, t, temps, basic)
        mpi.Barrier()

# --- truncation: 2 elements sent, 1 allowed; every receive kind returns
# MPI_ERR_TRUNCATE with the buffer untouched (MPI_ERRORS_RETURN)
mpi.Comm_set_errhandler(mpi.ERRORS_RETURN)
TRUNC = ["irecv_dev", "recv_dev", "irecv_host", "recv_host"]
for label, recipe in SIZES.items():
    for kind in TRUNC:
        case += 1
        tag = 100 + case
        tm, origin, buflen, src, packed = payload_of(recipe, 2, 5000 + case)
        t, temps, basic = typezoo.build(mpi, recipe)
        sreq = None
        if rank == SENDER:
            s_dev = torch.from_numpy(src).cuda()
            torch.cuda.synchronize()
            sreq = mpi.Isend(s_dev.data_ptr() + origin, 2, t, RECEIVER, tag)
        if rank == RECEIVER:
            where = f"truncation {label} {kind}"
            print(f"case {where}", flush=True)
            canvas = np.random.default_rng(case).integers(0, 256, buflen, dtype=np.uint8)
            if kind.endswith("dev"):
                d = torch.from_numpy(canvas).cuda()
                torch.cuda.synchronize()
                if kind == "irecv_dev":
                    rc, err = mpi.Wait_rc(mpi.Irecv(d.data_ptr() + origin, 1, t, SENDER, tag))
                else:
                    rc = err = mpi.Recv_rc(d.data_ptr() + origin, 1, t, SENDER, tag)
                torch.cuda.synchronize()
                after = d.cpu().numpy()
            else:
                h = canvas.copy()
                if kind == "irecv_host":
                    rc, err = mpi.Wait_rc(mpi.Irecv(h.ctypes.data + origin, 1, t, SENDER, tag))
                else:
                    rc = err = mpi.Recv_rc(h.ctypes.data + origin, 1, t, SENDER, tag)
                after = h
            # the library's truncation code carries an error class of
            # MPI_ERR_TRUNCATE in its low bits (MPICH adds details above)
            if rc == mpi.SUCCESS or (rc & 0x7F) != mpi.ERR_TRUNCATE or (err & 0x7F) != mpi.ERR_TRUNCATE:
                fail(f"{where}: rc {rc} status error {err}, expected MPI_ERR_TRUNCATE ({mpi.ERR_TRUNCATE})")
            # only what TEMPI carried is guaranteed untouched (the library may
            # write the part that fits into a host buffer it received into)
            if kind.endswith("dev") and not np.array_equal(after, canvas):
                fail(f"{where}: a truncated receive wrote its buffer")
        if sreq is not None:
            mpi.Wait(sreq)
        typezoo.free(mpi, t, temps, basic)
        mpi.Barrier()

c = mpi.counters()
# (one write with its newline: the ranks share the launcher's pipe)
sys.stdout.write(f"rank {rank} counters ipc={c['send_ipc']} ipc_copy={c['send_ipc_copy']} direct={c['send_direct']} "
                 f"oneshot={c['send_oneshot']} canary_ok={c['canary_ok']} canary_fail={c['canary_fail']}\n")
sys.stdout.flush()
mpi.Finalize()
print(f"RESULT errors={errors}", flush=True)
sys.exit(1 if errors else 0)
