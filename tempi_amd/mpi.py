"""ctypes binding of libtempi.so: the MPI C API as TEMPI exports it.

Every call goes through libtempi.so, so interposed functions (MPI_Pack,
MPI_Send, ...) run TEMPI's code and everything else resolves to the MPI
library libtempi.so was linked against (MPICH ABI: handles are C ints).
Buffers are raw addresses (ints): pass ``tensor.data_ptr()`` for GPU memory
or ``array.ctypes.data`` for host memory.
"""
import ctypes
import os

from . import LIBTEMPI, require_built

_singleton = None


class MPIError(RuntimeError):
    def __init__(self, fn, code):
        super().__init__(f"{fn} returned MPI error {code}")
        self.code = code


class TypeInfo(ctypes.Structure):
    _fields_ = [
        ("known", ctypes.c_int32),
        ("valid", ctypes.c_int32),
        ("ndims", ctypes.c_int32),
        ("pad_", ctypes.c_int32),
        ("start", ctypes.c_int64),
        ("block", ctypes.c_int64),
        ("size", ctypes.c_int64),
        ("lb", ctypes.c_int64),
        ("extent", ctypes.c_int64),
        ("counts", ctypes.c_int64 * 16),
        ("strides", ctypes.c_int64 * 16),
    ]


_COUNTER_FIELDS = [
    "packs", "unpacks", "pack_bytes", "unpack_bytes", "launches", "lib_packs", "lib_unpacks",
    "sends", "recvs", "isends", "irecvs", "send_device", "send_oneshot", "send_staged",
    "send_ipc", "lib_sends", "lib_recvs", "send_direct", "direct_fallbacks",
    "neighbor_colls", "send_ipc_copy", "copy_resends", "ipc_maps_replaced", "canary_ok", "canary_fail",
    "self_matched", "staged_packs", "staged_unpacks", "ticket_waits", "sync_waits",
    "ticket_batches", "persistent_starts", "batches", "gpu_inflight_ns",
    "bytes_ipc", "bytes_ipc_copy", "bytes_oneshot", "bytes_staged", "bytes_device", "bytes_direct",
]


class Counters(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in _COUNTER_FIELDS]


class KernelTimes(ctypes.Structure):
    _fields_ = [("pack_ms", ctypes.c_double), ("unpack_ms", ctypes.c_double),
                ("packs", ctypes.c_uint64), ("unpacks", ctypes.c_uint64)]


class MPI:
    """Thin wrapper: one method per MPI call used by tests / benchmarks."""

    def __init__(self, path=LIBTEMPI):
        require_built()
        self.L = ctypes.CDLL(path, mode=os.RTLD_NOW | ctypes.RTLD_GLOBAL)
        L = self.L
        L.tempi_mpi_constant.restype = ctypes.c_int64
        L.tempi_mpi_constant.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]
        for name in ("MPI_Datatype", "MPI_Comm", "MPI_Request", "MPI_Aint", "MPI_Op"):
            assert self.const(f"sizeof({name})") in (4, 8)
        self.Handle = ctypes.c_int if self.const("sizeof(MPI_Datatype)") == 4 else ctypes.c_int64
        self.Request = ctypes.c_int if self.const("sizeof(MPI_Request)") == 4 else ctypes.c_int64
        self.Aint = ctypes.c_int64
        self.status_size = self.const("sizeof(MPI_Status)")
        for n in ("BYTE", "CHAR", "SHORT", "INT", "LONG", "FLOAT", "DOUBLE", "PACKED", "INT64_T",
                  "UINT8_T", "COMM_WORLD", "COMM_SELF", "REQUEST_NULL", "ORDER_C", "ORDER_FORTRAN",
                  "SUCCESS", "ERR_TRUNCATE", "ANY_SOURCE", "ANY_TAG", "SUM", "MAX", "MIN",
                  "DATATYPE_NULL", "PROC_NULL", "UNDEFINED", "ERRORS_RETURN", "ERRORS_ARE_FATAL"):
            setattr(self, n, self.const("MPI_" + n))
        self.STATUS_IGNORE = ctypes.c_void_p(self.const("MPI_STATUS_IGNORE"))
        self.STATUSES_IGNORE = ctypes.c_void_p(self.const("MPI_STATUSES_IGNORE"))
        self.IN_PLACE = ctypes.c_void_p(self.const("MPI_IN_PLACE"))
        L.tempi_type_describe.argtypes = [ctypes.c_int64, ctypes.POINTER(TypeInfo)]
        L.tempi_get_stream.restype = ctypes.c_void_p
        L.tempi_get_stream.argtypes = [ctypes.c_int]
        L.tempi_version.restype = ctypes.c_char_p
        L.MPI_Wtime.restype = ctypes.c_double
        L.tempi_partition.restype = ctypes.c_int64
        I = ctypes.POINTER(ctypes.c_int)
        L.tempi_partition.argtypes = [ctypes.c_int, I, I, I, ctypes.c_int, I, ctypes.c_int, I]
        L.tempi_placement_info.argtypes = [ctypes.POINTER(ctypes.c_int64)]
        self.initialized = False

    # ------------------------------------------------------------- plumbing
    def const(self, name):
        found = ctypes.c_int(0)
        v = self.L.tempi_mpi_constant(name.encode(), ctypes.byref(found))
        if not found.value:
            raise KeyError(name)
        return v

    def _chk(self, fn, rc):
        if rc != 0:
            raise MPIError(fn, rc)

    def _call(self, fn, *args):
        rc = getattr(self.L, fn)(*args)
        self._chk(fn, rc)

    def h(self, v):
        return self.Handle(v)

    # ------------------------------------------------------------ lifecycle
    def Init(self):
        if not self.initialized:
            self._call("MPI_Init", None, None)
            self.initialized = True

    def Init_thread(self, required):
        """MPI_Init_thread; returns the level provided"""
        p = ctypes.c_int(-1)
        if not self.initialized:
            self._call("MPI_Init_thread", None, None, int(required), ctypes.byref(p))
            self.initialized = True
        return p.value

    def Query_thread(self):
        p = ctypes.c_int(-1)
        self._call("MPI_Query_thread", ctypes.byref(p))
        return p.value

    def Finalize(self):
        if self.initialized:
            self._call("MPI_Finalize")
            self.initialized = False

    def Initialized(self):
        f = ctypes.c_int(0)
        self._call("MPI_Initialized", ctypes.byref(f))
        return bool(f.value)

    def Comm_rank(self, comm=None):
        r = ctypes.c_int()
        self._call("MPI_Comm_rank", self.h(self.COMM_WORLD if comm is None else comm), ctypes.byref(r))
        return r.value

    def Comm_size(self, comm=None):
        r = ctypes.c_int()
        self._call("MPI_Comm_size", self.h(self.COMM_WORLD if comm is None else comm), ctypes.byref(r))
        return r.value

    def Barrier(self, comm=None):
        self._call("MPI_Barrier", self.h(self.COMM_WORLD if comm is None else comm))

    def Wtime(self):
        return self.L.MPI_Wtime()

    def Allreduce_double(self, value, op=None, comm=None):
        x = ctypes.c_double(value)
        y = ctypes.c_double()
        self._call("MPI_Allreduce", ctypes.byref(x), ctypes.byref(y), 1, self.h(self.DOUBLE),
                   self.h(self.MAX if op is None else op), self.h(self.COMM_WORLD if comm is None else comm))
        return y.value

    # ----------------------------------------------------------- datatypes
    def _newtype(self, fn, *args):
        out = self.Handle()
        self._call(fn, *args, ctypes.byref(out))
        return out.value

    def Type_contiguous(self, n, old):
        return self._newtype("MPI_Type_contiguous", n, self.h(old))

    def Type_vector(self, n, bl, stride, old):
        return self._newtype("MPI_Type_vector", n, bl, stride, self.h(old))

    def Type_create_hvector(self, n, bl, stride, old):
        return self._newtype("MPI_Type_create_hvector", n, bl, self.Aint(stride), self.h(old))

    def Type_create_subarray(self, sizes, subsizes, starts, order, old):
        n = len(sizes)
        A = ctypes.c_int * n
        return self._newtype("MPI_Type_create_subarray", n, A(*sizes), A(*subsizes), A(*starts), order,
                             self.h(old))

    def Type_create_resized(self, old, lb, extent):
        return self._newtype("MPI_Type_create_resized", self.h(old), self.Aint(lb), self.Aint(extent))

    def Type_dup(self, old):
        return self._newtype("MPI_Type_dup", self.h(old))

    def Type_indexed(self, bls, disps, old):
        n = len(bls)
        A = ctypes.c_int * max(n, 1)
        return self._newtype("MPI_Type_indexed", n, A(*bls), A(*disps), self.h(old))

    def Type_create_hindexed(self, bls, disps, old):
        n = len(bls)
        return self._newtype("MPI_Type_create_hindexed", n, (ctypes.c_int * max(n, 1))(*bls),
                             (ctypes.c_int64 * max(n, 1))(*disps), self.h(old))

    def Type_create_struct(self, bls, disps, types):
        n = len(bls)
        return self._newtype("MPI_Type_create_struct", n, (ctypes.c_int * max(n, 1))(*bls),
                             (ctypes.c_int64 * max(n, 1))(*disps),
                             (self.Handle * max(n, 1))(*[self.h(t).value for t in types]))

    def Type_create_indexed_block(self, bl, disps, old):
        n = len(disps)
        return self._newtype("MPI_Type_create_indexed_block", n, bl, (ctypes.c_int * max(n, 1))(*disps),
                             self.h(old))

    def Type_create_hindexed_block(self, bl, disps, old):
        n = len(disps)
        return self._newtype("MPI_Type_create_hindexed_block", n, bl, (ctypes.c_int64 * max(n, 1))(*disps),
                             self.h(old))

    def Type_commit(self, t):
        x = self.Handle(t)
        self._call("MPI_Type_commit", ctypes.byref(x))
        return x.value

    def Type_free(self, t):
        x = self.Handle(t)
        self._call("MPI_Type_free", ctypes.byref(x))

    def Type_size(self, t):
        s = ctypes.c_int()
        self._call("MPI_Type_size", self.h(t), ctypes.byref(s))
        return s.value

    def Type_get_extent(self, t):
        lb, ext = self.Aint(), self.Aint()
        self._call("MPI_Type_get_extent", self.h(t), ctypes.byref(lb), ctypes.byref(ext))
        return lb.value, ext.value

    def Type_get_true_extent(self, t):
        lb, ext = self.Aint(), self.Aint()
        self._call("MPI_Type_get_true_extent", self.h(t), ctypes.byref(lb), ctypes.byref(ext))
        return lb.value, ext.value

    # ---------------------------------------------------------- pack path
    def Pack_size(self, count, t, comm=None):
        s = ctypes.c_int()
        self._call("MPI_Pack_size", count, self.h(t), self.h(self.COMM_WORLD if comm is None else comm),
                   ctypes.byref(s))
        return s.value

    def Pack(self, inbuf, incount, t, outbuf, outsize, position=0, comm=None):
        """returns the new position"""
        pos = ctypes.c_int(position)
        self._call("MPI_Pack", ctypes.c_void_p(inbuf), incount, self.h(t), ctypes.c_void_p(outbuf), outsize,
                   ctypes.byref(pos), self.h(self.COMM_WORLD if comm is None else comm))
        return pos.value

    def Unpack(self, inbuf, insize, position, outbuf, outcount, t, comm=None):
        pos = ctypes.c_int(position)
        self._call("MPI_Unpack", ctypes.c_void_p(inbuf), insize, ctypes.byref(pos), ctypes.c_void_p(outbuf),
                   outcount, self.h(t), self.h(self.COMM_WORLD if comm is None else comm))
        return pos.value

    def Pack_rc(self, inbuf, incount, t, outbuf, outsize, position=0, comm=None):
        """MPI_Pack returning (rc, position) without raising"""
        pos = ctypes.c_int(position)
        rc = self.L.MPI_Pack(ctypes.c_void_p(inbuf), incount, self.h(t), ctypes.c_void_p(outbuf), outsize,
                             ctypes.byref(pos), self.h(self.COMM_WORLD if comm is None else comm))
        return rc, pos.value

    # ------------------------------------------------------ point to point
    def _status(self):
        return (ctypes.c_char * self.status_size)()

    def Send(self, buf, count, t, dest, tag, comm=None):
        self._call("MPI_Send", ctypes.c_void_p(buf), count, self.h(t), dest, tag,
                   self.h(self.COMM_WORLD if comm is None else comm))

    def Recv(self, buf, count, t, source, tag, comm=None):
        self._call("MPI_Recv", ctypes.c_void_p(buf), count, self.h(t), source, tag,
                   self.h(self.COMM_WORLD if comm is None else comm), self.STATUS_IGNORE)

    def Isend(self, buf, count, t, dest, tag, comm=None):
        r = self.Request()
        self._call("MPI_Isend", ctypes.c_void_p(buf), count, self.h(t), dest, tag,
                   self.h(self.COMM_WORLD if comm is None else comm), ctypes.byref(r))
        return r.value

    def Irecv(self, buf, count, t, source, tag, comm=None):
        r = self.Request()
        self._call("MPI_Irecv", ctypes.c_void_p(buf), count, self.h(t), source, tag,
                   self.h(self.COMM_WORLD if comm is None else comm), ctypes.byref(r))
        return r.value

    # send modes (device objects: TEMPI's transport with the library call of
    # the same mode)
    def _mode_send(self, fn, buf, count, t, dest, tag, comm, nonblocking):
        comm = self.h(self.COMM_WORLD if comm is None else comm)
        if not nonblocking:
            self._call(fn, ctypes.c_void_p(buf), count, self.h(t), dest, tag, comm)
            return None
        r = self.Request()
        self._call(fn, ctypes.c_void_p(buf), count, self.h(t), dest, tag, comm, ctypes.byref(r))
        return r.value

    def Ssend(self, buf, count, t, dest, tag, comm=None):
        self._mode_send("MPI_Ssend", buf, count, t, dest, tag, comm, False)

    def Bsend(self, buf, count, t, dest, tag, comm=None):
        self._mode_send("MPI_Bsend", buf, count, t, dest, tag, comm, False)

    def Rsend(self, buf, count, t, dest, tag, comm=None):
        self._mode_send("MPI_Rsend", buf, count, t, dest, tag, comm, False)

    def Issend(self, buf, count, t, dest, tag, comm=None):
        return self._mode_send("MPI_Issend", buf, count, t, dest, tag, comm, True)

    def Ibsend(self, buf, count, t, dest, tag, comm=None):
        return self._mode_send("MPI_Ibsend", buf, count, t, dest, tag, comm, True)

    def Irsend(self, buf, count, t, dest, tag, comm=None):
        return self._mode_send("MPI_Irsend", buf, count, t, dest, tag, comm, True)

    def Buffer_attach(self, nbytes):
        """attach a host buffer of nbytes for buffered sends (kept alive here)"""
        self._bsend_buf = (ctypes.c_char * nbytes)()
        self._call("MPI_Buffer_attach", self._bsend_buf, nbytes)

    def Buffer_detach(self):
        p, n = ctypes.c_void_p(), ctypes.c_int(0)
        self._call("MPI_Buffer_detach", ctypes.byref(p), ctypes.byref(n))
        self._bsend_buf = None
        return n.value

    # persistent requests
    def _init(self, fn, buf, count, t, peer, tag, comm):
        r = self.Request()
        self._call(fn, ctypes.c_void_p(buf), count, self.h(t), peer, tag,
                   self.h(self.COMM_WORLD if comm is None else comm), ctypes.byref(r))
        return r.value

    def Send_init(self, buf, count, t, dest, tag, comm=None):
        return self._init("MPI_Send_init", buf, count, t, dest, tag, comm)

    def Ssend_init(self, buf, count, t, dest, tag, comm=None):
        return self._init("MPI_Ssend_init", buf, count, t, dest, tag, comm)

    def Bsend_init(self, buf, count, t, dest, tag, comm=None):
        return self._init("MPI_Bsend_init", buf, count, t, dest, tag, comm)

    def Rsend_init(self, buf, count, t, dest, tag, comm=None):
        return self._init("MPI_Rsend_init", buf, count, t, dest, tag, comm)

    def Recv_init(self, buf, count, t, source, tag, comm=None):
        return self._init("MPI_Recv_init", buf, count, t, source, tag, comm)

    def Start(self, req):
        r = self.Request(req)
        self._call("MPI_Start", ctypes.byref(r))
        return r.value

    def Start_rc(self, req):
        """MPI_Start's return code (errors return under MPI_ERRORS_RETURN)"""
        r = self.Request(req)
        return self.L.MPI_Start(ctypes.byref(r))

    def Startall(self, reqs):
        arr = self._reqs(reqs)
        self._call("MPI_Startall", len(reqs), arr)
        return list(arr)[:len(reqs)]

    def Wait(self, req):
        r = self.Request(req)
        self._call("MPI_Wait", ctypes.byref(r), self.STATUS_IGNORE)
        return r.value

    def _decode(self, st, t):
        """(source, tag, count in elements of t) of an MPI_Status buffer"""
        def at(name):
            off = self.const(f"offsetof(MPI_Status,{name})")
            return ctypes.c_int.from_buffer(st, off).value
        n = ctypes.c_int(0)
        self._call("MPI_Get_count", st, self.h(t), ctypes.byref(n))
        return at("MPI_SOURCE"), at("MPI_TAG"), n.value

    def Wait_status(self, req, t):
        """MPI_Wait with a status: returns (request, (source, tag, count of t))"""
        r, st = self.Request(req), self._status()
        self._call("MPI_Wait", ctypes.byref(r), st)
        return r.value, self._decode(st, t)

    def Sendrecv(self, sbuf, scount, st, dest, stag, rbuf, rcount, rt, source, rtag, comm=None):
        """MPI_Sendrecv; returns (source, tag, count of rt) of the receive"""
        status = self._status()
        self._call("MPI_Sendrecv", ctypes.c_void_p(sbuf), scount, self.h(st), dest, stag, ctypes.c_void_p(rbuf),
                   rcount, self.h(rt), source, rtag, self.h(self.COMM_WORLD if comm is None else comm), status)
        return self._decode(status, rt)

    def Sendrecv_replace(self, buf, count, t, dest, stag, source, rtag, comm=None):
        """MPI_Sendrecv_replace; returns (source, tag, count of t) of the receive"""
        status = self._status()
        self._call("MPI_Sendrecv_replace", ctypes.c_void_p(buf), count, self.h(t), dest, stag, source, rtag,
                   self.h(self.COMM_WORLD if comm is None else comm), status)
        return self._decode(status, t)

    def Cancel(self, req):
        r = self.Request(req)
        self._call("MPI_Cancel", ctypes.byref(r))

    def Wait_cancelled(self, req):
        """MPI_Wait, then MPI_Test_cancelled on its status"""
        r, st, c = self.Request(req), self._status(), ctypes.c_int(0)
        self._call("MPI_Wait", ctypes.byref(r), st)
        self._call("MPI_Test_cancelled", st, ctypes.byref(c))
        return r.value, bool(c.value)

    def Request_get_status(self, req, t):
        """(complete?, (source, tag, count of t) when complete); the request stays"""
        st, flag = self._status(), ctypes.c_int(0)
        self._call("MPI_Request_get_status", self.Request(req), ctypes.byref(flag), st)
        return bool(flag.value), (self._decode(st, t) if flag.value else None)

    def Recv_status(self, buf, count, t, source, tag, comm=None):
        """MPI_Recv with a status: (source, tag, count of t)"""
        st = self._status()
        self._call("MPI_Recv", ctypes.c_void_p(buf), count, self.h(t), source, tag,
                   self.h(self.COMM_WORLD if comm is None else comm), st)
        return self._decode(st, t)

    def Waitall(self, reqs):
        n = len(reqs)
        arr = (self.Request * max(n, 1))(*reqs)
        self._call("MPI_Waitall", n, arr, self.STATUSES_IGNORE)
        return list(arr)[:n]

    def Waitall_errors(self, reqs):
        """MPI_Waitall with statuses, not raising: (return code, [MPI_ERROR
        of each status])"""
        n = len(reqs)
        arr = (self.Request * max(n, 1))(*reqs)
        sts = (ctypes.c_char * (self.status_size * max(n, 1)))()
        rc = self.L.MPI_Waitall(n, arr, sts)
        off = self.const("offsetof(MPI_Status,MPI_ERROR)")
        errs = [ctypes.c_int.from_buffer(sts, k * self.status_size + off).value for k in range(n)]
        return rc, errs

    def _reqs(self, reqs):
        return (self.Request * max(len(reqs), 1))(*reqs)

    def Testall(self, reqs):
        arr, flag = self._reqs(reqs), ctypes.c_int(0)
        self._call("MPI_Testall", len(reqs), arr, ctypes.byref(flag), self.STATUSES_IGNORE)
        return bool(flag.value), list(arr)[:len(reqs)]

    def Testany(self, reqs):
        arr, idx, flag = self._reqs(reqs), ctypes.c_int(-1), ctypes.c_int(0)
        self._call("MPI_Testany", len(reqs), arr, ctypes.byref(idx), ctypes.byref(flag), self.STATUS_IGNORE)
        return idx.value, bool(flag.value), list(arr)[:len(reqs)]

    def Waitany(self, reqs):
        arr, idx = self._reqs(reqs), ctypes.c_int(-1)
        self._call("MPI_Waitany", len(reqs), arr, ctypes.byref(idx), self.STATUS_IGNORE)
        return idx.value, list(arr)[:len(reqs)]

    def _some(self, fn, reqs):
        n = len(reqs)
        arr, out = self._reqs(reqs), ctypes.c_int(0)
        idx = (ctypes.c_int * max(n, 1))()
        self._call(fn, n, arr, ctypes.byref(out), idx, self.STATUSES_IGNORE)
        k = out.value
        return (list(idx)[:k] if k >= 0 else None), list(arr)[:n]

    def Testsome(self, reqs):
        return self._some("MPI_Testsome", reqs)

    def Waitsome(self, reqs):
        return self._some("MPI_Waitsome", reqs)

    def Request_free(self, req):
        r = self.Request(req)
        self._call("MPI_Request_free", ctypes.byref(r))
        return r.value

    def Test(self, req):
        r = self.Request(req)
        flag = ctypes.c_int(0)
        self._call("MPI_Test", ctypes.byref(r), ctypes.byref(flag), self.STATUS_IGNORE)
        return bool(flag.value), r.value

    # ------------------------------------------------ probes / matched receives
    def Comm_set_errhandler(self, errhandler, comm=None):
        self._call("MPI_Comm_set_errhandler", self.h(self.COMM_WORLD if comm is None else comm), self.h(errhandler))

    def Probe(self, source, tag, t, comm=None):
        """MPI_Probe: (source, tag, count of t)"""
        st = self._status()
        self._call("MPI_Probe", source, tag, self.h(self.COMM_WORLD if comm is None else comm), st)
        return self._decode(st, t)

    def Iprobe(self, source, tag, t, comm=None):
        """MPI_Iprobe: None, or (source, tag, count of t)"""
        st, flag = self._status(), ctypes.c_int(0)
        self._call("MPI_Iprobe", source, tag, self.h(self.COMM_WORLD if comm is None else comm), ctypes.byref(flag),
                   st)
        return self._decode(st, t) if flag.value else None

    def Mprobe(self, source, tag, t, comm=None):
        """MPI_Mprobe: (message, (source, tag, count of t))"""
        st, m = self._status(), self.Handle()
        self._call("MPI_Mprobe", source, tag, self.h(self.COMM_WORLD if comm is None else comm), ctypes.byref(m), st)
        return m.value, self._decode(st, t)

    def Improbe(self, source, tag, t, comm=None):
        """MPI_Improbe: None, or (message, (source, tag, count of t))"""
        st, m, flag = self._status(), self.Handle(), ctypes.c_int(0)
        self._call("MPI_Improbe", source, tag, self.h(self.COMM_WORLD if comm is None else comm), ctypes.byref(flag),
                   ctypes.byref(m), st)
        return (m.value, self._decode(st, t)) if flag.value else None

    def Mrecv(self, buf, count, t, message):
        """MPI_Mrecv: (source, tag, count of t)"""
        st, m = self._status(), self.Handle(message)
        self._call("MPI_Mrecv", ctypes.c_void_p(buf), count, self.h(t), ctypes.byref(m), st)
        return self._decode(st, t)

    def Imrecv(self, buf, count, t, message):
        r, m = self.Request(), self.Handle(message)
        self._call("MPI_Imrecv", ctypes.c_void_p(buf), count, self.h(t), ctypes.byref(m), ctypes.byref(r))
        return r.value

    def Wait_rc(self, req):
        """MPI_Wait without raising: (rc, MPI_ERROR of the status)"""
        r, st = self.Request(req), self._status()
        rc = self.L.MPI_Wait(ctypes.byref(r), st)
        return rc, ctypes.c_int.from_buffer(st, self.const("offsetof(MPI_Status,MPI_ERROR)")).value

    def Recv_rc(self, buf, count, t, source, tag, comm=None):
        """MPI_Recv without raising: rc"""
        return self.L.MPI_Recv(ctypes.c_void_p(buf), count, self.h(t), source, tag,
                               self.h(self.COMM_WORLD if comm is None else comm), self.STATUS_IGNORE)

    def Alltoallv(self, sbuf, scounts, sdispls, stype, rbuf, rcounts, rdispls, rtype, comm=None):
        n = len(scounts)
        A = ctypes.c_int * n
        self._call("MPI_Alltoallv", ctypes.c_void_p(sbuf), A(*scounts), A(*sdispls), self.h(stype),
                   ctypes.c_void_p(rbuf), A(*rcounts), A(*rdispls), self.h(rtype),
                   self.h(self.COMM_WORLD if comm is None else comm))

    # ------------------------------------------------ topologies / neighbours
    def Dist_graph_create_adjacent(self, sources, destinations, reorder=False, comm=None, sourceweights=None,
                                   destweights=None):
        """weights None: MPI_UNWEIGHTED (both or neither)"""
        A = ctypes.c_int * max(len(sources), 1)
        B = ctypes.c_int * max(len(destinations), 1)
        out = self.Handle()
        unweighted = ctypes.c_void_p(self.const("MPI_UNWEIGHTED"))
        empty = ctypes.c_void_p(self.const("MPI_WEIGHTS_EMPTY"))
        sw = unweighted if sourceweights is None else (A(*sourceweights) if sources else empty)
        dw = unweighted if destweights is None else (B(*destweights) if destinations else empty)
        self._call("MPI_Dist_graph_create_adjacent", self.h(self.COMM_WORLD if comm is None else comm),
                   len(sources), A(*sources), sw, len(destinations), B(*destinations), dw,
                   self.h(self.const("MPI_INFO_NULL")), int(reorder), ctypes.byref(out))
        return out.value

    def Dist_graph_neighbors(self, comm, indeg, outdeg, weights=False):
        """(sources, destinations), plus (sourceweights, destweights) when
        weights is True"""
        A = ctypes.c_int * max(indeg, 1)
        B = ctypes.c_int * max(outdeg, 1)
        s, d = A(), B()
        if weights:
            sw, dw = A(), B()
            self._call("MPI_Dist_graph_neighbors", self.h(comm), indeg, s, sw, outdeg, d, dw)
            return list(s)[:indeg], list(d)[:outdeg], list(sw)[:indeg], list(dw)[:outdeg]
        unweighted = ctypes.c_void_p(self.const("MPI_UNWEIGHTED"))
        self._call("MPI_Dist_graph_neighbors", self.h(comm), indeg, s, unweighted, outdeg, d, unweighted)
        return list(s)[:indeg], list(d)[:outdeg]

    def Allgather_int(self, value, comm=None):
        """every rank's int, in rank order of `comm`"""
        n = self.Comm_size(comm)
        out = (ctypes.c_int * n)()
        mine = ctypes.c_int(value)
        self._call("MPI_Allgather", ctypes.byref(mine), 1, self.h(self.INT), out, 1, self.h(self.INT),
                   self.h(self.COMM_WORLD if comm is None else comm))
        return list(out)

    def Cart_create(self, dims, periods, reorder=False, comm=None):
        n = len(dims)
        out = self.Handle()
        self._call("MPI_Cart_create", self.h(self.COMM_WORLD if comm is None else comm), n,
                   (ctypes.c_int * n)(*dims), (ctypes.c_int * n)(*[int(p) for p in periods]), int(reorder),
                   ctypes.byref(out))
        return out.value

    def Cart_shift(self, comm, direction, disp=1):
        lo, hi = ctypes.c_int(), ctypes.c_int()
        self._call("MPI_Cart_shift", self.h(comm), direction, disp, ctypes.byref(lo), ctypes.byref(hi))
        return lo.value, hi.value

    def Comm_free(self, comm):
        c = self.Handle(comm)
        self._call("MPI_Comm_free", ctypes.byref(c))
        return c.value

    def Comm_dup(self, comm=None):
        out = self.Handle()
        self._call("MPI_Comm_dup", self.h(self.COMM_WORLD if comm is None else comm), ctypes.byref(out))
        return out.value

    def Neighbor_alltoallw(self, sbuf, scounts, sdispls, stypes, rbuf, rcounts, rdispls, rtypes, comm):
        ns, nr = max(len(scounts), 1), max(len(rcounts), 1)
        I, J = ctypes.c_int * ns, ctypes.c_int * nr
        AS, AR = self.Aint * ns, self.Aint * nr
        HS, HR = self.Handle * ns, self.Handle * nr
        self._call("MPI_Neighbor_alltoallw", ctypes.c_void_p(sbuf), I(*scounts), AS(*sdispls), HS(*stypes),
                   ctypes.c_void_p(rbuf), J(*rcounts), AR(*rdispls), HR(*rtypes), self.h(comm))

    def Neighbor_alltoallv(self, sbuf, scounts, sdispls, stype, rbuf, rcounts, rdispls, rtype, comm):
        ns, nr = max(len(scounts), 1), max(len(rcounts), 1)
        I, J = ctypes.c_int * ns, ctypes.c_int * nr
        self._call("MPI_Neighbor_alltoallv", ctypes.c_void_p(sbuf), I(*scounts), I(*sdispls), self.h(stype),
                   ctypes.c_void_p(rbuf), J(*rcounts), J(*rdispls), self.h(rtype), self.h(comm))

    # --------------------------------------------------------------- TEMPI
    def describe(self, t):
        info = TypeInfo()
        self.L.tempi_type_describe(int(t), ctypes.byref(info))
        if not info.known:
            return None
        nd = info.ndims
        return {
            "valid": bool(info.valid),
            "start": info.start,
            "block": info.block,
            "counts": [info.counts[k] for k in range(nd)],
            "strides": [info.strides[k] for k in range(nd)],
            "size": info.size,
            "lb": info.lb,
            "extent": info.extent,
        }

    def counters(self):
        c = Counters()
        self.L.tempi_get_counters(ctypes.byref(c))
        return {n: getattr(c, n) for n in _COUNTER_FIELDS}

    def set_datatype_method(self, m):
        """tempi_set_datatype_method: 0 AUTO, 1 ONESHOT, 2 DEVICE, 3 STAGED, 4 IPC"""
        self.L.tempi_set_datatype_method(int(m))

    def reset_counters(self):
        self.L.tempi_reset_counters()

    def set_kernel_profiling(self, on=True):
        self.L.tempi_set_kernel_profiling(1 if on else 0)

    def kernel_times(self):
        k = KernelTimes()
        self.L.tempi_get_kernel_times(ctypes.byref(k))
        return {"pack_ms": k.pack_ms, "unpack_ms": k.unpack_ms, "packs": k.packs, "unpacks": k.unpacks}

    def partition(self, xadj, adjncy, adjwgt, nparts, sizes=None, method=0):
        """tempi_partition: (part list, edge cut); cut -1 for bad input"""
        n = len(xadj) - 1
        I = ctypes.c_int
        part = (I * max(n, 1))()
        w = (I * max(len(adjwgt), 1))(*adjwgt) if adjwgt is not None else None
        sz = (I * nparts)(*sizes) if sizes is not None else None
        cut = self.L.tempi_partition(n, (I * len(xadj))(*xadj), (I * max(len(adjncy), 1))(*adjncy), w, nparts, sz,
                                     method, part)
        return list(part)[:n], cut

    def placement_info(self):
        """the last rank placement of this process (tempi_placement_info)"""
        out = (ctypes.c_int64 * 6)()
        self.L.tempi_placement_info(out)
        return dict(zip(("placed", "nodes", "method", "app_rank", "cut_identity", "cut_placed"), list(out)))

    def stream(self, device=0):
        return self.L.tempi_get_stream(device)

    def gpu_available(self):
        return bool(self.L.tempi_gpu_available())

    def version(self):
        return self.L.tempi_version().decode()


def get():
    global _singleton
    if _singleton is None:
        _singleton = MPI()
    return _singleton
