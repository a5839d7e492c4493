"""oracle/pyoracle.py -- TEST INFRASTRUCTURE ONLY.

ctypes front end for oracle/_build/liboracle.so (typemap.c / recipe.c): the CPU
restatement of MPI_Pack / MPI_Unpack that TEMPI's GPU path is checked against.
Importable only from tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg; the product (libtempi / libtempi_hip) never loads it.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle.so")

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE, "all"])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        i64 = ctypes.c_int64
        P = ctypes.c_void_p
        L.oracle_tm_build.restype = P
        L.oracle_tm_build.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int]
        L.oracle_tm_free.argtypes = [P]
        for f in ("size", "lb", "extent", "true_lb", "true_extent", "nsegs"):
            fn = getattr(L, "oracle_tm_" + f)
            fn.restype = i64
            fn.argtypes = [P]
        L.oracle_tm_seg.argtypes = [P, i64, ctypes.POINTER(i64), ctypes.POINTER(i64)]
        L.oracle_tm_pack.argtypes = [P, i64, P, P, ctypes.POINTER(i64)]
        L.oracle_tm_unpack.argtypes = [P, i64, P, ctypes.POINTER(i64), P]
        sargs = [i64, i64, ctypes.c_int, ctypes.POINTER(i64), ctypes.POINTER(i64), i64, i64, P, P]
        L.oracle_strided_pack.argtypes = sargs
        L.oracle_strided_unpack.argtypes = sargs
        _lib = L
    return _lib


class TypeMap:
    """Type map of a recipe (oracle/recipe.h), MPI-3.1 sec. 4.1 rules."""

    def __init__(self, recipe):
        err = ctypes.create_string_buffer(256)
        self._h = lib().oracle_tm_build(recipe.encode(), err, 256)
        if not self._h:
            raise ValueError(f"bad recipe {recipe!r}: {err.value.decode()}")
        L = lib()
        self.size = L.oracle_tm_size(self._h)
        self.lb = L.oracle_tm_lb(self._h)
        self.extent = L.oracle_tm_extent(self._h)
        self.true_lb = L.oracle_tm_true_lb(self._h)
        self.true_extent = L.oracle_tm_true_extent(self._h)

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.oracle_tm_free(self._h)
            self._h = None

    def segments(self):
        L = lib()
        n = L.oracle_tm_nsegs(self._h)
        d, ln = ctypes.c_int64(), ctypes.c_int64()
        out = []
        for i in range(n):
            L.oracle_tm_seg(self._h, i, ctypes.byref(d), ctypes.byref(ln))
            out.append((d.value, ln.value))
        return out

    def geometry(self, count):
        """(origin, buflen) of a buffer holding `count` elements, as gen_golden.c."""
        lo, hi = self.true_lb, self.true_lb + self.true_extent
        if count > 1:
            d = (count - 1) * self.extent
            if d < 0:
                lo += d
            else:
                hi += d
        origin = -lo if lo < 0 else 0
        buflen = origin + (hi if hi > 0 else 0)
        return origin, max(buflen, 1)

    def pack(self, buf, origin, count):
        """MPI_Pack(buf + origin, count, type) -> bytes (numpy uint8)."""
        assert buf.dtype == np.uint8 and buf.flags.c_contiguous
        out = np.zeros(max(self.size * count, 1), dtype=np.uint8)
        pos = ctypes.c_int64(0)
        lib().oracle_tm_pack(self._h, count, buf.ctypes.data + origin, out.ctypes.data, ctypes.byref(pos))
        return out[: pos.value]

    def unpack(self, packed, buf, origin, count):
        assert buf.dtype == np.uint8 and buf.flags.c_contiguous
        packed = np.ascontiguousarray(packed, dtype=np.uint8)
        pos = ctypes.c_int64(0)
        lib().oracle_tm_unpack(self._h, count, packed.ctypes.data, ctypes.byref(pos), buf.ctypes.data + origin)
        return pos.value


def strided_pack(desc, count, extent, buf, origin):
    """Gather by a canonical descriptor {start, block, counts[], strides[]}
    (outermost first), `count` elements `extent` apart."""
    counts = desc["counts"]
    strides = desc["strides"]
    nd = len(counts)
    C = (ctypes.c_int64 * max(nd, 1))(*counts)
    S = (ctypes.c_int64 * max(nd, 1))(*strides)
    rows = 1
    for c in counts:
        rows *= c
    out = np.zeros(max(rows * desc["block"] * count, 1), dtype=np.uint8)
    lib().oracle_strided_pack(desc["start"], desc["block"], nd, C, S, count, extent,
                              buf.ctypes.data + origin, out.ctypes.data)
    return out[: rows * desc["block"] * count]


def strided_unpack(desc, count, extent, packed, buf, origin):
    counts = desc["counts"]
    strides = desc["strides"]
    nd = len(counts)
    C = (ctypes.c_int64 * max(nd, 1))(*counts)
    S = (ctypes.c_int64 * max(nd, 1))(*strides)
    packed = np.ascontiguousarray(packed, dtype=np.uint8)
    lib().oracle_strided_unpack(desc["start"], desc["block"], nd, C, S, count, extent,
                                packed.ctypes.data, buf.ctypes.data + origin)
