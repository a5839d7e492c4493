"""Application pinned host memory under TEMPI, in a process of
its own with ONE HIP runtime: the one libtempi_hip.so links (no torch, whose
wheel bundles a second HIP runtime).

KIND = noncoherent | registered | coherent: the application's host buffers
come from hipHostMalloc(NonCoherent) (coarse-grained), hipHostRegister of a
malloc'ed array, or hipHostMalloc(Coherent). 40 rounds with fresh data:
MPI_Pack of a device object into that packed buffer, MPI_Unpack of device
packed bytes into that strided object; the host reads the bytes right after
each call, so TEMPI must complete both with hipStreamSynchronize (a kernel
wrote host memory), never with its ticket. Then the buffers are unregistered
/ freed as an application would, and fresh pageable arrays -- which may land
on the freed addresses -- go through pageable copies and TEMPI's staged
MPI_Pack once more.

Round 4 and round 5 each saw one illegal address at a later pageable copy
after this sequence ran inside the pytest process, where TEMPI's runtime
and torch's bundled one share the device (profiles/r05/NOTES.md s21).
usage: app_pinned.py KIND   -> prints "RESULT ok" """
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)

import tempi_amd  # noqa: E402

kind = sys.argv[1]
assert kind in ("noncoherent", "registered", "coherent"), kind

ctypes.CDLL(tempi_amd.LIBTEMPI_HIP)
with open("/proc/self/maps") as f:
    libs = sorted({line.split()[-1] for line in f if "libamdhip64" in line})
assert len(libs) == 1, libs  # one HIP runtime in this process
hip = ctypes.CDLL(libs[0])
vp, sz = ctypes.c_void_p, ctypes.c_size_t
hip.hipMalloc.argtypes = [ctypes.POINTER(vp), sz]
hip.hipFree.argtypes = [vp]
hip.hipMemcpy.argtypes = [vp, vp, sz, ctypes.c_int]
hip.hipHostMalloc.argtypes = [ctypes.POINTER(vp), sz, ctypes.c_uint]
hip.hipHostFree.argtypes = [vp]
hip.hipHostRegister.argtypes = [vp, sz, ctypes.c_uint]
hip.hipHostUnregister.argtypes = [vp]
H2D, D2H = 1, 2


def check(rc, what):
    assert rc == 0, f"{what}: hip error {rc}"


def dmalloc(n):
    v = vp()
    check(hip.hipMalloc(ctypes.byref(v), n), "hipMalloc")
    return v.value


mpi = tempi_amd.get_mpi()
mpi.Init()
rows, block, stride = 4096, 24, 4608
n = rows * block
ext = (rows - 1) * stride + block
t = mpi.Type_commit(mpi.Type_vector(rows, block, stride, mpi.BYTE))
ptrs, arrays = [], []


def host_buf(nbytes):
    if kind == "registered":
        a = np.zeros(nbytes + 4096, dtype=np.uint8)
        p = (a.ctypes.data + 4095) & ~4095
        check(hip.hipHostRegister(p, nbytes, 0x2 | 0x1), "hipHostRegister")  # mapped, portable
        arrays.append(a)
        ptrs.append(("unreg", p))
    else:
        v = vp()
        flags = 0x2 | 0x1 | (0x80000000 if kind == "noncoherent" else 0x40000000)
        check(hip.hipHostMalloc(ctypes.byref(v), nbytes, flags), "hipHostMalloc")
        p = v.value
        ptrs.append(("free", p))
    return p, np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p))


src, pk = dmalloc(ext), dmalloc(n)
hp, hview = host_buf(n)
sp, sview = host_buf(ext)
c0 = mpi.counters()
rng = np.random.default_rng(5)
for r in range(40):
    h = rng.integers(0, 256, ext, dtype=np.uint8)
    check(hip.hipMemcpy(src, h.ctypes.data, ext, H2D), "hipMemcpy H2D")
    exp = np.lib.stride_tricks.as_strided(h, (rows, block), (stride, 1)).reshape(-1).copy()
    mpi.Pack(src, 1, t, hp, n, 0)  # device object -> application pinned packed buffer
    assert np.array_equal(hview, exp), f"round {r}: pack into {kind} host memory"
    sview[:] = 0
    check(hip.hipMemcpy(pk, exp.ctypes.data, n, H2D), "hipMemcpy H2D")
    mpi.Unpack(pk, n, 0, sp, 1, t)  # device packed -> application pinned object
    got = np.lib.stride_tricks.as_strided(sview, (rows, block), (stride, 1)).reshape(-1)
    assert np.array_equal(got, exp), f"round {r}: unpack into {kind} host memory"
c1 = mpi.counters()
assert c1["packs"] - c0["packs"] == 40 and c1["unpacks"] - c0["unpacks"] == 40, (c0, c1)  # the GPU path ran
assert c1["sync_waits"] - c0["sync_waits"] == 80 and c1["ticket_waits"] == c0["ticket_waits"], (c0, c1)

del hview, sview
for how, p in ptrs:
    check((hip.hipHostUnregister if how == "unreg" else hip.hipHostFree)(p), how)
arrays.clear()  # (the registered arrays go back to malloc once unregistered)

# fresh pageable arrays after the frees: pageable copies, and TEMPI's MPI_Pack
# of the device object into pageable host memory (staged through its slab)
for r in range(8):
    h = rng.integers(0, 256, ext, dtype=np.uint8)
    check(hip.hipMemcpy(src, h.ctypes.data, ext, H2D), "hipMemcpy H2D after the frees")
    exp = np.lib.stride_tricks.as_strided(h, (rows, block), (stride, 1)).reshape(-1)
    out = np.zeros(n + 4096, dtype=np.uint8)
    mpi.Pack(src, 1, t, out.ctypes.data, n, 0)
    assert np.array_equal(out[:n], exp), f"pageable round {r} after the frees"
    back = np.zeros(ext, dtype=np.uint8)
    check(hip.hipMemcpy(back.ctypes.data, src, ext, D2H), "hipMemcpy D2H after the frees")
    assert np.array_equal(back, h)
mpi.Type_free(t)
check(hip.hipFree(src), "hipFree")
check(hip.hipFree(pk), "hipFree")
mpi.Finalize()
print("RESULT ok", flush=True)
