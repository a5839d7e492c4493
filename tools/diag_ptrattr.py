"""hipPointerGetAttributes of application pinned memory as each HIP runtime in
a PyTorch process sees it: torch's bundled libamdhip64 (which allocates it
here, as an application using torch's runtime would) and ROCm's, which
libtempi_hip.so links. Order as in the test session: MPI_Init (TEMPI's runtime
first), then torch.cuda.init()."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))
import tempi_amd  # noqa: E402

mpi = tempi_amd.get_mpi()
mpi.Init()
import torch  # noqa: E402  (after TEMPI's runtime, as in the test session)

torch.cuda.init()
torch.zeros(1, device="cuda")


class Attr(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("device", ctypes.c_int), ("devicePointer", ctypes.c_void_p),
                ("hostPointer", ctypes.c_void_p), ("isManaged", ctypes.c_int), ("allocationFlags", ctypes.c_uint)]


app = ctypes.CDLL("libamdhip64.so")
H = ctypes.CDLL(tempi_amd.LIBTEMPI_HIP)


class PtrInfo(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int), ("device", ctypes.c_int), ("device_ptr", ctypes.c_void_p)]


H.tempi_hip_pointer_info.argtypes = [ctypes.c_void_p, ctypes.POINTER(PtrInfo)]
with open("/proc/self/maps") as f:
    print("hip runtimes mapped:", sorted({l.split()[-1] for l in f if "amdhip64" in l or "hsa-runtime" in l}),
          flush=True)
with open("/proc/self/maps") as f:
    other = sorted({l.split()[-1] for l in f if "libamdhip64" in l and "torch" not in l})
rocm = ctypes.CDLL(other[0]) if other else None
libs = [("app", app)] + ([("tempi", rocm)] if rocm else [])
for _, lib in libs:
    lib.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    lib.hipPointerGetAttributes.argtypes = [ctypes.POINTER(Attr), ctypes.c_void_p]
    lib.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
for who, alloc in (("app", app),):
    for name, flags in (("noncoherent", 0x80000003), ("coherent", 0x40000003), ("device", None)):
        v = ctypes.c_void_p()
        rc = alloc.hipMalloc(ctypes.byref(v), 1 << 20) if flags is None else alloc.hipHostMalloc(ctypes.byref(v), 1 << 20, flags)
        for seen, lib in libs:
            a = Attr()
            e = lib.hipPointerGetAttributes(ctypes.byref(a), v)
            pi = PtrInfo()
            H.tempi_hip_pointer_info(v, ctypes.byref(pi))
            print(f"alloc by {who} {name} rc={rc} seen by {seen}: err={e} type={a.type} dev={a.device} "
                  f"dptr={a.devicePointer is not None} hptr={a.hostPointer is not None} flags={a.allocationFlags:#x} "
                  f"tempi kind={pi.kind}", flush=True)
pinned = torch.zeros(1 << 20, dtype=torch.uint8).pin_memory()
for seen, lib in (("app", app),):
    a = Attr()
    e = lib.hipPointerGetAttributes(ctypes.byref(a), ctypes.c_void_p(pinned.data_ptr()))
    print(f"torch pin_memory seen by {seen}: err={e} type={a.type} hptr={a.hostPointer is not None}", flush=True)
mpi.Finalize()
