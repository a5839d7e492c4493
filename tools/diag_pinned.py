"""One MPI_Pack / MPI_Unpack per kind of application pinned host memory,
with TEMPI's counters printed around each (diagnosis of which completion a
call took). Run with TEMPI_LOG_LEVEL=DEBUG for the interposer's log."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))
import tempi_amd  # noqa: E402

mpi = tempi_amd.get_mpi()
torch.cuda.set_device(0)
mpi.Init()
hip = ctypes.CDLL("libamdhip64.so")
hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
hip.hipHostFree.argtypes = [ctypes.c_void_p]
H = ctypes.CDLL(tempi_amd.LIBTEMPI_HIP)


class PtrInfo(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int), ("device", ctypes.c_int), ("device_ptr", ctypes.c_void_p)]


H.tempi_hip_pointer_info.argtypes = [ctypes.c_void_p, ctypes.POINTER(PtrInfo)]
rows, block, stride = 4096, 24, 4608
n = rows * block
t = mpi.Type_commit(mpi.Type_vector(rows, block, stride, mpi.BYTE))
src = torch.randint(0, 256, ((rows - 1) * stride + block,), dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
keys = ("packs", "lib_packs", "ticket_waits", "sync_waits", "staged_packs")
for name, flags in (("coherent", 0x40000003), ("noncoherent", 0x80000003), ("default", 0x3), ("plain", 0x0)):
    v = ctypes.c_void_p()
    rc = hip.hipHostMalloc(ctypes.byref(v), n, flags)
    pi = PtrInfo()
    H.tempi_hip_pointer_info(v, ctypes.byref(pi))
    c0 = mpi.counters()
    mpi.Pack(src.data_ptr(), 1, t, v.value, n, 0)
    c1 = mpi.counters()
    print(name, "hipHostMalloc rc", rc, "kind", pi.kind, "device", pi.device, {k: c1[k] - c0[k] for k in keys},
          flush=True)
    hip.hipHostFree(v)
mpi.Type_free(t)
mpi.Finalize()
pinned = torch.zeros(n, dtype=torch.uint8).pin_memory()
pi = PtrInfo()
H.tempi_hip_pointer_info(ctypes.c_void_p(pinned.data_ptr()), ctypes.byref(pi))
print("torch pin_memory kind", pi.kind, "device", pi.device, flush=True)
