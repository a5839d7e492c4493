"""Run under mpiexec -n 1 with TEMPI_CACHE_DIR set: which perf model TEMPI
loaded at MPI_Init (tempi_perf_source) and what AUTO picks from it
(tempi_choose_method) for blocking strided sends of 2^6 .. 2^22 bytes in
512-byte blocks, to a co-located and to an off-node peer, and the IPC
threshold of non-blocking sends (tempi_ipc_threshold) for 8- and 512-byte
blocks. Prints one JSON line {"source": ..., "loaded": 0|1, "picks":
[[bytes, colocated, method, from_model], ...], "nb_threshold": [[block,
threshold, from_model], ...], "nb_picks": [[bytes, method, from_model],
...]}."""
import ctypes
import json
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)

import tempi_amd  # noqa: E402

mpi = tempi_amd.get_mpi()
mpi.Init()
L = mpi.L
buf = ctypes.create_string_buffer(4096)
loaded = L.tempi_perf_source(buf, 4096)
L.tempi_choose_method.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                  ctypes.POINTER(ctypes.c_int)]
picks = []
for lg in range(6, 23, 2):
    for co in (1, 0):
        fm = ctypes.c_int(-1)
        m = L.tempi_choose_method(1 << lg, 512, co, 1, ctypes.byref(fm))
        picks.append([1 << lg, co, m, fm.value])
L.tempi_ipc_threshold.restype = ctypes.c_int64
L.tempi_ipc_threshold.argtypes = [ctypes.c_int64, ctypes.POINTER(ctypes.c_int)]
nb = []
for bl in (8, 512):
    fm = ctypes.c_int(-1)
    nb.append([bl, L.tempi_ipc_threshold(bl, ctypes.byref(fm)), fm.value])
nb_picks = []
for lg in range(6, 23, 2):
    fm = ctypes.c_int(-1)
    nb_picks.append([1 << lg, L.tempi_choose_method(1 << lg, 512, 1, 0, ctypes.byref(fm)), fm.value])
mpi.Finalize()
print(json.dumps({"source": buf.value.decode(), "loaded": loaded, "picks": picks, "nb_threshold": nb,
                  "nb_picks": nb_picks}), flush=True)
