"""tempi_amd -- MI355X-native TEMPI.

The product is native: ``tempi_amd/lib/libtempi.so`` (the C++ MPI interposer,
include/tempi_mpi.h) over ``tempi_amd/lib/libtempi_hip.so`` (gfx950 HIP
kernels behind include/tempi_hip.h). This Python package only locates, builds
and binds them (ctypes) for tests, benchmarks and Python applications; there
is no Python or CPU fallback for any TEMPI operation.
"""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "tempi_amd", "lib")
LIBTEMPI = os.path.join(LIBDIR, "libtempi.so")
LIBTEMPI_HIP = os.path.join(LIBDIR, "libtempi_hip.so")


def build(jobs=8):
    """Compile libtempi_hip.so (hipcc, gfx950), libtempi.so and the oracle."""
    subprocess.check_call(["make", "-C", ROOT, f"-j{jobs}", "all"])


def require_built():
    for p in (LIBTEMPI, LIBTEMPI_HIP):
        if not os.path.exists(p):
            raise RuntimeError(f"{p} is missing: run `make` (or __graft_entry__.build()) first")


def get_mpi():
    """The process-wide ctypes binding of libtempi.so (see tempi_amd.mpi)."""
    import importlib

    return importlib.import_module("tempi_amd.mpi").get()
