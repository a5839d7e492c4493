"""The C-ABI libraries load without a GPU and export every function the
public headers declare (include/tempi_mpi.h -> libtempi.so, include/
tempi_ext.h -> libtempi.so, include/tempi_hip.h -> libtempi_hip.so)."""
import ctypes
import os
import re
import subprocess

import pytest

import tempi_amd

INC = os.path.join(tempi_amd.ROOT, "include")


def declared(header):
    src = open(os.path.join(INC, header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(\w+)\s*\(", src, flags=re.M)
    return sorted({n for n in names if n.startswith(("MPI_", "tempi_"))})


def exported(lib):
    out = subprocess.check_output(["nm", "-D", "--defined-only", lib], text=True)
    return {l.split()[-1] for l in out.splitlines() if " T " in l}


@pytest.mark.parametrize("header,lib", [("tempi_mpi.h", tempi_amd.LIBTEMPI), ("tempi_ext.h", tempi_amd.LIBTEMPI),
                                        ("tempi_hip.h", tempi_amd.LIBTEMPI_HIP)])
def test_header_symbols_exported(header, lib):
    names = declared(header)
    assert len(names) >= 5, names
    missing = [n for n in names if n not in exported(lib)]
    assert not missing, f"{os.path.basename(lib)} lacks {missing}"


def test_libraries_load_without_gpu():
    ctypes.CDLL(tempi_amd.LIBTEMPI_HIP)
    L = ctypes.CDLL(tempi_amd.LIBTEMPI)
    L.tempi_version.restype = ctypes.c_char_p
    assert b"gfx950" in L.tempi_version()


def test_only_mpi_and_tempi_symbols_exported():
    """No C++ runtime or internal symbols leak from the interposer."""
    bad = [s for s in exported(tempi_amd.LIBTEMPI) if not s.startswith(("MPI_", "tempi_"))]
    assert not bad, bad[:20]


def test_interposer_comes_before_mpi():
    out = subprocess.check_output(["readelf", "-d", tempi_amd.LIBTEMPI], text=True)
    needed = re.findall(r"NEEDED.*\[(.+)\]", out)
    assert needed.index("libtempi_hip.so") < needed.index("libmpi.so.12")


def test_kernels_are_gfx950():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/clang-offload-bundler", "--list", "--type=o",
                          f"--input={tempi_amd.LIBTEMPI_HIP}"], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                         text=True)
    blob = open(tempi_amd.LIBTEMPI_HIP, "rb").read()
    assert b"gfx950" in blob



_RUNTIMES = """
import ctypes, sys
sys.path.insert(0, {root!r})
import tempi_amd
if {order!r} == "torch_first":
    import torch  # noqa: F401  (its wheel bundles a HIP runtime of its own)
L = ctypes.CDLL(tempi_amd.LIBTEMPI)
if {order!r} == "tempi_first":
    import torch  # noqa: F401,F811
buf = ctypes.create_string_buffer(8192)
n = L.tempi_hip_runtimes(buf, 8192)
print(n, buf.value.decode())
"""


@pytest.mark.parametrize("order", ["tempi_only", "torch_first", "tempi_first"])
def test_hip_runtime_detection(order):
    """TEMPI counts the distinct HIP runtimes mapped into
    the process (dl_iterate_phdr over libamdhip64 objects) and reports more
    than one at MPI_Init (core/gpu.cpp). The count depends on load order:
    torch's wheel bundles libamdhip64.so with the SONAME libamdhip64.so.7,
    which is what libtempi_hip.so needs, so torch imported FIRST satisfies it
    (one runtime, torch's); libtempi loaded first maps ROCm's, and torch's
    libraries then load their own (they need the unversioned name): two.
    No GPU is needed to count them."""
    import sys

    code = _RUNTIMES.format(root=tempi_amd.ROOT, order=order)
    r = subprocess.run([sys.executable, "-c", code], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    n, _, paths = r.stdout.strip().partition(" ")
    paths = paths.split(";")
    assert int(n) == len(paths), r.stdout
    assert all("libamdhip64" in p for p in paths), paths
    if order == "tempi_only":
        assert paths == [p for p in paths if "torch" not in p] and int(n) == 1, paths
    elif order == "torch_first":
        assert int(n) == 1 and "torch" in paths[0], paths
    else:
        assert int(n) == 2 and sum("torch" in p for p in paths) == 1, paths
