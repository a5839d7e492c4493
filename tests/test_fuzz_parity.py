"""Parity fuzz over seeded random datatypes (tests/typegen.py): vectors and
hvectors with negative strides, 2-D / 3-D subarrays in C and Fortran order,
regular (h)indexed blocks, resized extents with shifted lower bounds, dups and
nestings of these, one-type structs, over every named element size, at counts 1-4, with the
object's origin misaligned and packing at a non-zero position.

CPU: the oracle (oracle/typemap.c) against the image's MPICH 3.3.2 MPI_Pack /
MPI_Unpack, in process, on every case -- the oracle's pin widened from the
153 golden vectors (tests/test_oracle.py) to these shapes.

GPU: MPI_Pack / MPI_Unpack of device buffers through libtempi.so against the
same MPICH calls on a host copy: bit-exact packed bytes, the same returned
position, and an unpack that leaves every byte outside the type map alone.
This is the reference's pack_unpack test (/root/reference/test/
pack_unpack.cpp:61-118) run over random types instead of its fixed matrix."""
import os

import numpy as np
import pytest

from oracle import pyoracle
from tests import typegen, typezoo

# TEMPI_FUZZ_CHUNKS widens a run (e.g. 1000 chunks = 50 000 types, a
# one-off GPU session); the suite's default is 40
CHUNKS = int(os.environ.get("TEMPI_FUZZ_CHUNKS", "40"))
PER_CHUNK = 50


def _case_buffers(tm, count, shift, seed):
    origin, buflen = tm.geometry(count)
    host = np.random.default_rng(seed).integers(0, 256, buflen + shift, dtype=np.uint8)
    return origin + shift, host


@pytest.mark.parametrize("chunk", range(CHUNKS))
def test_oracle_matches_mpich_random_types(mpi, chunk):
    for k, (recipe, count, shift, position) in enumerate(typegen.cases(0x51F7 + chunk, PER_CHUNK)):
        t, temps, basic = typezoo.build(mpi, recipe)
        try:
            tm = pyoracle.TypeMap(recipe)
            origin, host = _case_buffers(tm, count, shift, 1000 * chunk + k)
            size = mpi.Pack_size(count, t)
            assert size >= tm.size * count, recipe
            lib = np.zeros(position + size + 1, dtype=np.uint8)
            pos = mpi.Pack(host.ctypes.data + origin, count, t, lib.ctypes.data, lib.size, position)
            assert pos == position + tm.size * count, recipe
            assert np.array_equal(lib[position:pos], tm.pack(host, origin, count)), recipe
            # unpack into a canvas: the library and the oracle agree byte for byte
            canvas = np.random.default_rng(7 + k).integers(0, 256, host.size, dtype=np.uint8)
            exp = canvas.copy()
            upos = mpi.Unpack(lib.ctypes.data, lib.size, position, exp.ctypes.data + origin, count, t)
            assert upos == pos, recipe
            tm.unpack(lib[position:pos], canvas, origin, count)
            assert np.array_equal(canvas, exp), recipe
        finally:
            typezoo.free(mpi, t, temps, basic)


@pytest.mark.gpu
@pytest.mark.parametrize("chunk", range(CHUNKS))
def test_tempi_gpu_matches_mpich_random_types(mpi, gpu, chunk):
    import torch

    strided = 0
    for k, (recipe, count, shift, position) in enumerate(typegen.cases(0x51F7 + chunk, PER_CHUNK)):
        t, temps, basic = typezoo.build(mpi, recipe)
        try:
            tm = pyoracle.TypeMap(recipe)
            origin, host = _case_buffers(tm, count, shift, 1000 * chunk + k)
            size = mpi.Pack_size(count, t)
            lib = np.zeros(position + size + 1, dtype=np.uint8)
            lpos = mpi.Pack(host.ctypes.data + origin, count, t, lib.ctypes.data, lib.size, position)
            src = torch.from_numpy(host).to(gpu)
            out = torch.zeros(lib.size, dtype=torch.uint8, device=gpu)
            torch.cuda.synchronize()
            pos = mpi.Pack(src.data_ptr() + origin, count, t, out.data_ptr(), lib.size, position)
            assert pos == lpos, recipe
            got = out.cpu().numpy()
            assert np.array_equal(got[position:pos], lib[position:lpos]), recipe
            assert not got[:position].any() and not got[pos:].any(), f"{recipe}: bytes outside the packed range"
            # device unpack into a canvas == the library's unpack of the same bytes
            canvas = np.random.default_rng(7 + k).integers(0, 256, host.size, dtype=np.uint8)
            dcanvas = torch.from_numpy(canvas).to(gpu)
            torch.cuda.synchronize()
            upos = mpi.Unpack(out.data_ptr(), lib.size, position, dcanvas.data_ptr() + origin, count, t)
            exp = canvas.copy()
            mpi.Unpack(lib.ctypes.data, lib.size, position, exp.ctypes.data + origin, count, t)
            assert upos == lpos, recipe
            assert np.array_equal(dcanvas.cpu().numpy(), exp), recipe
            d = mpi.describe(t)
            strided += bool(d and d["valid"])
        finally:
            typezoo.free(mpi, t, temps, basic)
    # most cases must be ones TEMPI packs on the GPU itself (a strided descriptor)
    assert strided >= PER_CHUNK // 2, strided
