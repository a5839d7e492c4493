"""Host-side canonicalisation (no GPU): libtempi's StridedBlock for every
golden datatype, gathered by the oracle's strided restatement, must equal the
library's MPI_Pack bytes. This checks the order-preserving simplifier
(tempi_amd/csrc/core/types.cpp) against SURVEY F1/F2 and the whole zoo.
"""
import numpy as np
import pytest

from oracle import pyoracle
from tests import golden_data as G
from tests import typezoo

CASES = G.cases()

# datatypes that are NOT a single strided block; TEMPI must hand them to the
# library (never a null packer: SURVEY F3)
NOT_STRIDED = {"zoo_hi", "zoo_hib", "hindexed_irregular", "struct_irregular"}


@pytest.mark.parametrize("c", CASES, ids=[c["name"] for c in CASES])
def test_descriptor_packs_like_mpich(mpi, c):
    t, temps, basic = typezoo.build(mpi, c["recipe"])
    try:
        assert mpi.Type_size(t) == c["size"]
        d = mpi.describe(t)
        assert d is not None, "committed type missing from TEMPI's cache"
        if c["name"] in NOT_STRIDED:
            assert not d["valid"]
            return
        assert d["valid"], f"{c['recipe']} not canonicalised: {d}"
        assert d["size"] == c["size"]
        if c["size"]:
            assert d["extent"] == c["extent"] and d["lb"] == c["lb"]
        src = G.source_buffer(c)
        packed = pyoracle.strided_pack(d, c["count"], d["extent"], src, c["origin"])
        G.check_packed(c, packed)
        dst = np.zeros(c["buflen"], dtype=np.uint8)
        pyoracle.strided_unpack(d, c["count"], d["extent"], packed, dst, c["origin"])
        G.check_unpacked(c, dst)
    finally:
        typezoo.free(mpi, t, temps, basic)


def test_f1_order_preserved(mpi):
    """by_rows and by_cols have the same blocks but different pack order."""
    rows = typezoo.build(mpi, G.case("f1_hv_by_rows")["recipe"])
    cols = typezoo.build(mpi, G.case("f1_hv_by_cols")["recipe"])
    try:
        dr, dc = mpi.describe(rows[0]), mpi.describe(cols[0])
        assert dr["counts"] == [5, 3] and dr["strides"] == [53, 16]
        assert dc["counts"] == [3, 5] and dc["strides"] == [16, 53]
    finally:
        typezoo.free(mpi, *rows)
        typezoo.free(mpi, *cols)


def test_f2_extent_kept(mpi):
    t = typezoo.build(mpi, "subarray(C,[100],[10],[5],byte)")
    try:
        d = mpi.describe(t[0])
        assert d["start"] == 5 and d["block"] == 10 and d["counts"] == [] and d["extent"] == 100
    finally:
        typezoo.free(mpi, *t)


def test_cfg1_descriptor(mpi):
    t = typezoo.build(mpi, "vector(1024,512,1024,byte)")
    try:
        d = mpi.describe(t[0])
        assert (d["start"], d["block"], d["counts"], d["strides"]) == (0, 512, [1024], [1024])
    finally:
        typezoo.free(mpi, *t)


def test_type_free_drops_cache(mpi):
    t, temps, basic = typezoo.build(mpi, "vector(3,2,5,byte)")
    assert mpi.describe(t) is not None
    typezoo.free(mpi, t, temps, basic)
    assert mpi.describe(t) is None


@pytest.mark.parametrize("name", ["cfg1_vector_1024_512_1024", "sweep2d_bl3_st19_x3", "f1_hv_by_cols_x2",
                                  "halo32_1_1_1_ext", "zoo_hi"])
def test_library_pack_on_host_buffers(mpi, name):
    """Host buffers take the library path through the interposer unchanged."""
    c = G.case(name)
    t, temps, basic = typezoo.build(mpi, c["recipe"])
    try:
        src = G.source_buffer(c)
        out = np.zeros(max(c["pack_size"], 1), dtype=np.uint8)
        pos = mpi.Pack(src.ctypes.data + c["origin"], c["count"], t, out.ctypes.data, c["pack_size"], 0)
        assert pos == c["position"]
        G.check_packed(c, out[:pos])
    finally:
        typezoo.free(mpi, t, temps, basic)
