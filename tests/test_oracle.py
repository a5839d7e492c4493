"""Pin the CPU oracle (oracle/typemap.c) against the host MPI's own MPI_Pack.

Every golden record in tests/golden/ was produced by MPICH 3.3.2 MPI_Pack /
MPI_Unpack (oracle/gen_golden.c); the oracle must reproduce size, lb, extent,
true extent, packed bytes and unpacked buffers exactly. This is the check that
makes the oracle trustworthy before it judges the GPU path.
"""
import numpy as np
import pytest

from oracle import pyoracle
from tests import golden_data as G

CASES = G.cases()


@pytest.mark.parametrize("c", CASES, ids=[c["name"] for c in CASES])
def test_typemap_matches_mpich(c):
    t = pyoracle.TypeMap(c["recipe"])
    assert t.size == c["size"]
    if c["size"]:
        # lb/extent of an EMPTY type map are implementation-defined (MPICH
        # reports extent 1 for vector(n, 0, s, BYTE)); compare only real ones
        assert t.lb == c["lb"]
        assert t.extent == c["extent"]
        assert t.true_lb == c["true_lb"]
        assert t.true_extent == c["true_extent"]
        assert t.geometry(c["count"]) == (c["origin"], c["buflen"])
    origin, buflen = c["origin"], c["buflen"]
    src = G.source_buffer(c)
    packed = t.pack(src, origin, c["count"])
    G.check_packed(c, packed)
    dst = np.zeros(buflen, dtype=np.uint8)
    n = t.unpack(packed, dst, origin, c["count"])
    assert n == c["unpack_position"]
    G.check_unpacked(c, dst)


def test_strided_restatement_2d():
    # cfg1: vector(1024, 512, 1024, BYTE) == {start 0, block 512, [1024] x [1024]}
    c = G.case("cfg1_vector_1024_512_1024")
    src = G.source_buffer(c)
    desc = {"start": 0, "block": 512, "counts": [1024], "strides": [1024]}
    G.check_packed(c, pyoracle.strided_pack(desc, 1, c["extent"], src, 0))


def test_strided_restatement_f1_cols():
    # make_2d_hv_by_cols(13,3,16,5,53): outer = the 3 columns (stride 16),
    # inner = 5 blocks (stride 53). Order matters.
    c = G.case("f1_hv_by_cols_x2")
    src = G.source_buffer(c)
    desc = {"start": 0, "block": 13, "counts": [3, 5], "strides": [16, 53]}
    G.check_packed(c, pyoracle.strided_pack(desc, 2, c["extent"], src, 0))
    dst = np.zeros(c["buflen"], dtype=np.uint8)
    pyoracle.strided_unpack(desc, 2, c["extent"], pyoracle.strided_pack(desc, 2, c["extent"], src, 0), dst, 0)
    G.check_unpacked(c, dst)


def test_strided_restatement_f2_extent():
    # subarray1d(100,10,5) x3: elements 100 bytes apart
    c = G.case("f2_subarray1d_100_10_5")
    src = G.source_buffer(c)
    desc = {"start": 5, "block": 10, "counts": [], "strides": []}
    G.check_packed(c, pyoracle.strided_pack(desc, 3, 100, src, 0))
