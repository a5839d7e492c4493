"""The reference's type-equivalence test
(/root/reference/test/type_equivalence.cpp:13-187), restated through
libtempi.so on the CPU: datatypes built in different ways that describe the
same bytes must agree in size (and extent, where MPI defines them alike),
pack the same bytes through the interposer (host buffers: the library's
MPI_Pack), and -- TEMPI's side -- canonicalise to one and the same strided
descriptor, so that the GPU packs them identically. The factories are those
of /root/reference/support/type.cpp, as tests/typezoo.py recipes. (The
reference's pack comparison packs types[0] every time, :136; here every type
packs itself.)"""
import numpy as np
import pytest

from tests import typezoo

# contiguous bytes four ways (type_equivalence.cpp:20-49)
CONTIG = ["vector({n},1,1,byte)", "vector(1,{n},{n},byte)", "subarray(C,[{n}],[{n}],[0],byte)", "contig({n},byte)"]


def _descr(d):
    return (d["valid"], d["start"], d["block"], tuple(d["counts"]), tuple(d["strides"]), d["size"], d["extent"])


@pytest.mark.parametrize("n", [1, 2, 3, 4])
def test_contiguous_bytes_are_one_type(mpi, n):
    built = [typezoo.build(mpi, r.format(n=n)) for r in CONTIG]
    try:
        views = {(mpi.Type_size(b[0]), mpi.Type_get_extent(b[0])) for b in built}
        assert len(views) == 1, views
        descs = {_descr(mpi.describe(b[0])) for b in built}
        assert len(descs) == 1, descs
        (d,) = descs
        assert d[0] and d[2] == n and d[3] == ()  # one dense block of n bytes
    finally:
        for b in built:
            typezoo.free(mpi, *b)


def _box_recipes(cx, cy, cz, ax, ay, az):
    """the 3-D byte-box factories of support/type.cpp for a cx x cy x cz copy
    out of an ax x ay x az allocation (x fastest)"""
    plane = ax * ay
    return {
        "byte_v_hv": f"hvector({cz},1,{plane},vector({cy},{cx},{ax},byte))",
        "byte_v1_hv_hv": f"hvector({cz},1,{plane},hvector({cy},1,{ax},vector(1,{cx},{ax},byte)))",
        "byte_vn_hv_hv": f"hvector({cz},1,{plane},hvector({cy},1,{ax},vector({cx},1,1,byte)))",
        "subarray": f"subarray(C,[{az},{ay},{ax}],[{cz},{cy},{cx}],[0,0,0],byte)",
    }


def _hi_recipes(cx, cy, cz, ax, ay):
    """make_hi / make_hib: one block per row (not a strided block for TEMPI)"""
    displs = [z * ax * ay + y * ax for z in range(cz) for y in range(cy)]
    d = ",".join(str(v) for v in displs)
    return {"hi": f"hindexed([{','.join([str(cx)] * len(displs))}],[{d}],byte)",
            "hib": f"hindexed_block({cx},[{d}],byte)"}


def test_byte_box_factories_agree(mpi):
    """copy 100 x 13 x 47 out of 256 x 512 x 1024 (type_equivalence.cpp:51-148)"""
    cx, cy, cz, ax, ay, az = 100, 13, 47, 256, 512, 1024
    strided = _box_recipes(cx, cy, cz, ax, ay, az)
    irregular = _hi_recipes(cx, cy, cz, ax, ay)
    built = {k: typezoo.build(mpi, r) for k, r in {**strided, **irregular}.items()}
    try:
        sizes = {k: mpi.Type_size(b[0]) for k, b in built.items()}
        assert set(sizes.values()) == {cx * cy * cz}, sizes
        # the library's extents: every construction but the subarray spans up to
        # the box's last touched byte; a subarray's extent is its whole array
        # (MPI-3.1 4.1.3; the reference's check compares types[0] with itself,
        # :118-119, and so never saw the difference)
        exts = {k: mpi.Type_get_extent(b[0]) for k, b in built.items()}
        last = (cz - 1) * ax * ay + (cy - 1) * ax + cx
        assert exts == {**{k: (0, last) for k in built}, "subarray": (0, ax * ay * az)}, exts
        # TEMPI: one strided descriptor for every strided construction (each
        # keeps its own extent: SURVEY F2), the library for the rest
        descs = {k: _descr(mpi.describe(built[k][0]))[:-1] for k in strided}
        assert len(set(descs.values())) == 1, descs
        assert {k: mpi.describe(built[k][0])["extent"] for k in strided} == {k: exts[k][1] for k in strided}
        d = next(iter(descs.values()))
        assert d[0] and d[2] == cx and d[3] == (cz, cy) and d[4] == (ax * ay, ax)
        for k in irregular:
            assert not mpi.describe(built[k][0])["valid"]
        # every construction packs the same bytes (the interposer hands host
        # buffers to the library)
        src = (np.arange(ax * ay * (cz + 1), dtype=np.int64) % 251).astype(np.uint8)
        packed = {}
        for k, b in built.items():
            out = np.zeros(cx * cy * cz, dtype=np.uint8)
            pos = mpi.Pack(src.ctypes.data, 1, b[0], out.ctypes.data, out.size, 0)
            assert pos == out.size
            packed[k] = out
        ref = src.reshape(cz + 1, ay, ax)[:cz, :cy, :cx].reshape(-1)
        for k, v in packed.items():
            assert np.array_equal(v, ref), k
    finally:
        for b in built.values():
            typezoo.free(mpi, *b)


def test_v1_hv_hv_size(mpi):
    """a 100 x 100 x 1 copy out of 100^3 (type_equivalence.cpp:150-158)"""
    b = typezoo.build(mpi, _box_recipes(100, 100, 1, 100, 100, 100)["byte_v1_hv_hv"])
    try:
        assert mpi.Type_size(b[0]) == 100 * 100
    finally:
        typezoo.free(mpi, *b)


def test_by_rows_by_cols_library_view(mpi):
    """make_2d_hv_by_rows / _by_cols(13, 3, 16, 5, 53): same size and extent
    (type_equivalence.cpp:160-183); their pack orders differ (SURVEY F1,
    tests/test_canonical.py::test_f1_order_preserved)"""
    rows = typezoo.build(mpi, "hvector(5,1,53,vector(3,13,16,byte))")
    cols = typezoo.build(mpi, "hvector(3,1,16,vector(5,13,53,byte))")
    try:
        for b in (rows, cols):
            assert mpi.Type_size(b[0]) == 15 * 13
            assert mpi.Type_get_extent(b[0])[1] == 53 * 4 + 16 * 2 + 13
    finally:
        typezoo.free(mpi, *rows)
        typezoo.free(mpi, *cols)


# /root/reference/test/type_commit.cpp:13-90: the factories committed at the
# reference's sizes (100 x 13 x 47 out of 256 x 512 x 1024; by rows / by
# cols 13, 5, 16, 3, 53); here each must also canonicalise to a valid strided
# descriptor covering exactly the type's bytes
COMMIT_CASES = {
    "hv_by_rows": "hvector(3,1,53,vector(5,13,16,byte))",
    "hv_by_cols": "hvector(5,1,16,vector(3,13,53,byte))",
    "subarray": "subarray(C,[1024,512,256],[47,13,100],[0,0,0],byte)",
    "off_subarray": "subarray(C,[1024,512,256],[47,13,100],[4,4,4],byte)",
    "subarray_v": "vector(47,1,1,subarray(C,[512,256],[13,100],[0,0],byte))",
    "byte_v_hv": _box_recipes(100, 13, 47, 256, 512, 1024)["byte_v_hv"],
    "float_v_hv": "hvector(47,1,131072,vector(13,25,64,float))",
    "byte_v1_hv_hv": _box_recipes(100, 13, 47, 256, 512, 1024)["byte_v1_hv_hv"],
    "byte_vn_hv_hv": _box_recipes(100, 13, 47, 256, 512, 1024)["byte_vn_hv_hv"],
    "v1_hv_hv_plane": _box_recipes(100, 100, 1, 100, 100, 100)["byte_v1_hv_hv"],
}


@pytest.mark.parametrize("name", sorted(COMMIT_CASES))
def test_reference_factories_commit_to_strided_blocks(mpi, name):
    b = typezoo.build(mpi, COMMIT_CASES[name])
    try:
        d = mpi.describe(b[0])
        assert d is not None and d["valid"], d
        n = d["block"]
        for c in d["counts"]:
            n *= c
        assert d["size"] == n == mpi.Type_size(b[0])
    finally:
        typezoo.free(mpi, *b)
