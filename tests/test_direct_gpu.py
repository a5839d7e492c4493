"""Sends to the same process (DIRECT): the strided -> strided copy kernel
(tempi_hip_copy_batch, include/tempi_hip.h) and the transport route built on
it (p2p.cpp IsendDirectOp / IrecvOp), on the GPU.

Oracle: oracle/typemap.c through pyoracle -- the destination must equal
unpack(dst type, pack(src type, src)) over an untouched canvas, the MPI
semantics of a message between two type maps of equal size
(/root/reference/test/pack_unpack.cpp:61-97 checks the same identity against
the library). Bit-exact.
"""
import ctypes
import random

import numpy as np
import pytest

from oracle import pyoracle
from tests import typezoo
from tests.test_pack_gpu import HipDesc, _random_recipe, release_l2

pytestmark = pytest.mark.gpu


class CopyItem(ctypes.Structure):
    _fields_ = [("dst_first", ctypes.c_void_p), ("src_first", ctypes.c_void_p), ("dst", HipDesc),
                ("src", HipDesc), ("flags", ctypes.c_uint32), ("reserved_", ctypes.c_uint32)]


ITEM_REMOTE = 1  # TEMPI_HIP_ITEM_REMOTE


def _hip():
    import tempi_amd

    H = ctypes.CDLL(tempi_amd.LIBTEMPI_HIP)
    H.tempi_hip_copy_batch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    H.tempi_hip_copy_supported.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(HipDesc),
                                           ctypes.POINTER(HipDesc)]
    return H


def _flat(mpi, recipe, count):
    t, temps, basic = typezoo.build(mpi, recipe)
    d = mpi.describe(t)
    typezoo.free(mpi, t, temps, basic)
    dims = ([(count, d["extent"])] if count > 1 else []) + list(zip(d["counts"], d["strides"]))
    desc = HipDesc()
    desc.block = d["block"]
    desc.ndims = len(dims)
    for j, (cn, st) in enumerate(dims):
        desc.counts[j] = cn
        desc.strides[j] = st
    return d, desc, len(dims) <= 5


def _reshape(rng, size):
    """a byte layout of exactly `size` bytes with another shape"""
    divs = [b for b in (1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 64, 128, 512, 4096) if size % b == 0 and size // b < 200000]
    bl = rng.choice(divs or [size])
    nb = size // bl
    if rng.random() < 0.5 or nb < 4:
        return f"vector({nb},{bl},{bl + rng.choice([0, 1, 8, 16, bl])},byte)", 1
    for z in (2, 3, 4, 5, 7):
        if nb % z == 0:
            y = nb // z
            return f"subarray(C,[{z + 1},{y + 2},{bl + 24}],[{z},{y},{bl}],[1,{rng.randrange(3)},{rng.choice([0, 3, 8, 24])}],byte)", 1
    return f"vector({nb},{bl},{2 * bl},byte)", 1


@pytest.mark.parametrize("remote", [False, True])
@pytest.mark.parametrize("seed", range(8))
def test_copy_kernel_c_abi(mpi, gpu, seed, remote):
    """tempi_hip_copy_batch: 1-60 (src, dst) pairs of equal size -- same shape
    at other offsets (the halo case), or a different shape entirely -- mixed
    word widths and ranks in one call; the canvas outside each dst type map
    stays untouched. remote: two items in three carry TEMPI_HIP_ITEM_REMOTE
    (source read with system-scope loads, the IPC-copy route)."""
    import torch

    H = _hip()
    rng = random.Random(seed)
    n = rng.choice([1, 5, 24, 60])
    cases = []
    for i in range(n):
        srecipe, scount = _random_recipe(rng), rng.choice([1, 1, 2])
        stm = pyoracle.TypeMap(srecipe)
        size = stm.size * scount
        if size == 0:
            continue
        if rng.random() < 0.4:
            drecipe, dcount = srecipe, scount
        else:
            drecipe, dcount = _reshape(rng, size)
        dtm = pyoracle.TypeMap(drecipe)
        if dtm.size * dcount != size:
            continue
        sd, sdesc, sok = _flat(mpi, srecipe, scount)
        dd, ddesc, dok = _flat(mpi, drecipe, dcount)
        if not (sok and dok):
            continue
        so, slen = stm.geometry(scount)
        do, dlen = dtm.geometry(dcount)
        sshift, dshift = rng.choice([0, 0, 8, 3]), rng.choice([0, 0, 8, 5])
        sh = np.random.default_rng(seed * 977 + i).integers(0, 256, slen + sshift, dtype=np.uint8)
        canvas = np.random.default_rng(seed * 1931 + i).integers(0, 256, dlen + dshift, dtype=np.uint8)
        src = torch.from_numpy(sh).to(gpu)
        dst = torch.from_numpy(canvas).to(gpu)
        it = CopyItem()
        it.src_first = src.data_ptr() + so + sshift + sd["start"]
        it.dst_first = dst.data_ptr() + do + dshift + dd["start"]
        it.src, it.dst = sdesc, ddesc
        it.flags = ITEM_REMOTE if remote and i % 3 != 0 else 0
        ok = H.tempi_hip_copy_supported(it.dst_first, it.src_first, ctypes.byref(it.dst), ctypes.byref(it.src))
        if not ok:
            continue
        exp = canvas.copy()
        dtm.unpack(stm.pack(sh, so + sshift, scount), exp, do + dshift, dcount)
        cases.append((it, src, dst, exp, srecipe, drecipe))
    if not cases:
        pytest.skip("no supported pair drawn")
    items = (CopyItem * len(cases))(*[c[0] for c in cases])
    torch.cuda.synchronize()
    if remote:
        release_l2(H)
    assert H.tempi_hip_copy_batch(items, len(cases), None) == 0
    torch.cuda.synchronize()
    for it, src, dst, exp, sr, dr in cases:
        assert np.array_equal(dst.cpu().numpy(), exp), f"{sr} -> {dr}"


def test_copy_unsupported_and_size_mismatch(mpi, gpu):
    """> 3 dims a side after normalisation, or unequal byte counts: refused
    (the transport then packs + unpacks instead)."""
    import torch

    H = _hip()
    buf = torch.zeros(1 << 16, dtype=torch.uint8, device=gpu)
    deep = HipDesc()
    deep.block, deep.ndims = 1, 4
    for k, (c, s) in enumerate([(2, 4096), (2, 1024), (2, 256), (2, 16)]):
        deep.counts[k], deep.strides[k] = c, s
    flat = HipDesc()
    flat.block, flat.ndims = 16, 0
    p = buf.data_ptr()
    assert H.tempi_hip_copy_supported(p, p + 8192, ctypes.byref(flat), ctypes.byref(deep)) == 0
    three = HipDesc()
    three.block, three.ndims = 2, 3
    for k, (c, s) in enumerate([(2, 1024), (2, 256), (2, 16)]):
        three.counts[k], three.strides[k] = c, s
    assert H.tempi_hip_copy_supported(p, p + 8192, ctypes.byref(flat), ctypes.byref(three)) == 1
    flat.block = 15
    assert H.tempi_hip_copy_supported(p, p + 8192, ctypes.byref(flat), ctypes.byref(three)) == 0
    it = CopyItem(p, p + 8192, flat, three)
    assert H.tempi_hip_copy_batch(ctypes.byref(it), 1, None) != 0


SELF_RECIPES = [
    ("subarray(C,[40,38,512],[30,3,24],[5,3,24],byte)", 2),  # halo x-face shape
    ("subarray(C,[20,30,600],[3,24,512],[2,3,24],byte)", 1),  # y-face, 8-byte aligned rows
    ("vector(1024,512,1024,byte)", 1),
    ("vector(300,3,7,byte)", 2),
    ("hvector(5,1,53,hvector(3,1,16,contig(13,byte)))", 3),
]


def _setup(mpi, gpu, recipe, count, seed):
    import torch

    tm = pyoracle.TypeMap(recipe)
    origin, buflen = tm.geometry(count)
    t, temps, basic = typezoo.build(mpi, recipe)
    sh = np.random.default_rng(seed).integers(0, 256, buflen, dtype=np.uint8)
    canvas = np.random.default_rng(seed + 1).integers(0, 256, buflen, dtype=np.uint8)
    exp = canvas.copy()
    tm.unpack(tm.pack(sh, origin, count), exp, origin, count)
    src = torch.from_numpy(sh).to(gpu)
    dst = torch.from_numpy(canvas).to(gpu)
    torch.cuda.synchronize()
    return tm, origin, (t, temps, basic), src, dst, exp


@pytest.mark.parametrize("recipe,count", SELF_RECIPES)
def test_self_isend_irecv_direct(mpi, gpu, recipe, count):
    """Irecv posted, Isend to self, Waitall: one strided -> strided copy, no
    pack, no fallback."""
    tm, origin, tt, src, dst, exp = _setup(mpi, gpu, recipe, count, 11)
    t = tt[0]
    try:
        before = mpi.counters()
        r = mpi.Irecv(dst.data_ptr() + origin, count, t, 0, 5)
        s = mpi.Isend(src.data_ptr() + origin, count, t, 0, 5)
        assert mpi.Waitall([s, r]) == [mpi.REQUEST_NULL] * 2
        after = mpi.counters()
        assert after["send_direct"] == before["send_direct"] + 1
        assert after["direct_fallbacks"] == before["direct_fallbacks"]
        assert np.array_equal(dst.cpu().numpy(), exp)
    finally:
        typezoo.free(mpi, *tt)


@pytest.mark.parametrize("recipe,count", SELF_RECIPES[:3])
def test_self_send_waited_before_receive(mpi, gpu, recipe, count):
    """Isend to self and Wait on it before the Irecv exists: the send gathers
    into a slab and completes; the later receive unpacks that slab."""
    tm, origin, tt, src, dst, exp = _setup(mpi, gpu, recipe, count, 21)
    t = tt[0]
    try:
        before = mpi.counters()
        s = mpi.Isend(src.data_ptr() + origin, count, t, 0, 6)
        assert mpi.Wait(s) == mpi.REQUEST_NULL
        src.zero_()  # the send is complete: the buffer may be reused
        import torch

        torch.cuda.synchronize()
        r = mpi.Irecv(dst.data_ptr() + origin, count, t, 0, 6)
        assert mpi.Wait(r) == mpi.REQUEST_NULL
        after = mpi.counters()
        assert after["direct_fallbacks"] == before["direct_fallbacks"] + 1
        assert np.array_equal(dst.cpu().numpy(), exp)
    finally:
        typezoo.free(mpi, *tt)


def test_self_direct_other_shape_and_test_loop(mpi, gpu):
    """The receive type differs from the send type (same size): the copy maps
    one shape onto the other; completion is polled with MPI_Test."""
    import torch

    srecipe, drecipe = "subarray(C,[40,38,512],[30,3,24],[5,3,24],byte)", "vector(30,24,100,byte)"
    stm, dtm = pyoracle.TypeMap(srecipe), pyoracle.TypeMap(drecipe)
    dcount = stm.size // dtm.size
    so, slen = stm.geometry(1)
    do, dlen = dtm.geometry(dcount)
    st_ = typezoo.build(mpi, srecipe)
    dt_ = typezoo.build(mpi, drecipe)
    try:
        sh = np.random.default_rng(3).integers(0, 256, slen, dtype=np.uint8)
        canvas = np.random.default_rng(4).integers(0, 256, dlen, dtype=np.uint8)
        assert dcount == 3 and dcount * dtm.size == stm.size
        exp = canvas.copy()
        dtm.unpack(stm.pack(sh, so, 1), exp, do, dcount)
        src, dst = torch.from_numpy(sh).to(gpu), torch.from_numpy(canvas).to(gpu)
        torch.cuda.synchronize()
        r = mpi.Irecv(dst.data_ptr() + do, dcount, dt_[0], 0, 7)
        s = mpi.Isend(src.data_ptr() + so, 1, st_[0], 0, 7)
        for req in (r, s):
            done = False
            while not done:
                done, req = mpi.Test(req)
        assert np.array_equal(dst.cpu().numpy(), exp)
    finally:
        typezoo.free(mpi, *st_)
        typezoo.free(mpi, *dt_)


def test_self_direct_into_library_receives(mpi, gpu):
    """A direct descriptor landing in receives that cannot copy in place: a
    blocking MPI_Recv into host memory, and a device receive of a type TEMPI
    does not pack (library path) -- both fetch the sender's bytes."""
    import torch

    recipe, count = "vector(300,3,7,byte)", 2
    tm, origin, tt, src, dst, exp = _setup(mpi, gpu, recipe, count, 31)
    t = tt[0]
    try:
        host = np.random.default_rng(32).integers(0, 256, exp.size, dtype=np.uint8)
        hexp = host.copy()
        sh = src.cpu().numpy()
        tm.unpack(tm.pack(sh, origin, count), hexp, origin, count)
        s = mpi.Isend(src.data_ptr() + origin, count, t, 0, 8)
        mpi.Recv(host.ctypes.data + origin, count, t, 0, 8)
        assert mpi.Wait(s) == mpi.REQUEST_NULL
        assert np.array_equal(host, hexp)
        # irregular receive type (library-packed) of the same size: 1800 bytes
        irr = "hindexed([700,1100],[0,1000],byte)"
        itm = pyoracle.TypeMap(irr)
        assert itm.size == tm.size * count
        io, ilen = itm.geometry(1)
        it_ = typezoo.build(mpi, irr)
        try:
            canvas = np.random.default_rng(33).integers(0, 256, ilen, dtype=np.uint8)
            iexp = canvas.copy()
            itm.unpack(tm.pack(sh, origin, count), iexp, io, 1)
            idst = torch.from_numpy(canvas).to(gpu)
            torch.cuda.synchronize()
            r = mpi.Irecv(idst.data_ptr() + io, 1, it_[0], 0, 9)
            s = mpi.Isend(src.data_ptr() + origin, count, t, 0, 9)
            mpi.Waitall([r, s])
            assert np.array_equal(idst.cpu().numpy(), iexp)
        finally:
            typezoo.free(mpi, *it_)
    finally:
        typezoo.free(mpi, *tt)


def test_self_any_source_any_tag_and_type_freed_in_flight(mpi, gpu):
    """A direct send matched by an MPI_ANY_SOURCE / MPI_ANY_TAG device receive,
    with both datatypes freed (MPI_Type_free) while the operations are still
    in flight: the transport keeps its own reference to the type record."""
    import torch

    recipe, count = "subarray(C,[40,38,512],[30,3,24],[5,3,24],byte)", 2
    tm, origin, tt, src, dst, exp = _setup(mpi, gpu, recipe, count, 41)
    t = tt[0]
    t2, temps2, basic2 = typezoo.build(mpi, recipe)
    r = mpi.Irecv(dst.data_ptr() + origin, count, t2, mpi.ANY_SOURCE, mpi.ANY_TAG)
    s = mpi.Isend(src.data_ptr() + origin, count, t, 0, 77)
    typezoo.free(mpi, *tt)
    typezoo.free(mpi, t2, temps2, basic2)
    assert mpi.Waitall([r, s]) == [mpi.REQUEST_NULL] * 2
    torch.cuda.synchronize()
    assert np.array_equal(dst.cpu().numpy(), exp)


def _halo_desc(block, counts, strides):
    d = HipDesc()
    d.block = block
    d.ndims = len(counts)
    for j, (cn, st) in enumerate(zip(counts, strides)):
        d.counts[j] = cn
        d.strides[j] = st
    return d


@pytest.mark.parametrize("remote", [False, True])
@pytest.mark.parametrize("l,nq", [(16, 1), (37, 3), (64, 5)])
def test_copy_paired_halo_faces(mpi, gpu, l, nq, remote):
    """The paired copy route (pack_kernels.hip CArgs::s2, pair_jobs): the +-x
    faces of each quantity of a radius-3 periodic halo, where the sector one
    item writes ([0,24) of a row) is the sector its partner reads ([24,48)),
    plus the y faces (16-byte words, another launch) and one extra x face on
    its own buffer that is left unpaired. Bit-exact against numpy's slicing of
    the same halo (the 1-rank case of bench-halo-exchange,
    /root/reference/bin/bench_halo_exchange.cpp:679-704 decomposition)."""
    import torch

    H = _hip()
    r, q = 3, 8
    width = (l + 2 * r) * q
    pitch = (width + 511) // 512 * 512
    ysz = zsz = l + 2 * r
    plane = pitch * ysz
    rng = np.random.default_rng(l * 31 + nq)
    hosts = [rng.integers(0, 256, plane * zsz, dtype=np.uint8) for _ in range(nq + 1)]
    devs = [torch.from_numpy(h).to(gpu) for h in hosts]
    exps = [h.reshape(zsz, ysz, pitch).copy() for h in hosts]
    items = []

    def add(k, s3, d3, e3):
        # s3 / d3: (z, y, x-cell) origins; e3: extents in cells
        src = devs[k].data_ptr() + s3[0] * plane + s3[1] * pitch + s3[2] * q
        dst = devs[k].data_ptr() + d3[0] * plane + d3[1] * pitch + d3[2] * q
        desc = _halo_desc(e3[2] * q, [e3[0], e3[1]], [plane, pitch])
        it = CopyItem()
        it.src_first, it.dst_first, it.src, it.dst = src, dst, desc, desc
        it.flags = ITEM_REMOTE if remote else 0
        items.append(it)
        h = hosts[k].reshape(zsz, ysz, pitch)
        xs, xd, n = s3[2] * q, d3[2] * q, e3[2] * q
        exps[k][d3[0]:d3[0] + e3[0], d3[1]:d3[1] + e3[1], xd:xd + n] = \
            h[s3[0]:s3[0] + e3[0], s3[1]:s3[1] + e3[1], xs:xs + n]

    for k in range(nq):
        add(k, (r, r, r), (r, r, l + r), (l, l, r))  # -x face -> +x halo
        add(k, (r, r, l), (r, r, 0), (l, l, r))      # +x face -> -x halo (its partner)
        add(k, (r, r, r), (r, l + r, r), (l, r, l))  # -y face -> +y halo
        add(k, (r, l, r), (r, 0, r), (l, r, l))      # +y face -> -y halo
    add(nq, (r, r, r), (r, r, l + r), (l, l, r))     # unpaired
    torch.cuda.synchronize()
    if remote:
        release_l2(H)
    arr = (CopyItem * len(items))(*items)
    assert H.tempi_hip_copy_batch(arr, len(items), None) == 0
    torch.cuda.synchronize()
    for k in range(nq + 1):
        got = devs[k].cpu().numpy().reshape(zsz, ysz, pitch)
        assert np.array_equal(got, exps[k]), f"quantity {k}"


def _desc2d(rows, block, stride):
    d = HipDesc()
    d.block, d.ndims = block, 1
    d.counts[0], d.strides[0] = rows, stride
    return d


def test_copy_xcd_mapped_large(gpu):
    """copies whose destination takes the XCD-range tile map (rows sharing
    lines, sectors written in part), two such items of one word width in one
    launch with tile counts that are not multiples of 8, next to an unmapped
    item: every destination byte against torch views, gaps untouched"""
    import torch

    H = _hip()
    g = torch.Generator().manual_seed(7)
    specs = [  # rows, block, src stride, dst stride, dst offset
        (2000003, 8, 24, 40, 8),
        (1000001, 8, 16, 48, 24),
        (3000001, 1, 2, 3, 1),
        (262147, 512, 1024, 1024, 0),
    ]
    cases = []
    for rows, bl, ss, ds, off in specs:
        src = torch.randint(0, 256, (rows * ss,), dtype=torch.uint8, generator=g).to(gpu)
        dst = torch.zeros(rows * ds + off, dtype=torch.uint8, device=gpu)
        it = CopyItem()
        it.src_first, it.dst_first = src.data_ptr(), dst.data_ptr() + off
        it.src, it.dst = _desc2d(rows, bl, ss), _desc2d(rows, bl, ds)
        it.flags = 0
        assert H.tempi_hip_copy_supported(it.dst_first, it.src_first, ctypes.byref(it.dst), ctypes.byref(it.src))
        cases.append((it, src, dst, rows, bl, ss, ds, off))
    items = (CopyItem * len(cases))(*[c[0] for c in cases])
    torch.cuda.synchronize()
    assert H.tempi_hip_copy_batch(items, len(cases), None) == 0
    torch.cuda.synchronize()
    for it, src, dst, rows, bl, ss, ds, off in cases:
        got = dst[off:].view(rows, ds)
        assert torch.equal(got[:, :bl], src.view(rows, ss)[:, :bl]), (rows, bl, ss, ds)
        assert int(got[:, bl:].count_nonzero()) == 0 and int(dst[:off].count_nonzero()) == 0


@pytest.mark.parametrize("remote", [False, True])
def test_copy_peeled_rows(mpi, gpu, remote):
    """The peeled copy (pack_kernels.hip copy_body_peel):
    both sides 8 bytes past a 16-byte boundary, blocks and strides multiples
    of 16, so 16-byte chunks move as one aligned dwordx4 a side except the
    chunks a row seam splits (two 8-byte halves) and the object's first and
    last. Shapes: the halo's y / z faces at a 4608-byte pitch, a single
    16-byte row, rows of 16 / 32 / 48 bytes, and sides of different shapes
    (seams at different chunks on each side), several in one batch with a
    same-shape pair; every destination byte against numpy, gaps untouched,
    and the plan is the peeled one (tempi_hip_copy_word_width == 0)."""
    import torch

    H = _hip()
    H.tempi_hip_copy_word_width.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(HipDesc),
                                            ctypes.POINTER(HipDesc)]

    def desc(block, dims):
        d = HipDesc()
        d.block, d.ndims = block, len(dims)
        for j, (c, st) in enumerate(dims):
            d.counts[j], d.strides[j] = c, st
        return d

    def view(_, off, block, dims):
        """the object's bytes in type-map order, as numpy indices"""
        idx = np.arange(block, dtype=np.int64)
        for c, st in reversed(dims):
            idx = (np.arange(c, dtype=np.int64)[:, None] * st + idx[None, :]).reshape(-1)
        return off + idx

    rng = np.random.default_rng(11)
    plane = 4608 * 70
    specs = [  # (src block, src dims), (dst block, dst dims): equal byte counts
        ((4096, [(9, plane), (3, 4608)]), (4096, [(9, plane), (3, 4608)])),  # y face
        ((4096, [(3, plane), (64, 4608)]), (4096, [(3, plane), (64, 4608)])),  # z face
        ((4096, [(3, plane), (64, 4608)]), (4096, [(3, plane), (64, 4608)])),  # its pair (same shape)
        ((16, []), (16, [])),
        ((16, [(1000, 48)]), (32, [(500, 80)])),
        ((48, [(7, 4096), (11, 64)]), (16, [(231, 32)])),
        ((32, [(3000, 32)]), (96, [(1000, 128), (1, 0)])),
    ]
    cases = []
    for (sb, sdims), (db, ddims) in specs:
        sdims = [d for d in sdims if d[0] != 1]
        ddims = [d for d in ddims if d[0] != 1]
        sd, dd = desc(sb, sdims), desc(db, ddims)
        sidx, didx = view(None, 8, sb, sdims), view(None, 8, db, ddims)
        assert sidx.size == didx.size
        sh = rng.integers(0, 256, int(sidx.max()) + 64, dtype=np.uint8)
        canvas = rng.integers(0, 256, int(didx.max()) + 64, dtype=np.uint8)
        src = torch.from_numpy(sh).to(gpu)
        dst = torch.from_numpy(canvas).to(gpu)
        assert src.data_ptr() % 16 == 0 and dst.data_ptr() % 16 == 0  # (so +8 is the phase)
        it = CopyItem()
        it.src_first, it.dst_first = src.data_ptr() + 8, dst.data_ptr() + 8
        it.src, it.dst = sd, dd
        it.flags = ITEM_REMOTE if remote else 0
        assert H.tempi_hip_copy_word_width(it.dst_first, it.src_first, ctypes.byref(dd), ctypes.byref(sd)) == 0
        exp = canvas.copy()
        exp[didx] = sh[sidx]
        cases.append((it, dst, exp, src))  # (src kept alive: torch's allocator would hand its memory on)
    items = (CopyItem * len(cases))(*[c[0] for c in cases])
    torch.cuda.synchronize()
    if remote:
        release_l2(H)
    assert H.tempi_hip_copy_batch(items, len(cases), None) == 0
    torch.cuda.synchronize()
    for k, (it, dst, exp, _) in enumerate(cases):
        assert np.array_equal(dst.cpu().numpy(), exp), f"case {k}"
    # one phase off on one side, or a 16-byte-misaligned stride: not peeled
    sd = desc(32, [(100, 48)])
    p = cases[0][1].data_ptr()
    assert H.tempi_hip_copy_word_width(p + 8, p + 24 + 4096, ctypes.byref(sd), ctypes.byref(sd)) == 0
    assert H.tempi_hip_copy_word_width(p + 8, p + 4 + 4096, ctypes.byref(sd), ctypes.byref(sd)) == 4
    odd = desc(32, [(100, 40)])
    assert H.tempi_hip_copy_word_width(p + 8, p + 8 + 8192, ctypes.byref(odd), ctypes.byref(odd)) == 8


@pytest.mark.parametrize("seed", range(6))
def test_copy_peeled_random(mpi, gpu, seed):
    """The peeled copy on random shapes: both sides 8 bytes past a 16-byte
    boundary, blocks of 16-byte multiples (16 B - 4 KiB) over 1-3 strided
    dimensions with strides that are multiples of 16 (positive and
    negative), the destination another random shape of the same byte count
    or the same shape; 1-40 items a batch mixed with 8-byte-word items, some
    paired (same shapes), half of them remote. Every destination byte
    against numpy, gaps untouched."""
    import torch

    H = _hip()
    H.tempi_hip_copy_word_width.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(HipDesc),
                                            ctypes.POINTER(HipDesc)]
    rng = random.Random(seed)

    def shape(total=None):
        """(block, [(count, stride) outermost first]) with strides multiples of 16"""
        while True:
            bl = 16 * rng.choice([1, 2, 3, 4, 8, 16, 32, 64, 256])
            nd = rng.choice([0, 1, 1, 2, 2, 3])
            dims, inner = [], bl
            for _ in range(nd):
                c = rng.choice([1, 2, 3, 5, 7, 16, 33])
                st = inner + 16 * rng.choice([0, 1, 2, 5, 32])
                st = -st if rng.random() < 0.15 else st
                dims.insert(0, (c, st))
                inner = c * abs(st)
            size = bl
            for c, _ in dims:
                size *= c
            if total is None or size == total:
                return bl, dims
            if total % bl == 0 and total // bl < 100000:  # the same bytes as one strided dimension
                n = total // bl
                return bl, [(n, bl + 16 * rng.choice([0, 1, 3]))]

    def index(block, dims):
        idx = np.arange(block, dtype=np.int64)
        for c, st in reversed(dims):
            idx = (np.arange(c, dtype=np.int64)[:, None] * st + idx[None, :]).reshape(-1)
        return idx

    def desc(block, dims):
        d = HipDesc()
        d.block, d.ndims = block, len(dims)
        for j, (c, st) in enumerate(dims):
            d.counts[j], d.strides[j] = c, st
        return d

    cases = []
    n = rng.choice([1, 5, 17, 40])
    for i in range(n):
        sb, sdims = shape()
        size = sb
        for c, _ in sdims:
            size *= c
        db, ddims = (sb, sdims) if rng.random() < 0.4 else shape(size)
        sidx, didx = index(sb, sdims), index(db, ddims)
        if sidx.size != didx.size:
            continue
        phase = 8 if rng.random() < 0.8 else 0  # (some ordinary 16-byte-aligned items in the batch)
        sh0, dh0 = int(-sidx.min()) + phase, int(-didx.min()) + phase  # room for negative strides
        host = np.random.default_rng(seed * 1000 + i).integers(0, 256, sh0 + int(sidx.max()) + 64, dtype=np.uint8)
        canvas = np.random.default_rng(seed * 3000 + i).integers(0, 256, dh0 + int(didx.max()) + 64, dtype=np.uint8)
        src, dst = torch.from_numpy(host).to(gpu), torch.from_numpy(canvas).to(gpu)
        it = CopyItem()
        it.src_first, it.dst_first = src.data_ptr() + sh0, dst.data_ptr() + dh0
        it.src, it.dst = desc(sb, sdims), desc(db, ddims)
        it.flags = ITEM_REMOTE if i % 2 else 0
        w = H.tempi_hip_copy_word_width(it.dst_first, it.src_first, ctypes.byref(it.dst), ctypes.byref(it.src))
        if w < 0:
            continue
        assert (w == 0) == (phase == 8), (w, phase, sb, sdims, db, ddims)
        exp = canvas.copy()
        exp[dh0 + didx] = host[sh0 + sidx]
        cases.append((it, src, dst, exp))
    if not cases:
        pytest.skip("no supported item drawn")
    items = (CopyItem * len(cases))(*[c[0] for c in cases])
    torch.cuda.synchronize()
    release_l2(H)
    assert H.tempi_hip_copy_batch(items, len(cases), None) == 0
    torch.cuda.synchronize()
    for k, (it, src, dst, exp) in enumerate(cases):
        assert np.array_equal(dst.cpu().numpy(), exp), f"item {k}"
