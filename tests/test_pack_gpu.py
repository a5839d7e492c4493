"""GPU parity of MPI_Pack / MPI_Unpack through libtempi.so (MI355X).

The oracle is the host MPI's own MPI_Pack, as in the reference's parity test
(/root/reference/test/pack_unpack.cpp:61-97): (1) the committed MPICH 3.3.2
golden vectors, (2) the in-process library MPI_Pack on host copies of the
same data, (3) oracle/typemap.c. At full sizes the check is exact via strided
torch views and pack -> unpack round trips. Bit-exact everywhere.
"""
import ctypes
import hashlib
import os
import random

import numpy as np
import pytest

from oracle import pyoracle
from tests import golden_data as G
from tests import typezoo

pytestmark = pytest.mark.gpu

CASES = G.cases()
NOT_STRIDED = {"zoo_hi", "zoo_hib", "hindexed_irregular", "struct_irregular"}


def _torch():
    import torch

    return torch


def dev_pattern(n, device):
    torch = _torch()
    return (torch.arange(n, dtype=torch.int64, device=device) & 0xFF).to(torch.uint8)


def to_np(t):
    return t.cpu().numpy()


@pytest.mark.parametrize("c", CASES, ids=[c["name"] for c in CASES])
def test_pack_unpack_golden(mpi, gpu, c):
    torch = _torch()
    t, temps, basic = typezoo.build(mpi, c["recipe"])
    try:
        src = dev_pattern(c["buflen"], gpu)
        out = torch.zeros(max(c["pack_size"], 1), dtype=torch.uint8, device=gpu)
        torch.cuda.synchronize()
        before = mpi.counters()
        pos = mpi.Pack(src.data_ptr() + c["origin"], c["count"], t, out.data_ptr(), c["pack_size"], 0)
        after = mpi.counters()
        assert pos == c["position"]
        G.check_packed(c, to_np(out[:pos]))
        if c["size"] and c["count"]:
            if c["name"] in NOT_STRIDED:
                assert after["lib_packs"] == before["lib_packs"] + 1
            else:  # the GPU path ran, not the library
                assert after["packs"] == before["packs"] + 1
                assert after["lib_packs"] == before["lib_packs"]
        dst = torch.zeros(c["buflen"], dtype=torch.uint8, device=gpu)
        torch.cuda.synchronize()
        upos = mpi.Unpack(out.data_ptr(), c["pack_size"], 0, dst.data_ptr() + c["origin"], c["count"], t)
        assert upos == c["unpack_position"]
        G.check_unpacked(c, to_np(dst))
    finally:
        typezoo.free(mpi, t, temps, basic)


@pytest.mark.parametrize("name", ["cfg1_vector_1024_512_1024", "sweep2d_bl3_st19_x3", "sweep2d_bl24_st40_x2",
                                  "halo32_-1_0_0_int", "sweep3d_bl8_x2", "f1_hv_by_cols_x2",
                                  "double_subarray_F", "vector_neg_stride"])
@pytest.mark.parametrize("prefix,shift", [(1, 0), (3, 5), (8, 0), (13, 7), (16, 3), (0, 9)])
def test_misaligned_position(mpi, gpu, name, prefix, shift):
    """Append at odd positions in odd-aligned buffers: head/tail chunks and
    word-width selection; bytes before the position untouched."""
    torch = _torch()
    c = G.case(name)
    t, temps, basic = typezoo.build(mpi, c["recipe"])
    try:
        src_raw = torch.zeros(c["buflen"] + 64, dtype=torch.uint8, device=gpu)
        src = src_raw[shift:shift + c["buflen"]]  # same content at a `shift`-misaligned address
        src.copy_(dev_pattern(c["buflen"], gpu))
        assert src.data_ptr() == src_raw.data_ptr() + shift
        base = torch.full((c["pack_size"] + prefix + 64,), 0xA5, dtype=torch.uint8, device=gpu)
        torch.cuda.synchronize()
        outp = base.data_ptr() + shift
        pos = mpi.Pack(src.data_ptr() + c["origin"], c["count"], t, outp, prefix + c["pack_size"], prefix)
        assert pos == prefix + c["position"]
        host = to_np(base)
        assert (host[:shift + prefix] == 0xA5).all()
        assert (host[shift + pos:] == 0xA5).all()
        G.check_packed(c, host[shift + prefix:shift + pos])
        # and back
        dst = torch.zeros(c["buflen"] + 16, dtype=torch.uint8, device=gpu)
        torch.cuda.synchronize()
        upos = mpi.Unpack(outp, prefix + c["pack_size"], prefix, dst.data_ptr() + shift + c["origin"], c["count"], t)
        assert upos == prefix + c["position"]
        G.check_unpacked(c, to_np(dst[shift:shift + c["buflen"]]))
    finally:
        typezoo.free(mpi, t, temps, basic)


def _random_recipe(rng):
    k = rng.randrange(6)
    bl = rng.choice([1, 2, 3, 4, 5, 7, 8, 12, 16, 24, 31, 32, 48, 64, 100, 128, 256, 512, 1000, 4096])
    if k == 0:
        nb = rng.randrange(1, 3000)
        st = bl + rng.choice([0, 1, 3, 8, 16, 17, bl, 3 * bl])
        return f"vector({nb},{bl},{st},byte)"
    if k == 1:
        nb = rng.randrange(1, 2000)
        st = bl + rng.choice([0, 5, 16, 64])
        return f"hvector({nb},1,{st},contig({bl},byte))"
    if k == 2:
        rows = rng.randrange(1, 500)
        pitch = bl + rng.choice([0, 1, 13, 16, 256])
        r0 = rng.randrange(0, 8)
        c0 = rng.randrange(0, pitch - bl + 1)
        return f"subarray(C,[{rows + r0 + 3},{pitch}],[{rows},{bl}],[{r0},{c0}],byte)"
    if k == 3:
        z, y = rng.randrange(1, 40), rng.randrange(1, 40)
        x = bl
        Z, Y, X = z + rng.randrange(0, 5), y + rng.randrange(0, 5), x + rng.choice([0, 3, 16, 64])
        return f"subarray(C,[{Z},{Y},{X}],[{z},{y},{x}],[{Z - z},{rng.randrange(0, Y - y + 1)},{X - x}],byte)"
    if k == 4:
        n = rng.randrange(1, 30)
        e = rng.choice(["float", "double", "int", "short"])
        return f"hvector({rng.randrange(1, 40)},1,{rng.choice([4096, 10000, 777 * 8])},vector({n},{rng.randrange(1, 9)},{rng.randrange(9, 20)},{e}))"
    z, y = rng.randrange(1, 12), rng.randrange(1, 12)
    return f"subarray(F,[{y + 2},{z + 3},7],[{y},{z},3],[1,2,4],double)"


@pytest.mark.parametrize("seed", range(40))
def test_random_types_vs_library_and_oracle(mpi, gpu, seed):
    """Random strided types, counts 1-3: TEMPI on the GPU == the library's
    MPI_Pack on a host copy (in-process) == oracle/typemap.c."""
    torch = _torch()
    rng = random.Random(0x7E3D1 + seed)
    recipe = _random_recipe(rng)
    count = rng.choice([1, 1, 2, 3])
    t, temps, basic = typezoo.build(mpi, recipe)
    try:
        tm = pyoracle.TypeMap(recipe)
        origin, buflen = tm.geometry(count)
        size = mpi.Pack_size(count, t)
        host = np.random.default_rng(seed).integers(0, 256, buflen, dtype=np.uint8)
        src = torch.from_numpy(host).to(gpu)
        out = torch.zeros(max(size, 1), dtype=torch.uint8, device=gpu)
        torch.cuda.synchronize()
        pos = mpi.Pack(src.data_ptr() + origin, count, t, out.data_ptr(), size, 0)
        lib_out = np.zeros(max(size, 1), dtype=np.uint8)
        lpos = mpi.Pack(host.ctypes.data + origin, count, t, lib_out.ctypes.data, size, 0)
        assert pos == lpos == tm.size * count
        got = to_np(out[:pos])
        assert np.array_equal(got, lib_out[:lpos]), recipe
        assert np.array_equal(got, tm.pack(host, origin, count)), recipe
        # unpack into a canvas: bytes outside the type map must survive
        canvas = np.random.default_rng(seed + 99).integers(0, 256, buflen, dtype=np.uint8)
        dcanvas = torch.from_numpy(canvas).to(gpu)
        torch.cuda.synchronize()
        mpi.Unpack(out.data_ptr(), size, 0, dcanvas.data_ptr() + origin, count, t)
        exp = canvas.copy()
        mpi.Unpack(lib_out.ctypes.data, size, 0, exp.ctypes.data + origin, count, t)
        assert np.array_equal(to_np(dcanvas), exp), recipe
    finally:
        typezoo.free(mpi, t, temps, basic)


def _subarray2d(mpi, rows, pitch, bl):
    t = mpi.Type_create_subarray([rows, pitch], [rows, bl], [0, 0], mpi.ORDER_C, mpi.BYTE)
    return mpi.Type_commit(t)


@pytest.mark.parametrize("rows,pitch,bl", [(2 * 1024 * 1024, 1024, 512),   # 1 GiB packed, cfg1 shape
                                           (64 * 1024 * 1024, 16, 8),      # 512 MiB, narrow
                                           (256 * 1024, 4096 + 64, 4096),  # 1 GiB, wide rows
                                           (10 * 1024 * 1024, 37, 24)])    # ragged, W=1
def test_full_size_2d_exact(mpi, gpu, rows, pitch, bl):
    """Config-2 sizes: exact comparison against torch strided views, and the
    pack -> unpack round trip restores exactly the type map."""
    torch = _torch()
    t = _subarray2d(mpi, rows, pitch, bl)
    try:
        n = rows * pitch
        src = torch.randint(0, 256, (n,), dtype=torch.uint8, device=gpu)
        out = torch.empty(rows * bl, dtype=torch.uint8, device=gpu)
        torch.cuda.synchronize()
        pos = mpi.Pack(src.data_ptr(), 1, t, out.data_ptr(), rows * bl, 0)
        assert pos == rows * bl
        view = src.view(rows, pitch)[:, :bl]
        assert torch.equal(out.view(rows, bl), view)
        dst = torch.zeros(n, dtype=torch.uint8, device=gpu)
        torch.cuda.synchronize()
        mpi.Unpack(out.data_ptr(), rows * bl, 0, dst.data_ptr(), 1, t)
        torch.cuda.synchronize()
        d2 = dst.view(rows, pitch)
        assert torch.equal(d2[:, :bl], view)
        assert int(d2[:, bl:].count_nonzero()) == 0
    finally:
        mpi.Type_free(t)


@pytest.mark.parametrize("z,y,pitch,bl", [(4000, 4000, 8, 4),       # 3D, planes 24 B off line alignment
                                          (3001, 3000, 18, 2),       # 3D, 2-byte words
                                          (1, 1000003, 144, 128),    # 2D, 16-byte gap
                                          (1, 262147, 4112, 4096)])  # 2D 4 KiB rows, 16-byte gap (round 6)
def test_xcd_mapped_scatter_exact(mpi, gpu, z, y, pitch, bl):
    """Shapes whose unpack takes the XCD-range tile map (partial sectors,
    neighbouring rows sharing lines), with tile counts that are not multiples
    of 8: pack against torch views, then unpack into zeros restores exactly
    the type map and leaves every gap byte untouched."""
    torch = _torch()
    t = mpi.Type_commit(mpi.Type_create_subarray([z, y + 3, pitch], [z, y, bl], [0, 0, 0], mpi.ORDER_C, mpi.BYTE))
    try:
        n = z * (y + 3) * pitch
        size = z * y * bl
        src = torch.randint(0, 256, (n,), dtype=torch.uint8, device=gpu)
        out = torch.empty(size, dtype=torch.uint8, device=gpu)
        torch.cuda.synchronize()
        assert mpi.Pack(src.data_ptr(), 1, t, out.data_ptr(), size, 0) == size
        view = src.view(z, y + 3, pitch)[:, :y, :bl]
        assert torch.equal(out.view(z, y, bl), view)
        dst = torch.zeros(n, dtype=torch.uint8, device=gpu)
        torch.cuda.synchronize()
        mpi.Unpack(out.data_ptr(), size, 0, dst.data_ptr(), 1, t)
        torch.cuda.synchronize()
        d3 = dst.view(z, y + 3, pitch)
        assert torch.equal(d3[:, :y, :bl], view)
        assert int(d3[:, :y, bl:].count_nonzero()) == 0 and int(d3[:, y:, :].count_nonzero()) == 0
    finally:
        mpi.Type_free(t)


def test_halo_faces_512(mpi, gpu):
    """Halo-exchange face/edge/corner types of the 512^3 bench (radius 3,
    8-byte quantities, pitch 4608), against torch 3-D views."""
    torch = _torch()
    r, q, L = 3, 8, 512
    pitch = (L + 2 * r) * q
    pitch = (pitch + 511) // 512 * 512
    ysize = L + 2 * r
    zsize = L + 2 * r
    buf = torch.randint(0, 256, (zsize * ysize * pitch,), dtype=torch.uint8, device=gpu)
    cube = buf.view(zsize, ysize, pitch)
    for d in [(-1, 0, 0), (0, 1, 0), (0, 0, -1), (1, 1, 0), (1, -1, 1)]:
        pos, ext = [], []
        for k in range(3):
            pos.append({-1: r, 1: L, 0: r}[d[k]])
            ext.append(L if d[k] == 0 else r)
        t = mpi.Type_create_subarray([pos[2] + ext[2], ysize, pitch], [ext[2], ext[1], ext[0] * q],
                                     [pos[2], pos[1], pos[0] * q], mpi.ORDER_C, mpi.BYTE)
        t = mpi.Type_commit(t)
        size = mpi.Type_size(t)
        out = torch.empty(size, dtype=torch.uint8, device=gpu)
        torch.cuda.synchronize()
        assert mpi.Pack(buf.data_ptr(), 1, t, out.data_ptr(), size, 0) == size
        exp = cube[pos[2]:pos[2] + ext[2], pos[1]:pos[1] + ext[1], pos[0] * q:(pos[0] + ext[0]) * q]
        assert torch.equal(out, exp.reshape(-1)), d
        mpi.Type_free(t)


def test_truncation_is_an_error(mpi, gpu):
    torch = _torch()
    L = mpi.L
    assert L.MPI_Comm_set_errhandler(mpi.COMM_WORLD, mpi.const("MPI_ERRORS_RETURN")) == 0
    try:
        t = mpi.Type_commit(mpi.Type_vector(64, 8, 16, mpi.BYTE))
        src = torch.zeros(64 * 16, dtype=torch.uint8, device=gpu)
        out = torch.zeros(512, dtype=torch.uint8, device=gpu)
        torch.cuda.synchronize()
        rc, pos = mpi.Pack_rc(src.data_ptr(), 1, t, out.data_ptr(), 511, 0)
        assert rc == mpi.ERR_TRUNCATE and pos == 0
        rc, pos = mpi.Pack_rc(src.data_ptr(), 1, t, out.data_ptr(), 512, 1)
        assert rc == mpi.ERR_TRUNCATE
        mpi.Type_free(t)
    finally:
        L.MPI_Comm_set_errhandler(mpi.COMM_WORLD, mpi.const("MPI_ERRORS_ARE_FATAL"))


def test_pinned_host_output(mpi, gpu):
    """Mapped pinned host memory is device-accessible: the GPU kernel writes
    straight into it (the ONE_SHOT idea)."""
    torch = _torch()
    t = mpi.Type_commit(mpi.Type_vector(4096, 24, 4608, mpi.BYTE))
    try:
        src = torch.randint(0, 256, (4096 * 4608,), dtype=torch.uint8, device=gpu)
        out = torch.zeros(4096 * 24, dtype=torch.uint8).pin_memory()
        torch.cuda.synchronize()
        before = mpi.counters()["packs"]
        mpi.Pack(src.data_ptr(), 1, t, out.data_ptr(), out.numel(), 0)
        assert mpi.counters()["packs"] == before + 1
        assert torch.equal(out, src.view(4096, 4608)[:, :24].reshape(-1).cpu())
    finally:
        mpi.Type_free(t)


@pytest.mark.parametrize("count,prefix", [(1, 0), (2, 5), (3, 13)])
def test_device_to_pageable_host(mpi, gpu, count, prefix):
    """Device object, pageable host packed buffer (both directions): the GPU
    kernel gathers into / scatters from a pinned slab (no library pack, no
    copy of the object's span), bit-exact, at odd positions; bytes before the
    position and gap bytes untouched"""
    torch = _torch()
    t = mpi.Type_commit(mpi.Type_vector(1000, 12, 40, mpi.BYTE))
    try:
        ext = 999 * 40 + 12
        src = torch.randint(0, 256, (ext * count,), dtype=torch.uint8, device=gpu)
        n = 12000 * count
        out = np.full(prefix + n + 7, 0xA5, dtype=np.uint8)
        torch.cuda.synchronize()
        before = mpi.counters()
        pos = mpi.Pack(src.data_ptr(), count, t, out.ctypes.data, prefix + n, prefix)
        after = mpi.counters()
        assert pos == prefix + n
        assert after["staged_packs"] == before["staged_packs"] + 1 and after["lib_packs"] == before["lib_packs"]
        hs = to_np(src)
        exp = np.concatenate([hs[e * ext + r * 40:e * ext + r * 40 + 12] for e in range(count) for r in range(1000)])
        assert np.array_equal(out[prefix:prefix + n], exp)
        assert (out[:prefix] == 0xA5).all() and (out[prefix + n:] == 0xA5).all()
        # and back into a device object whose gaps must keep their bytes
        dst = torch.full((ext * count,), 0x3C, dtype=torch.uint8, device=gpu)
        torch.cuda.synchronize()
        upos = mpi.Unpack(out.ctypes.data, prefix + n, prefix, dst.data_ptr(), count, t)
        assert upos == prefix + n and mpi.counters()["staged_unpacks"] == after["staged_unpacks"] + 1
        hd = to_np(dst)
        ref = np.full(ext * count, 0x3C, dtype=np.uint8)
        for e in range(count):
            for r in range(1000):
                ref[e * ext + r * 40:e * ext + r * 40 + 12] = hs[e * ext + r * 40:e * ext + r * 40 + 12]
        assert np.array_equal(hd, ref)
        # a packed buffer too small: MPI_ERR_TRUNCATE, nothing written
        assert mpi.L.MPI_Comm_set_errhandler(mpi.COMM_WORLD, mpi.const("MPI_ERRORS_RETURN")) == 0
        try:
            out[:] = 0xA5
            rc, p2 = mpi.Pack_rc(src.data_ptr(), count, t, out.ctypes.data, prefix + n - 1, prefix)
            assert rc == mpi.ERR_TRUNCATE and p2 == prefix and (out == 0xA5).all()
        finally:
            mpi.L.MPI_Comm_set_errhandler(mpi.COMM_WORLD, mpi.const("MPI_ERRORS_ARE_FATAL"))
    finally:
        mpi.Type_free(t)


class HipDesc(ctypes.Structure):
    _fields_ = [("block", ctypes.c_int64), ("ndims", ctypes.c_int32), ("pad_", ctypes.c_int32),
                ("counts", ctypes.c_int64 * 5), ("strides", ctypes.c_int64 * 5)]


class HipItem(ctypes.Structure):
    _fields_ = [("packed", ctypes.c_void_p), ("first", ctypes.c_void_p), ("desc", HipDesc),
                ("flags", ctypes.c_uint32), ("reserved_", ctypes.c_uint32)]


ITEM_REMOTE = 1  # TEMPI_HIP_ITEM_REMOTE


def release_l2(H):
    """a HIP event recorded and waited for: its system-scope release writes
    the L2 back, as the transport's batch event does before an IPC reader on
    another GPU is told (TEMPI_HIP_ITEM_REMOTE loads bypass this GPU's L2)"""
    H.tempi_hip_event_create.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int]
    H.tempi_hip_event_record.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    H.tempi_hip_event_synchronize.argtypes = [ctypes.c_void_p]
    H.tempi_hip_event_destroy.argtypes = [ctypes.c_void_p]
    ev = ctypes.c_void_p()
    assert H.tempi_hip_event_create(ctypes.byref(ev), 0) == 0
    assert H.tempi_hip_event_record(ev, None) == 0
    assert H.tempi_hip_event_synchronize(ev) == 0
    H.tempi_hip_event_destroy(ev)


@pytest.mark.parametrize("remote", [False, True])
@pytest.mark.parametrize("seed", range(6))
def test_batched_kernel_c_abi(mpi, gpu, seed, remote):
    """tempi_hip_pack_batch / tempi_hip_unpack_batch (include/tempi_hip.h):
    up to 100 objects of mixed word width / rank / alignment in one call,
    against oracle/typemap.c, and the scatter back restores every type map.
    remote: every other item carries TEMPI_HIP_ITEM_REMOTE, so its scatter
    reads the packed bytes with system-scope buffer loads (the IPC path)."""
    torch = _torch()
    import tempi_amd

    H = ctypes.CDLL(tempi_amd.LIBTEMPI_HIP)
    H.tempi_hip_pack_batch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    H.tempi_hip_unpack_batch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    rng = random.Random(seed)
    n = rng.choice([1, 7, 40, 100])
    cases = []
    off = 0
    for i in range(n):
        recipe = _random_recipe(rng)
        count = rng.choice([1, 2])
        t, temps, basic = typezoo.build(mpi, recipe)
        d = mpi.describe(t)
        typezoo.free(mpi, t, temps, basic)
        dims = ([(count, d["extent"])] if count > 1 else []) + list(zip(d["counts"], d["strides"]))
        if len(dims) > 5:
            continue
        tm = pyoracle.TypeMap(recipe)
        origin, buflen = tm.geometry(count)
        shift = rng.choice([0, 0, 1, 4, 8])
        host = np.random.default_rng(seed * 1000 + i).integers(0, 256, buflen + shift, dtype=np.uint8)
        off += rng.choice([0, 3])
        size = tm.size * count
        cases.append(dict(tm=tm, origin=origin + shift, count=count, host=host, off=off, size=size, d=d,
                          dims=dims, src=torch.from_numpy(host).to(gpu)))
        off += size
    packed = torch.zeros(off + 64, dtype=torch.uint8, device=gpu)
    items = (HipItem * len(cases))()
    for k, c in enumerate(cases):
        it = items[k]
        it.packed = packed.data_ptr() + c["off"]
        it.first = c["src"].data_ptr() + c["origin"] + c["d"]["start"]
        it.desc.block = c["d"]["block"]
        it.desc.ndims = len(c["dims"])
        for j, (cn, st) in enumerate(c["dims"]):
            it.desc.counts[j] = cn
            it.desc.strides[j] = st
        it.flags = ITEM_REMOTE if remote and k % 2 == 0 else 0
    torch.cuda.synchronize()
    assert H.tempi_hip_pack_batch(items, len(cases), None) == 0
    torch.cuda.synchronize()
    got = packed.cpu().numpy()
    for c in cases:
        assert np.array_equal(got[c["off"]:c["off"] + c["size"]], c["tm"].pack(c["host"], c["origin"], c["count"]))
    for c in cases:
        c["src"].zero_()
    torch.cuda.synchronize()
    if remote:
        release_l2(H)
    assert H.tempi_hip_unpack_batch(items, len(cases), None) == 0
    torch.cuda.synchronize()
    for c in cases:
        exp = np.zeros_like(c["host"])
        c["tm"].unpack(c["tm"].pack(c["host"], c["origin"], c["count"]), exp, c["origin"], c["count"])
        assert np.array_equal(c["src"].cpu().numpy(), exp)


def _slab_rounds(H, host_ptr, dev_ptr, obj, n_rows, rounds, seed):
    """kernel writes the slab -> host reads it; host writes the reused slab ->
    kernel reads it; `rounds` times, as the transport does it: kernels on a
    non-blocking stream of TEMPI's kind, completion seen by polling an event
    (no device-wide synchronisation between the host's write and the kernel
    that reads). Returns (host-read mismatches, kernel-read mismatches) in
    bytes."""
    torch = _torch()
    d = HipDesc()
    d.block, d.ndims = 64, 1
    d.counts[0], d.strides[0] = n_rows, 128
    vp = ctypes.c_void_p
    H.tempi_hip_pack.argtypes = [vp, vp, ctypes.POINTER(HipDesc), vp]
    H.tempi_hip_unpack.argtypes = [vp, vp, ctypes.POINTER(HipDesc), vp]
    H.tempi_hip_stream_create.argtypes = [ctypes.POINTER(vp)]
    H.tempi_hip_stream_destroy.argtypes = [vp]
    H.tempi_hip_stream_synchronize.argtypes = [vp]
    H.tempi_hip_event_create.argtypes = [ctypes.POINTER(vp), ctypes.c_int]
    H.tempi_hip_event_record.argtypes = [vp, vp]
    H.tempi_hip_event_query.argtypes = [vp]
    H.tempi_hip_event_destroy.argtypes = [vp]
    s, ev = vp(), vp()
    assert H.tempi_hip_stream_create(ctypes.byref(s)) == 0
    assert H.tempi_hip_event_create(ctypes.byref(ev), 0) == 0

    def run_and_poll():
        assert H.tempi_hip_event_record(ev, s) == 0
        while True:
            q = H.tempi_hip_event_query(ev)
            if q == 0:
                return
            assert q == 1, q

    nbytes = n_rows * 64
    slab = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(host_ptr))
    view = obj.view(n_rows, 128)[:, :64]
    rng = np.random.default_rng(seed)
    bad_host = bad_kernel = 0
    try:
        for _ in range(rounds):
            obj.copy_(torch.from_numpy(rng.integers(0, 256, obj.numel(), dtype=np.uint8)).to(obj.device))
            torch.cuda.synchronize()
            # a kernel writes the slab (the sender's gather), the host reads it (the library sends it)
            assert H.tempi_hip_pack(dev_ptr, obj.data_ptr(), ctypes.byref(d), s) == 0
            run_and_poll()
            bad_host += int((slab != view.reshape(-1).cpu().numpy()).sum())
            # the host writes the reused slab (the library receives into it), a kernel reads it (the scatter)
            new = rng.integers(0, 256, nbytes, dtype=np.uint8)
            slab[:] = new
            assert H.tempi_hip_unpack(obj.data_ptr(), dev_ptr, ctypes.byref(d), s) == 0
            run_and_poll()
            bad_kernel += int((view.reshape(-1).cpu().numpy() != new).sum())
    finally:
        H.tempi_hip_stream_synchronize(s)
        H.tempi_hip_event_destroy(ev)
        H.tempi_hip_stream_destroy(s)
    return bad_host, bad_kernel


def test_pinned_slab_reuse_ordering(gpu):
    """The ordering behind round 1's host-route mismatch (commit d840279), run
    deterministically: a pinned slab that a kernel wrote and the host read is
    rewritten by the host -- not a HIP operation, so no HIP fence orders it
    against lines the GPU kept from the slab's earlier use -- and then read by
    a kernel, and reused, 64 times in one process. TEMPI's pinned slabs
    (tempi_hip_host_alloc) are fine-grained, so the GPU keeps none of their
    lines: every byte must arrive both ways."""
    torch = _torch()
    import tempi_amd

    H = ctypes.CDLL(tempi_amd.LIBTEMPI_HIP)
    H.tempi_hip_host_alloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p),
                                       ctypes.c_size_t]
    H.tempi_hip_host_free.argtypes = [ctypes.c_void_p]
    rows = 4096
    host, dev = ctypes.c_void_p(), ctypes.c_void_p()
    assert H.tempi_hip_host_alloc(ctypes.byref(host), ctypes.byref(dev), rows * 64) == 0
    try:
        obj = torch.zeros(rows * 128, dtype=torch.uint8, device=gpu)
        assert _slab_rounds(H, host.value, dev.value, obj, rows, 64, 11) == (0, 0)
    finally:
        H.tempi_hip_host_free(host)


def test_pinned_slab_reuse_coarse_grained_contrast(gpu, capsys):
    """The same rounds on a coarse-grained slab (hipHostMalloc without
    hipHostMallocCoherent, HIP's default before d840279). Reported, not
    asserted: whether this box's L2 returns a stale line here is the
    hazard the fine-grained allocation rules out."""
    torch = _torch()
    import tempi_amd

    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostGetDevicePointer.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p, ctypes.c_uint]
    hip.hipHostFree.argtypes = [ctypes.c_void_p]
    H = ctypes.CDLL(tempi_amd.LIBTEMPI_HIP)
    rows = 4096
    host, dev = ctypes.c_void_p(), ctypes.c_void_p()
    assert hip.hipHostMalloc(ctypes.byref(host), rows * 64, 0x2 | 0x1 | 0x80000000) == 0  # mapped, portable, non-coherent
    assert hip.hipHostGetDevicePointer(ctypes.byref(dev), host, 0) == 0
    try:
        obj = torch.zeros(rows * 128, dtype=torch.uint8, device=gpu)
        bad = _slab_rounds(H, host.value, dev.value, obj, rows, 64, 12)
        with capsys.disabled():
            print(f"\n[coarse-grained slab] stale bytes over 64 rounds: host read {bad[0]}, kernel read {bad[1]}")
    finally:
        hip.hipHostFree(host)


def test_gpu_failure_falls_back_to_the_library(gpu):
    """a failed GPU pack / unpack (TEMPI_FAULT_PACK makes every launch fail)
    is redone by the library through host staging, bit-exact, instead of
    exiting"""
    import subprocess
    import sys

    code = (
        "import numpy as np, torch, tempi_amd\n"
        "mpi = tempi_amd.get_mpi(); mpi.Init()\n"
        "t = mpi.Type_commit(mpi.Type_vector(1000, 12, 40, mpi.BYTE))\n"
        "src = torch.randint(0, 256, (40000,), dtype=torch.uint8, device='cuda')\n"
        "out = torch.zeros(12000, dtype=torch.uint8, device='cuda')\n"
        "torch.cuda.synchronize()\n"
        "assert mpi.Pack(src.data_ptr(), 1, t, out.data_ptr(), 12000, 0) == 12000\n"
        "assert torch.equal(out.cpu(), src.view(1000, 40)[:, :12].reshape(-1).cpu())\n"
        "dst = torch.full((40000,), 7, dtype=torch.uint8, device='cuda'); torch.cuda.synchronize()\n"
        "assert mpi.Unpack(out.data_ptr(), 12000, 0, dst.data_ptr(), 1, t) == 12000\n"
        "ref = torch.full((40000,), 7, dtype=torch.uint8); ref.view(1000, 40)[:, :12] = src.view(1000, 40)[:, :12].cpu()\n"
        "assert torch.equal(dst.cpu(), ref)\n"
        "c = mpi.counters(); assert c['lib_packs'] == 1 and c['lib_unpacks'] == 1 and c['packs'] == 0, c\n"
        "mpi.Finalize(); print('RESULT ok')\n")
    env = dict(os.environ, TEMPI_FAULT_PACK="1")
    root = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, text=True, timeout=200)
    assert r.returncode == 0 and "RESULT ok" in r.stdout, r.stdout[-3000:]


def test_pack_bench_app(gpu):
    """the reference's bench_pack and bench_pack_kernels at the C-ABI (apps/
    pack_bench.cpp): every point's first pack and unpack checked byte for
    byte, packed side in pinned host memory (oneshot) and in device memory"""
    import json
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([os.path.join(root, "tempi_amd", "lib", "pack_bench"), "3", "--max-target", str(1 << 20)],
                       capture_output=True, text=True, timeout=200)
    recs = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    assert p.returncode == 0, p.stderr[-2000:]
    # bench_pack: 2 destinations x 8 targets <= 1 MiB x 12 rows x {pack, unpack};
    # bench_pack_kernels: 2 destinations x 2 targets x 2 counts x (7 + 15) rows
    assert sum(r["bench"] == "bench_pack" for r in recs) == 2 * 8 * 12 * 2
    assert sum(r["bench"] == "bench_pack_kernels" for r in recs) == 2 * 2 * 2 * 22
    assert all(r["errors"] == 0 and r["us"] > 0 for r in recs)


def test_unpack_batch_xcd_mapped_large(gpu):
    """tempi_hip_unpack_batch with large items whose scatter takes the
    XCD-range tile map (per item within one launch: 4-byte rows at strides 8
    and 12, 2-byte rows at 18) beside an unmapped one (512-byte rows): every
    row against torch views, the gaps untouched"""
    import tempi_amd
    import torch

    H = ctypes.CDLL(tempi_amd.LIBTEMPI_HIP)
    H.tempi_hip_unpack_batch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    g = torch.Generator().manual_seed(11)
    specs = [(4000003, 4, 8), (2500001, 4, 12), (3000017, 2, 18), (131075, 512, 1024)]  # rows, block, stride
    items = (HipItem * len(specs))()
    bufs = []
    for k, (rows, bl, st) in enumerate(specs):
        packed = torch.randint(0, 256, (rows * bl,), dtype=torch.uint8, generator=g).to(gpu)
        dst = torch.zeros(rows * st, dtype=torch.uint8, device=gpu)
        it = items[k]
        it.packed, it.first, it.flags = packed.data_ptr(), dst.data_ptr(), 0
        it.desc.block, it.desc.ndims = bl, 1
        it.desc.counts[0], it.desc.strides[0] = rows, st
        bufs.append((packed, dst, rows, bl, st))
    torch.cuda.synchronize()
    assert H.tempi_hip_unpack_batch(items, len(specs), None) == 0
    torch.cuda.synchronize()
    for packed, dst, rows, bl, st in bufs:
        got = dst.view(rows, st)
        assert torch.equal(got[:, :bl], packed.view(rows, bl)), (rows, bl, st)
        assert int(got[:, bl:].count_nonzero()) == 0


def _ticket_stats():
    import tempi_amd

    H = ctypes.CDLL(tempi_amd.LIBTEMPI_HIP)
    f, q = ctypes.c_uint64(), ctypes.c_uint64()
    H.tempi_hip_ticket_stats(ctypes.byref(f), ctypes.byref(q))
    return f.value, q.value


# (pack, unpack) calls whose ticket the work kernel stores itself: gathers
# and 16-byte-word scatters (write-through) fold up to
# TEMPI_FOLD_MAX_BLOCKS_WT = 2048 workgroups, other scatters up to
# TEMPI_FOLD_MAX_BLOCKS = 128 (hip/ticket.hpp)
@pytest.mark.parametrize("rows,block,stride,folds", [
    (1024, 512, 1024, (60, 60)),  # config 1: 256 workgroups, both folded (16-byte words)
    (300, 512, 1024, (60, 60)),   # 75 workgroups, 16-byte words, not a multiple of the 8 shards
    (4096, 24, 4608, (60, 60)),   # halo x-face rows (interleaved unpack), 24 / 48 workgroups
    (20000, 3, 7, (60, 60)),      # dense-window gather (1-byte words), 30 workgroups
    (64, 512, 1024, (60, 60)),    # 32 KiB: 16 workgroups
    (2, 512, 1024, (60, 60)),     # one workgroup: one shard, the top counted once
    (100, 500, 1000, (60, 60)),   # 4-byte words, 13 / 25 workgroups: shards of unequal counts
    (16384, 512, 1024, (0, 0))])  # 8 MiB: 4096 workgroups, ticket kernel both ways
def test_synchronous_ticket_visible_device_wide(mpi, gpu, rows, block, stride, folds):
    """Synchronous MPI_Pack / MPI_Unpack between device buffers complete by a
    ticket -- stored by the work kernel's last workgroup for small grids
    (VERDICT r02 next 5), by the ticket kernel behind larger ones. Right
    after each call returns, a kernel on ANOTHER stream (torch's) compares
    the result: the bytes must already be visible device-wide. 60 rounds
    with fresh contents each, so a stale line would show."""
    torch = _torch()
    import tempi_amd

    H = ctypes.CDLL(tempi_amd.LIBTEMPI_HIP)
    prev = H.tempi_hip_resident_enable(0)  # (launched calls only: the resident packer has its own test file)
    t = mpi.Type_commit(mpi.Type_vector(rows, block, stride, mpi.BYTE))
    ext = (rows - 1) * stride + block
    try:
        src = torch.empty(ext, dtype=torch.uint8, device=gpu)
        packed = torch.empty(rows * block, dtype=torch.uint8, device=gpu)
        back = torch.zeros(ext, dtype=torch.uint8, device=gpu)
        c0, f0 = mpi.counters(), _ticket_stats()
        g = torch.Generator(device=gpu).manual_seed(rows)
        for r in range(60):
            src.random_(0, 256, generator=g)
            idx = torch.arange(rows, device=gpu).unsqueeze(1) * stride + torch.arange(block, device=gpu)
            exp = src[idx.reshape(-1)]
            torch.cuda.synchronize()
            mpi.Pack(src.data_ptr(), 1, t, packed.data_ptr(), packed.numel(), 0)
            assert torch.equal(packed, exp), f"round {r}: packed bytes not visible on torch's stream"
            back.fill_(r & 0xFF)
            torch.cuda.synchronize()
            mpi.Unpack(packed.data_ptr(), packed.numel(), 0, back.data_ptr(), 1, t)
            assert torch.equal(back[idx.reshape(-1)], exp), f"round {r}: unpacked bytes not visible"
        c1, f1 = mpi.counters(), _ticket_stats()
        assert c1["ticket_waits"] - c0["ticket_waits"] == 120 and c1["sync_waits"] == c0["sync_waits"]
        assert f1[0] - f0[0] == sum(folds) and f1[1] - f0[1] == 120 - sum(folds)
    finally:
        H.tempi_hip_resident_enable(prev)
        mpi.Type_free(t)


@pytest.mark.parametrize("kind", ["noncoherent", "registered", "coherent"])
def test_application_pinned_memory_waits_with_stream_sync(gpu, kind):
    """a kernel writing the APPLICATION's pinned host memory --
    hipHostMalloc(NonCoherent) (coarse-grained), a hipHostRegister'ed buffer,
    or coherent -- completes MPI_Pack (packed side there) and MPI_Unpack
    (strided object there) with hipStreamSynchronize, never a ticket; the
    host reads the bytes right after the call, 40 rounds with fresh data;
    then the buffers are freed and fresh pageable arrays go through copies
    and TEMPI's staged pack. Runs in a process of its own with one HIP runtime
    (tests/mpi_progs/app_pinned.py): inside this process -- TEMPI's runtime
    beside torch's bundled one -- registering, unregistering and freeing host
    memory was followed by one illegal address at a later pageable copy in
    round 4 and again in round 5 (profiles/r05/NOTES.md s21)."""
    import subprocess
    import sys

    root = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
    r = subprocess.run([sys.executable, os.path.join(root, "tests", "mpi_progs", "app_pinned.py"), kind], cwd=root,
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=200)
    assert r.returncode == 0 and "RESULT ok" in r.stdout, r.stdout[-3000:]


PEEL_SHAPES = [  # (block, dims outermost first): rows and strides multiples of 16
    (4096, [(9, 4608 * 70), (3, 4608)]),   # halo y face at a 4608-byte pitch
    (4096, [(3, 4608 * 70), (64, 4608)]),  # halo z face
    (16, [(1000, 48)]),
    (48, [(7, 4096), (11, 64)]),
    (32, [(3000, 32)]),                    # (normalises to one contiguous block)
    (16, []),
]


@pytest.mark.parametrize("remote", [False, True])
def test_pack_unpack_phase8_rows(gpu, remote):
    """Rows of 16-byte multiples starting 8 bytes past a 16-byte boundary (the
    halo's y / z faces), packed at the same phase or at phase 0: single
    objects through tempi_hip_pack / tempi_hip_unpack and the ticketed
    synchronous forms, and one batch of both -- packed bytes and unpacked
    canvases exact against numpy, gaps and neighbours untouched. (Round 6
    ran the phase-matched ones as the peeled copy for a while: a separate
    launch beside the batch's 8-byte-word items, which made the 2-rank halo
    8 % slower; they keep 8-byte words, tempi_hip_word_width == 8.) remote:
    the unpacks' packed side is read with system-scope loads."""
    torch = _torch()
    import tempi_amd

    H = ctypes.CDLL(tempi_amd.LIBTEMPI_HIP)
    vp = ctypes.c_void_p
    for f in ("tempi_hip_pack", "tempi_hip_unpack"):
        getattr(H, f).argtypes = [vp, vp, ctypes.POINTER(HipDesc), vp]
    H.tempi_hip_word_width.argtypes = [vp, vp, ctypes.POINTER(HipDesc)]
    H.tempi_hip_pack_batch.argtypes = [vp, ctypes.c_int, vp]
    H.tempi_hip_unpack_batch.argtypes = [vp, ctypes.c_int, vp]
    for f in ("tempi_hip_pack_ticket", "tempi_hip_unpack_ticket"):
        getattr(H, f).argtypes = [vp, vp, ctypes.POINTER(HipDesc), vp, ctypes.POINTER(ctypes.POINTER(ctypes.c_uint32)),
                                  ctypes.POINTER(ctypes.c_uint32)]
    H.tempi_hip_ticket_wait.argtypes = [vp, ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32]

    def desc(block, dims):
        d = HipDesc()
        d.block, d.ndims = block, len(dims)
        for j, (c, st) in enumerate(dims):
            d.counts[j], d.strides[j] = c, st
        return d

    def index(block, dims):
        idx = np.arange(block, dtype=np.int64)
        for c, st in reversed(dims):
            idx = (np.arange(c, dtype=np.int64)[:, None] * st + idx[None, :]).reshape(-1)
        return idx

    rng = np.random.default_rng(5)
    cases = []
    for k, (bl, dims) in enumerate(PEEL_SHAPES * 2):
        idx = index(bl, dims)
        host = rng.integers(0, 256, int(idx.max()) + 64, dtype=np.uint8)
        src = torch.from_numpy(host).to(gpu)
        ppos = 8 if k < len(PEEL_SHAPES) else 0  # the second round: packed at phase 0 (not peeled)
        packed = torch.full((idx.size + 32,), 0xA5, dtype=torch.uint8, device=gpu)
        cases.append(dict(d=desc(bl, dims), idx=idx, host=host, src=src, packed=packed, ppos=ppos))
    torch.cuda.synchronize()
    for c in cases:
        first, pk = c["src"].data_ptr() + 8, c["packed"].data_ptr() + c["ppos"]
        assert H.tempi_hip_word_width(pk, first, ctypes.byref(c["d"])) == 8

    def check_packed(c):
        got = c["packed"].cpu().numpy()
        n = c["idx"].size
        assert np.array_equal(got[c["ppos"]:c["ppos"] + n], c["host"][8 + c["idx"]])
        assert (got[:c["ppos"]] == 0xA5).all() and (got[c["ppos"] + n:] == 0xA5).all()

    def check_unpacked(c, dst):
        exp = np.full_like(c["host"], 0x5A)
        exp[8 + c["idx"]] = c["host"][8 + c["idx"]]
        assert np.array_equal(dst.cpu().numpy(), exp)

    # single objects, plain and ticketed
    for c in cases[:len(PEEL_SHAPES)]:
        for ticket in (False, True):
            c["packed"].fill_(0xA5)
            dst = torch.full_like(c["src"], 0x5A)
            torch.cuda.synchronize()
            first, pk = c["src"].data_ptr() + 8, c["packed"].data_ptr() + c["ppos"]
            if ticket:
                flag, tk = ctypes.POINTER(ctypes.c_uint32)(), ctypes.c_uint32()
                assert H.tempi_hip_pack_ticket(pk, first, ctypes.byref(c["d"]), None, ctypes.byref(flag),
                                               ctypes.byref(tk)) == 0
                assert H.tempi_hip_ticket_wait(None, flag, tk.value) == 0
            else:
                assert H.tempi_hip_pack(pk, first, ctypes.byref(c["d"]), None) == 0
            torch.cuda.synchronize()
            check_packed(c)
            if remote:
                release_l2(H)
            if ticket:
                assert H.tempi_hip_unpack_ticket(dst.data_ptr() + 8, pk, ctypes.byref(c["d"]), None,
                                                 ctypes.byref(flag), ctypes.byref(tk)) == 0
                assert H.tempi_hip_ticket_wait(None, flag, tk.value) == 0
            else:
                assert H.tempi_hip_unpack(dst.data_ptr() + 8, pk, ctypes.byref(c["d"]), None) == 0
            torch.cuda.synchronize()
            check_unpacked(c, dst)
    # one batch: peeled and ordinary items together
    for c in cases:
        c["packed"].fill_(0xA5)
        c["dst"] = torch.full_like(c["src"], 0x5A)
    items = (HipItem * len(cases))()
    for k, c in enumerate(cases):
        items[k].packed = c["packed"].data_ptr() + c["ppos"]
        items[k].first = c["src"].data_ptr() + 8
        items[k].desc = c["d"]
        items[k].flags = 0
    torch.cuda.synchronize()
    assert H.tempi_hip_pack_batch(items, len(cases), None) == 0
    torch.cuda.synchronize()
    for c in cases:
        check_packed(c)
    for k, c in enumerate(cases):
        items[k].first = c["dst"].data_ptr() + 8
        items[k].flags = ITEM_REMOTE if remote else 0
    if remote:
        release_l2(H)
    assert H.tempi_hip_unpack_batch(items, len(cases), None) == 0
    torch.cuda.synchronize()
    for c in cases:
        check_unpacked(c, c["dst"])


@pytest.mark.parametrize("launch_check", [False, True])
def test_goldens_with_torch_runtime_only(gpu, launch_check):
    """The 153 MPICH goldens through TEMPI in a process whose ONLY HIP
    runtime is torch's (torch imported before libtempi is loaded: the
    configuration bench.py and smoke() run in; this pytest process holds two,
    DESIGN §2.2): packed bytes, positions and unpacked buffers bit-exact, the
    strided cases on the GPU path (tests/mpi_progs/torch_runtime_parity.py).
    launch_check: the same under TEMPI_LAUNCH_CHECK=1 (every launch
    synchronised and checked): the same bytes, no report."""
    import subprocess
    import sys

    root = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
    env = dict(os.environ, **({"TEMPI_LAUNCH_CHECK": "1"} if launch_check else {}))
    r = subprocess.run([sys.executable, os.path.join(root, "tests", "mpi_progs", "torch_runtime_parity.py")],
                       cwd=root, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300, env=env)
    assert r.returncode == 0 and f"RESULT ok {len(CASES)} cases" in r.stdout, r.stdout[-3000:]
    assert "TEMPI_LAUNCH_CHECK" not in r.stdout and "HIP runtimes in this process" not in r.stdout


_TWO_RUNTIMES = """
import sys
sys.path.insert(0, {root!r})
import tempi_amd
mpi = tempi_amd.get_mpi()  # libtempi (and ROCm's runtime) first
import torch  # then torch, which loads its own
torch.cuda.init()
mpi.Init()
mpi.Finalize()
print("RESULT ok")
"""


def test_two_runtimes_reported_at_init(gpu):
    """libtempi loaded before torch leaves two HIP runtimes in
    the process, and MPI_Init says so once, naming both (the torch-first
    order above reports nothing)"""
    import subprocess
    import sys

    root = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
    r = subprocess.run([sys.executable, "-c", _TWO_RUNTIMES.format(root=root)], cwd=root, stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, text=True, timeout=300)
    assert r.returncode == 0 and "RESULT ok" in r.stdout, r.stdout[-3000:]
    warn = [l for l in r.stdout.splitlines() if "HIP runtimes in this process" in l]
    assert len(warn) == 1 and "torch" in warn[0] and warn[0].count("libamdhip64") == 2, r.stdout[-3000:]
