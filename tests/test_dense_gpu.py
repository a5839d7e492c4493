"""The dense-window gather (pack_dense_kernel, pack_kernels.hip): 1- and
2-byte-word rows at inner stride <= 4 x block, taken for MPI_Pack (the other
shapes here exercise the per-word path beside it). Checked byte-exact against oracle/typemap.c on 1-D, 2-D and 3-D
shapes, tiles that straddle outer-dimension segments, odd packed positions
(head / tail chunks), odd buffer alignment and counts > 1; plus a large 1-D
case through an exact strided torch view."""
import random

import numpy as np
import pytest

from oracle import pyoracle
from tests import typezoo

pytestmark = pytest.mark.gpu


def _cases():
    rng = random.Random(11)
    out = []
    for bl in (1, 2, 3, 4, 5, 6, 7, 12, 24, 32):
        for ratio in (1, 2, 3, 8):
            st = bl * ratio + (rng.choice([0, 1]) if ratio > 1 else 0)
            n = max(1, 200000 // bl)
            out.append((f"vector({n},{bl},{st},byte)", 1))
    # 2-D / 3-D subarrays with long inner segments (>= 16 KiB of payload)
    out.append(("subarray(C,[9,40000],[7,20000],[1,3],byte)", 1))          # wide rows: not dense (control)
    out.append(("subarray(C,[30,20002,2],[28,20000,1],[1,1,1],byte)", 1))  # 1-byte rows, stride 2, 28 segments
    out.append(("subarray(C,[12,6003,6],[10,6000,3],[1,2,2],byte)", 2))    # 3-byte rows, stride 6, count 2
    out.append(("subarray(C,[5,8,8200,4],[4,6,8192,2],[1,1,2,1],byte)", 1))  # 3 outer dims
    out.append(("hvector(6,1,100003,vector(20000,1,3,byte))", 1))          # segments not 16-B aligned
    out.append(("subarray(C,[40,40,8],[38,38,3],[1,1,5],byte)", 1))        # short segments: per-word path (control)
    return out


@pytest.mark.parametrize("recipe,count", _cases())
@pytest.mark.parametrize("pos,shift", [(0, 0), (5, 3), (16, 1)])
def test_dense_pack_matches_oracle(mpi, gpu, recipe, count, pos, shift):
    import torch

    tm = pyoracle.TypeMap(recipe)
    origin, buflen = tm.geometry(count)
    host = np.random.default_rng(len(recipe) + pos).integers(0, 256, buflen + shift, dtype=np.uint8)
    t, temps, basic = typezoo.build(mpi, recipe)
    try:
        size = mpi.Pack_size(count, t)
        src = torch.from_numpy(host).to(gpu)
        out = torch.full((pos + size + 32,), 0xA5, dtype=torch.uint8, device=gpu)
        torch.cuda.synchronize()
        before = mpi.counters()["packs"]
        got_pos = mpi.Pack(src.data_ptr() + origin + shift, count, t, out.data_ptr(), pos + size, pos)
        assert mpi.counters()["packs"] == before + 1
        assert got_pos == pos + size
        exp = tm.pack(host, origin + shift, count)
        got = out.cpu().numpy()
        assert np.array_equal(got[pos:pos + size], exp), recipe
        assert (got[:pos] == 0xA5).all() and (got[pos + size:] == 0xA5).all()
    finally:
        typezoo.free(mpi, t, temps, basic)


@pytest.mark.parametrize("bl,st", [(1, 2), (3, 7), (2, 16), (4, 8)])
def test_dense_pack_large_exact(mpi, gpu, bl, st):
    """256 MiB of payload through MPI_Pack against an exact strided view."""
    import torch

    rows = (256 << 20) // bl
    t = mpi.Type_commit(mpi.Type_vector(rows, bl, st, mpi.BYTE))
    try:
        src = (torch.arange(rows * st, dtype=torch.int64, device=gpu) * 7 & 0xFF).to(torch.uint8)
        out = torch.empty(rows * bl, dtype=torch.uint8, device=gpu)
        torch.cuda.synchronize()
        mpi.Pack(src.data_ptr(), 1, t, out.data_ptr(), rows * bl, 0)
        exp = src.view(rows, st)[:, :bl].reshape(-1)
        assert torch.equal(out, exp)
    finally:
        mpi.Type_free(t)
