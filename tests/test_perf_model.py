"""Perf-model interpolation (tempi_amd/csrc/core/perf_model.cpp) against the
reference's known-answer tests (/root/reference/test/measure_system.cpp:13-92)
and the perf.json schema round trip. No GPU needed."""
import ctypes
import json
import math

import pytest

import tempi_amd

L = ctypes.CDLL(tempi_amd.LIBTEMPI)
L.tempi_interp_time.restype = ctypes.c_double
L.tempi_interp_time.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.c_int, ctypes.c_int64]
L.tempi_interp_2d.restype = ctypes.c_double
L.tempi_interp_2d.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.c_int, ctypes.c_int, ctypes.c_int64,
                              ctypes.c_int64]
L.tempi_perf_roundtrip.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int]


def t1(v, b):
    arr = (ctypes.c_double * len(v))(*v)
    return L.tempi_interp_time(arr, len(v), b)


def t2(rows, b, x):
    flat = [c for r in rows for c in r]
    arr = (ctypes.c_double * len(flat))(*flat)
    return L.tempi_interp_2d(arr, len(rows), len(rows[0]), b, x)


# /root/reference/test/measure_system.cpp:16-42
@pytest.mark.parametrize("b,exp", [(1, 2), (2, 4), (3, 6), (5, 10), (7, 14)])
def test_interp_time_kat(b, exp):
    assert t1([2, 4, 8, 16], b) == exp


A = [[14, 18, 22], [16, 20, 24]]  # rows 64 B, 256 B; cols block 1, 2, 4


# /root/reference/test/measure_system.cpp:52-89 (bytes=512 is past the table:
# the reference reads out of bounds there; we must not, and must
# still give its answers)
@pytest.mark.parametrize("b,x,exp", [(64, 1, 14), (160, 1, 15), (256, 1, 16), (64, 2, 18), (256, 2, 20),
                                     (64, 3, 20), (64, 4, 22), (160, 3, 21), (512, 1, 32), (512, 3, 44)])
def test_interp_2d_kat(b, x, exp):
    assert t2(A, b, x) == pytest.approx(exp, rel=0, abs=1e-5)


@pytest.mark.parametrize("b, lo, hi, frac", [(1, 0, 0, 0.0), (2, 1, 1, 0.0), (3, 1, 2, 0.5), (4, 2, 2, 0.0),
                                             (5, 2, 3, 0.25)])
def test_log2_floor_ceil(b, lo, hi, frac):
    """the reference's numeric test (/root/reference/test/numeric.cpp:13-26:
    log2_ceil / log2_floor of 1..5), seen through the interpolation that uses
    them: `b` bytes lie between table entries floor(log2 b) and ceil(log2 b)"""
    v = [1.0 + 10.0 * i for i in range(6)]
    assert t1(v, b) == pytest.approx(v[lo] * (1 - frac) + v[hi] * frac, rel=1e-6)


def test_unknown_is_inf():
    assert math.isinf(L.tempi_interp_time((ctypes.c_double * 1)(), 0, 100))


def test_interp_time_beyond_table_scales():
    assert t1([2, 4, 8, 16], 32) == pytest.approx(64)  # 16 s for 8 B, scaled linearly


def test_perf_json_roundtrip():
    doc = {"cudaKernelLaunch": 3.5e-6,
           "intraNodeCpuCpuPingpong": [{"time": 1e-6, "iid": True}, {"time": 2e-6, "iid": False}],
           "intraNodeGpuGpuPingpong": [{"time": 3e-6, "iid": True}],
           "interNodeCpuCpuPingpong": [], "interNodeGpuGpuPingpong": [],
           "d2h": [{"time": 4e-6, "iid": True}], "h2d": [{"time": 5e-6, "iid": True}],
           "packDevice": [[{"time": 1e-5, "iid": True}, {"time": 2e-5, "iid": False}]],
           "unpackDevice": [[{"time": 1e-5, "iid": True}]], "packHost": [], "unpackHost": []}
    out = ctypes.create_string_buffer(1 << 16)
    assert L.tempi_perf_roundtrip(json.dumps(doc).encode(), out, 1 << 16) == 0
    back = json.loads(out.value.decode())
    for k, v in doc.items():
        assert back[k] == v, k


def test_perf_json_rejects_missing_keys():
    out = ctypes.create_string_buffer(1024)
    assert L.tempi_perf_roundtrip(b'{"d2h": []}', out, 1024) != 0


L.tempi_sp800_90b_iid.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.c_int, ctypes.c_int, ctypes.c_uint64]


def iid(v, perms=10000, seed=1):
    return bool(L.tempi_sp800_90b_iid((ctypes.c_double * len(v))(*v), len(v), perms, seed))


def test_iid_rejects_monotone():
    # /root/reference/test/iid.cpp:18-24
    assert not iid([-1, 0, 1, 2, 3, 4, 5])
    assert not iid(list(range(100)))


def test_iid_accepts_random_eventually():
    # /root/reference/test/iid.cpp:26-45: uniform samples of 10 pass eventually
    import numpy as np

    rng = np.random.default_rng(5)
    passed = any(iid(list(rng.uniform(0, 10000, 10)), perms=2000, seed=k) for k in range(20))
    assert passed


def test_iid_rejects_periodic():
    assert not iid([1.0, 2.0] * 50, perms=2000)


def test_shipped_mi355x_model():
    """tempi_amd/data/perf_mi355x.json (apps/measure_system on an MI355X box,
    2 ranks sharing one GPU) parses, round-trips, and has every curve the
    reference's schema names (measure_system.cpp:100-132)."""
    import os

    import tempi_amd

    path = os.path.join(tempi_amd.ROOT, "tempi_amd", "data", "perf_mi355x.json")
    doc = json.load(open(path))
    for k in ("d2h", "h2d", "intraNodeCpuCpuPingpong", "intraNodeGpuGpuPingpong"):
        assert len(doc[k]) == 24 and all(p["time"] > 0 for p in doc[k]), k
    for k in ("packDevice", "unpackDevice", "packHost", "unpackHost"):
        assert len(doc[k]) == 9 and all(len(r) == 10 for r in doc[k]), k
    out = ctypes.create_string_buffer(1 << 17)
    assert L.tempi_perf_roundtrip(open(path, "rb").read(), out, 1 << 17) == 0


L.tempi_batch_ipc_threshold.restype = ctypes.c_int64
L.tempi_batch_ipc_threshold.argtypes = [ctypes.c_char_p, ctypes.c_int64]
INT64_MAX = (1 << 63) - 1


def _synthetic_perf(fixed_ipc, xgmi, pack_host=True):
    """a perf.json whose curves are straight lines: device (un)pack 10 us +
    b / 2 TB/s, host (un)pack 10 us + b / 40 GB/s, CPU ping-pong 1 us + b /
    20 GB/s, and the GPU-GPU ping-pong 20 us at 1 byte, 20 us + fixed_ipc +
    b / xgmi above -- so per batch (marginal costs) IPC costs about fixed_ipc
    + b / xgmi and ONESHOT b / 10 GB/s"""
    def line(a, rate, b):
        return {"time": a + b / rate, "iid": True}
    table = lambda a, rate: [[line(a, rate, 1 << (2 * i + 6)) for _ in range(10)] for i in range(9)]
    gpu = [{"time": 20e-6, "iid": True}] + [line(20e-6 + fixed_ipc, xgmi, 1 << i) for i in range(1, 24)]
    return {"cudaKernelLaunch": 3e-6,
            "intraNodeCpuCpuPingpong": [line(1e-6, 20e9, 1 << i) for i in range(24)],
            "intraNodeGpuGpuPingpong": gpu, "interNodeCpuCpuPingpong": [], "interNodeGpuGpuPingpong": [],
            "d2h": [line(5e-6, 50e9, 1 << i) for i in range(24)], "h2d": [line(5e-6, 50e9, 1 << i) for i in range(24)],
            "packDevice": table(10e-6, 2e12), "unpackDevice": table(10e-6, 2e12),
            "packHost": table(10e-6, 40e9) if pack_host else [], "unpackHost": table(10e-6, 40e9)}


@pytest.mark.parametrize("fixed,xgmi,block,exp", [
    (1.1e-6, 100e9, 512, 16384),   # crossover at ~12 KiB: IPC from 16 KiB up
    (4.4e-6, 100e9, 512, 65536),   # a larger per-message IPC cost moves it to 64 KiB
    (4.4e-6, 100e9, 8, 65536),     # (straight-line tables: the block does not matter)
    (0.0, 100e9, 512, 64),         # IPC cheaper at every size: the smallest priced
    (1.1e-6, 9e9, 512, INT64_MAX),  # xGMI slower than the host path: never IPC
])
def test_batch_ipc_threshold(fixed, xgmi, block, exp):
    """the IPC / ONESHOT threshold of non-blocking AUTO
    sends, priced per batch from a perf.json (perf_model.cpp
    batch_ipc_threshold: marginal cost of each stage's bytes, launch and
    latency paid once per batch), moves with the curves"""
    doc = json.dumps(_synthetic_perf(fixed, xgmi)).encode()
    assert L.tempi_batch_ipc_threshold(doc, block) == exp


def test_batch_ipc_threshold_unknown():
    """a curve the pricing needs is missing (-1: the built-in 4 KiB stays), or
    the document does not parse (-2)"""
    assert L.tempi_batch_ipc_threshold(json.dumps(_synthetic_perf(1.1e-6, 100e9, pack_host=False)).encode(),
                                       512) == -1
    assert L.tempi_batch_ipc_threshold(b"{not json", 512) == -2
