"""The config 3-5 apps on pageable host buffers (TEMPI_BENCH_HOST=1), on CPU:
the library path the reference takes for host memory, which is also
bench.py's CPU baseline (TEMPI_DISABLE=1), and the same apps with TEMPI
loaded and active but no GPU (every call reaches the library through the
interposer). Every exchanged byte is checked; the halo runs the
decompositions of 1, 2, 4 and 8 ranks, the alltoallv config 5's 8 ranks."""
import json
import os

import pytest

from tests import mpi_launch

LIB = os.path.join(mpi_launch.ROOT, "tempi_amd", "lib")
HOST = {"TEMPI_BENCH_HOST": "1"}
MODES = {"library": dict(HOST, TEMPI_DISABLE="1"), "interposed": HOST}


def _json(out):
    for line in out.splitlines():
        if line.startswith("{"):
            return json.loads(line)
    raise AssertionError(out[-3000:])


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("ranks,grid,extra", [(1, "24", []), (2, "24", []), (4, "24", []), (8, "24", []),
                                              (8, "24", ["--neighbor"]), (3, "18", []),
                                              (8, "24", ["--reorder"]), (8, "24", ["--reorder", "--neighbor"])])
def test_halo_host(mode, ranks, grid, extra):
    env = dict(MODES[mode])
    if "--reorder" in extra:  # placement over two fake nodes (the library ignores it: ranks unchanged)
        env.update(TEMPI_PLACEMENT_KAHIP="", TEMPI_FAKE_NODE_SIZE="4")
    rc, out = mpi_launch.run(ranks, [os.path.join(LIB, "halo_exchange"), "2", grid, "--quants", "2", "--check"] + extra,
                             env=env, timeout=200)
    r = _json(out)
    assert rc == 0 and r["checked"] and r["errors"] == 0 and r["buffers"] == "host", out[-3000:]
    if ranks == 8:
        assert r["dims"] == [2, 2, 2]


def test_halo_host_check_finds_a_planted_error():
    rc, out = mpi_launch.run(2, [os.path.join(LIB, "halo_exchange"), "1", "16", "--quants", "1", "--check-control"],
                             env=MODES["library"], timeout=120)
    assert _json(out)["errors"] == 1, out[-3000:]


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("total,block", [(1024, 8), (1 << 20, 64), (1 << 20, 1)])
def test_pingpong_host(mode, total, block):
    rc, out = mpi_launch.run(2, [os.path.join(LIB, "pingpong_nd"), "3", str(total), str(block), "--check"],
                             env=MODES[mode], timeout=120)
    r = _json(out)
    assert rc == 0 and r["checked"] and r["errors"] == 0 and r["buffers"] == "host", out[-3000:]


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("ranks,scale,density", [(8, 1000, 1.0), (8, 10, 0.5), (8, 100000, 0.125), (3, 100, 1.0)])
def test_alltoallv_host(mode, ranks, scale, density):
    rc, out = mpi_launch.run(ranks, [os.path.join(LIB, "alltoallv_sparse"), "2", "--scale", str(scale), "--density",
                                     str(density), "--check"], env=MODES[mode], timeout=120)
    r = _json(out)
    assert rc == 0 and r["checked"] and r["errors"] == 0 and r["buffers"] == "host", out[-3000:]


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("ranks,scale,density,extra", [
    (8, 1000, 0.5, []), (8, 100000, 0.125, []), (3, 100, 1.0, []), (8, 10, 1.0, ["--no-reorder"]),
    (8, 1000, 0.5, ["placed"])])
def test_nbr_alltoallv_host(mode, ranks, scale, density, extra):
    """config 5's neighbourhood form (bench_nbr_alltoallv_random_sparse): the
    matrix as a distributed graph created with reorder = 1, then
    MPI_Neighbor_alltoallv; "placed": TEMPI_PLACEMENT_KAHIP over two fake
    nodes of 4 ranks (the library ignores it)"""
    env = dict(MODES[mode])
    if "placed" in extra:
        env.update(TEMPI_PLACEMENT_KAHIP="", TEMPI_FAKE_NODE_SIZE="4")
        extra = []
    rc, out = mpi_launch.run(ranks, [os.path.join(LIB, "alltoallv_sparse"), "2", "--scale", str(scale), "--density",
                                     str(density), "--check", "--neighbor"] + extra, env=env, timeout=120)
    r = _json(out)
    assert rc == 0 and r["checked"] and r["errors"] == 0 and r["buffers"] == "host", out[-3000:]
    assert r["api"] == "MPI_Neighbor_alltoallv" and r["reorder"] == ("--no-reorder" not in extra)
    assert r["total_on_node_bytes"] + r["total_off_node_bytes"] > 0


def test_nbr_alltoallv_placement_cuts_off_node_bytes():
    """with two fake nodes, TEMPI's placement of the reference's matrix moves
    fewer bytes between nodes than the identity placement (reorder = 0)"""
    env = dict(MODES["interposed"], TEMPI_PLACEMENT_KAHIP="", TEMPI_FAKE_NODE_SIZE="4")
    off = {}
    for extra in ([], ["--no-reorder"]):
        rc, out = mpi_launch.run(8, [os.path.join(LIB, "alltoallv_sparse"), "1", "--scale", "1000", "--density",
                                     "0.5", "--check", "--neighbor"] + extra, env=env, timeout=120)
        r = _json(out)
        assert rc == 0 and r["errors"] == 0 and r["nodes"] == 2, out[-3000:]
        off[bool(extra)] = r["total_off_node_bytes"]
    assert off[False] < off[True], off


@pytest.mark.parametrize("mode", list(MODES))
def test_mpi_pack_host(mode):
    """the reference's bench_mpi_pack shapes (1 KiB per element here) on host
    buffers: every point's packed bytes checked against the type map"""
    rc, out = mpi_launch.run(1, [os.path.join(LIB, "mpi_pack"), "2", "--host", "--max-target", "1024"],
                             env=MODES[mode], timeout=120)
    recs = [json.loads(l) for l in out.splitlines() if l.startswith("{")]
    assert rc == 0 and len(recs) == 2 * 9 * 3, out[-3000:]
    assert all(r["errors"] == 0 and r["buffers"] == "host" and r["pack_MiBps"] > 0 for r in recs)


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("ranks", [2, 4, 3])
def test_pingpong_1d_host(mode, ranks):
    """the reference's bench_mpi_pingpong_1d (MPI_BYTE, all pairs r <-> r + N/2;
    an odd rank out idles) on host buffers, every byte checked"""
    rc, out = mpi_launch.run(ranks, [os.path.join(LIB, "pingpong_1d"), "2", "65536", str(1 << 21), "--check"],
                             env=MODES[mode], timeout=120)
    recs = [json.loads(l) for l in out.splitlines() if l.startswith("{")]
    assert rc == 0 and len(recs) == 2 and all(r["errors"] == 0 and r["checked"] for r in recs), out[-3000:]
    assert recs[0]["pairs"] == ranks // 2


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("ranks", [2, 3])
def test_mpi_isend_host(mode, ranks):
    """the reference's bench_mpi_isend (10 overlapping MPI_BYTE messages each
    way between ranks 0 and 1, others idle) on host buffers, every byte checked"""
    rc, out = mpi_launch.run(ranks, [os.path.join(LIB, "mpi_isend"), "2", "1", "4096", str(1 << 20), "--check"],
                             env=MODES[mode], timeout=120)
    recs = [json.loads(l) for l in out.splitlines() if l.startswith("{")]
    assert rc == 0 and len(recs) == 3 and all(r["errors"] == 0 and r["checked"] for r in recs), out[-3000:]
    assert all(r["tags"] == 10 and r["buffers"] == "host" for r in recs)



def test_measure_system_host_curves(tmp_path):
    """apps/measure_system (the perf.json writer, /root/reference/src/internal/
    measure_system.cu:377-606) at 2 ranks without a GPU: the host ping-pong
    curve over 2^0 .. 2^20 bytes with IID flags, the GPU curves empty; the
    file round-trips through TEMPI's parser, and TEMPI then loads it from
    TEMPI_CACHE_DIR -- with no GPU curves AUTO keeps its built-in policy"""
    from tests import perf_json_check

    out = tmp_path / "perf.json"
    rc, log = mpi_launch.run(2, [os.path.join(LIB, "measure_system"), "--quick", "--out", str(out)], timeout=200)
    assert rc == 0 and '"gpu": false' in log, log[-3000:]
    doc, bad = perf_json_check.check(str(out), gpu=False)
    assert not bad, bad[:10]
    rc, log = mpi_launch.run(1, mpi_launch.py("perf_pick.py"), env={"TEMPI_CACHE_DIR": str(tmp_path)}, timeout=120)
    assert rc == 0, log[-3000:]
    pick = json.loads(next(l for l in log.splitlines() if l.startswith("{")))
    assert pick["loaded"] == 1 and pick["source"] == str(out), pick
    assert all(fm == 0 for _, _, _, fm in pick["picks"]), pick  # no GPU curve priced


def test_timeline_records_entry_points(tmp_path):
    """TEMPI_TIMELINE=PREFIX (core/trace.cpp) writes PREFIX.r<rank>.csv at
    MPI_Finalize: every interposed MPI_Isend / MPI_Irecv / MPI_Wait as a
    begin / end pair on CLOCK_BOOTTIME, in order, one file per rank, which
    tools/halo_timeline.py then splits into substeps"""
    import csv
    import subprocess
    import sys

    pre = str(tmp_path / "tl")
    rc, out = mpi_launch.run(2, [os.path.join(LIB, "halo_exchange"), "2", "16", "--quants", "1"],
                             env={"TEMPI_TIMELINE": pre, "TEMPI_BENCH_HOST": "1"}, timeout=120)
    assert rc == 0, out[-3000:]
    for r in (0, 1):
        rows = list(csv.DictReader(open(f"{pre}.r{r}.csv")))
        ns = [int(x["ns"]) for x in rows]
        assert ns == sorted(ns) and len(rows) > 100
        for name in ("MPI_Isend", "MPI_Irecv", "MPI_Wait", "MPI_Barrier"):
            b = sum(1 for x in rows if x["name"] == name and x["phase"] == "0")
            e = sum(1 for x in rows if x["name"] == name and x["phase"] == "1")
            assert b == e > 0, (r, name, b, e)
    # 3 iterations x 3 substeps of 26 sends each; the analysis finds them
    # (no batches on host buffers: all idle is host time)
    p = subprocess.run([sys.executable, os.path.join(mpi_launch.ROOT, "tools", "halo_timeline.py"), f"{pre}.r0.csv",
                        "-", "3"], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=60)
    assert p.returncode == 0 and "substeps" in p.stdout, p.stdout


def test_nonblocking_ipc_threshold_follows_node_perf_json(tmp_path):
    """non-blocking AUTO sends take IPC from a threshold
    priced per batch from THIS node's perf.json (TEMPI_CACHE_DIR) when one was
    measured here -- synthetic files whose curves cross at ~150 B and ~1.2 KiB
    move it to 256 B and 2 KiB, and tempi_choose_method's non-blocking picks
    follow it; one crossing at ~12 KiB is held at the built-in 4 KiB, which
    the model may lower but never raise (p2p_routes.cpp) -- and stay at 4 KiB
    with only the shipped model (measured with both ranks on one GPU)."""
    from tests.test_perf_model import _synthetic_perf

    def pick(cache):
        rc, log = mpi_launch.run(1, mpi_launch.py("perf_pick.py"), env={"TEMPI_CACHE_DIR": str(cache)}, timeout=120)
        assert rc == 0, log[-3000:]
        return json.loads(next(l for l in log.splitlines() if l.startswith("{")))

    shipped = pick(tmp_path / "none")
    assert shipped["loaded"] == 1 and shipped["source"].endswith("perf_mi355x.json"), shipped
    assert shipped["nb_threshold"] == [[8, 4096, 0], [512, 4096, 0]], shipped
    for fixed, exp in ((0.0135e-6, 256), (0.11e-6, 2048), (1.1e-6, 4096)):
        d = tmp_path / f"node_{exp}"
        d.mkdir()
        (d / "perf.json").write_text(json.dumps(_synthetic_perf(fixed, 100e9)))
        node = pick(d)
        assert node["source"] == str(d / "perf.json"), node
        assert node["nb_threshold"] == [[8, exp, 1], [512, exp, 1]], node
        for b, m, fm in node["nb_picks"]:  # 4 = IPC, 1 = ONESHOT (co-located peer)
            assert (m, fm) == ((4, 1) if b >= exp else (1, 1)), (b, m, fm, node)
