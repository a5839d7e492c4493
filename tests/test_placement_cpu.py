"""Rank placement (/root/reference/src/
dist_graph_create_adjacent.cpp:55-470) on CPU.

The partitioner (tempi_partition) against exhaustive search over every
balanced assignment of small graphs: it must find the optimum on structured
graphs (interleaved cliques, grids, rings) and stay within 10 % of it on
random ones; sizes are always honoured; the random rule keeps part sizes.
The reference's own partition tests (test/partition_kahip*.cpp) pin only
balance -- KaHIP/METIS output is not reproducible here, so the
oracle is the exhaustive optimum.

Then the MPI path at 8 ranks in two fake nodes (TEMPI_FAKE_NODE_SIZE=4) with
the partitioner and with the random rule: tests/mpi_progs/placement.py."""
import itertools
import random

import pytest

import tempi_amd
from tests import mpi_launch


@pytest.fixture(scope="module")
def mpi():
    return tempi_amd.get_mpi()


def csr(n, wedges):
    """symmetric CSR of {(u, v): w}: both directions listed"""
    adj = {u: [] for u in range(n)}
    for (u, v), w in wedges.items():
        adj[u].append((v, w))
        adj[v].append((u, w))
    xadj, adjncy, wt = [0], [], []
    for u in range(n):
        for v, w in adj[u]:
            adjncy.append(v)
            wt.append(w)
        xadj.append(len(adjncy))
    return xadj, adjncy, wt


def cut_of(wedges, part):
    # each undirected edge is listed in both directions, and the partitioner
    # sums directions: the cut it reports is twice the undirected one
    return 2 * sum(w for (u, v), w in wedges.items() if part[u] != part[v])


def optimum(n, wedges, sizes):
    """exhaustive: the least cut over every assignment with these part sizes"""
    best = None
    labels = [k for k, s in enumerate(sizes) for _ in range(s)]
    for perm in set(itertools.permutations(labels)):
        c = cut_of(wedges, perm)
        best = c if best is None or c < best else best
    return best


def interleaved_cliques(n=8):
    e = {(u, v): 10 for u in range(n) for v in range(u + 1, n) if u % 2 == v % 2}
    e[(0, 1)] = 1
    return n, e


def grid(x, y):
    e = {}
    for j in range(y):
        for i in range(x):
            u = j * x + i
            if i + 1 < x:
                e[(u, u + 1)] = 1
            if j + 1 < y:
                e[(u, u + x)] = 1
    return x * y, e


def parity_rings(n=8):
    e = {}
    for r in range(n):
        e[tuple(sorted((r, (r + 2) % n)))] = e.get(tuple(sorted((r, (r + 2) % n))), 0) + 100
        e[tuple(sorted((r, (r + 1) % n)))] = e.get(tuple(sorted((r, (r + 1) % n))), 0) + 1
    return n, e


@pytest.mark.parametrize("name,graph,sizes", [
    ("cliques-2", interleaved_cliques(), [4, 4]),
    ("cliques-332", interleaved_cliques(), [2, 3, 3]),
    ("grid4x2-2", grid(4, 2), [4, 4]),
    ("grid4x3-3", grid(4, 3), [4, 4, 4]),
    ("grid3x3-uneven", grid(3, 3), [3, 6]),
    ("parity-rings", parity_rings(), [4, 4]),
    ("parity-rings-4", parity_rings(), [2, 2, 2, 2]),
])
def test_structured_optimum(mpi, name, graph, sizes):
    n, e = graph
    part, cut = mpi.partition(*csr(n, e), len(sizes), sizes=sizes)
    assert [part.count(k) for k in range(len(sizes))] == sizes
    assert cut == cut_of(e, part)
    assert cut == optimum(n, e, sizes), (name, part)


@pytest.mark.parametrize("seed", range(12))
def test_random_graph_near_optimum(mpi, seed):
    rng = random.Random(seed)
    n = rng.choice([6, 8, 9])
    e = {}
    for u in range(n):
        for v in range(u + 1, n):
            if rng.random() < 0.45:
                e[(u, v)] = rng.randint(1, 20)
    sizes = [n // 2, n - n // 2] if seed % 2 else [n // 3] * 2 + [n - 2 * (n // 3)]
    part, cut = mpi.partition(*csr(n, e), len(sizes), sizes=sizes)
    assert [part.count(k) for k in range(len(sizes))] == sizes
    assert cut == cut_of(e, part)
    opt = optimum(n, e, sizes)
    assert cut <= 1.1 * opt + 1e-9, (cut, opt)


def test_larger_grid_quality(mpi):
    """a 16 x 16 grid into 4 parts of 64: the optimum is 4 quadrants, cut 32
    edges (64 counted both ways); greedy growth + swaps must get close"""
    n, e = grid(16, 16)
    part, cut = mpi.partition(*csr(n, e), 4)
    assert [part.count(k) for k in range(4)] == [64] * 4
    assert cut == cut_of(e, part) and cut <= 1.5 * 64, cut


def test_random_rule_keeps_sizes(mpi):
    n, e = grid(4, 4)
    part, cut = mpi.partition(*csr(n, e), 4, method=1)
    assert sorted(part) == sorted([k for k in range(4) for _ in range(4)])
    assert cut == cut_of(e, part)


def test_bad_input(mpi):
    n, e = grid(3, 3)
    assert mpi.partition(*csr(n, e), 2)[1] == -1  # 9 vertices do not split evenly
    assert mpi.partition(*csr(n, e), 2, sizes=[4, 4])[1] == -1  # sizes do not add up to n
    assert mpi.partition(*csr(n, e), 2, sizes=[4, 5])[1] >= 0


@pytest.mark.parametrize("method", ["TEMPI_PLACEMENT_KAHIP", "TEMPI_PLACEMENT_METIS", "TEMPI_PLACEMENT_RANDOM"])
def test_placement_mpi(method):
    rc, out = mpi_launch.run(8, mpi_launch.py("placement.py"), env={method: "", "TEMPI_FAKE_NODE_SIZE": "4"},
                             timeout=180)
    assert rc == 0 and "RESULT errors=0" in out, out[-3000:]


def test_placement_off_by_default():
    """no TEMPI_PLACEMENT_*: reorder = 1 is the library's (ranks unchanged)"""
    rc, out = mpi_launch.run(4, mpi_launch.py("placement.py", "--expect-none"), env={"TEMPI_FAKE_NODE_SIZE": "2"},
                             timeout=180)
    assert rc == 0 and "RESULT errors=0" in out, out[-3000:]


@pytest.mark.parametrize("n, node", [(4, 2), (8, 4), (8, 2)])
@pytest.mark.parametrize("method", ["TEMPI_PLACEMENT_METIS", "TEMPI_PLACEMENT_RANDOM"])
def test_reference_pairs_graph(n, node, method):
    """the reference's dist_graph_create_adjacent test: rank <-> rank + n/2"""
    rc, out = mpi_launch.run(n, mpi_launch.py("dist_graph_pairs.py"), env={method: "", "TEMPI_FAKE_NODE_SIZE": str(node)},
                             timeout=180)
    assert rc == 0 and "RESULT errors=0" in out, out[-3000:]
