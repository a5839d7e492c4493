// tempi_amd/csrc/core/placement.cpp -- see placement.hpp
#include "placement.hpp"

#include "log.hpp"
#include "next_mpi.hpp"
#include "topology.hpp"
#include "trace.hpp"

#include <algorithm>
#include <cstdlib>
#include <limits>
#include <map>
#include <random>
#include <utility>

namespace tempi {
namespace placement {

namespace {
Info lastInfo;
// one generator for every random placement of the process, seeded 0, as the
// reference's (partition.cpp:15): every rank draws the same sequence
std::default_random_engine randomGen(0);

// conn[v] for the part being grown: pick the unassigned vertex with the
// largest connection, scanning from `start` so restarts differ
int pick(const std::vector<int> &part, const std::vector<int64_t> &conn, int start) {
  const int n = int(part.size());
  int best = -1;
  int64_t bestConn = -1;
  for (int j = 0; j < n; ++j) {
    const int v = (start + j) % n;
    if (part[size_t(v)] >= 0) continue;
    if (conn[size_t(v)] > bestConn) {
      best = v;
      bestConn = conn[size_t(v)];
    }
  }
  return best;
}

// graph growing: part k starts at the unassigned vertex most connected to
// the parts already grown (the first at `seed`) and takes, one at a time,
// the unassigned vertex most connected to it
std::vector<int> grow(const Graph &g, const std::vector<int> &sizes, int seed) {
  const int n = g.n;
  std::vector<int> part(size_t(n), -1);
  std::vector<int64_t> toAssigned(size_t(n), 0), conn(size_t(n), 0);
  int assigned = 0;
  for (size_t k = 0; k < sizes.size(); ++k) {
    if (sizes[k] <= 0) continue;
    const int s = assigned == 0 ? seed : pick(part, toAssigned, seed);
    std::fill(conn.begin(), conn.end(), 0);
    int v = s;
    for (int taken = 0; taken < sizes[k] && v >= 0; ++taken) {
      part[size_t(v)] = int(k);
      ++assigned;
      for (int e = g.xadj[size_t(v)]; e < g.xadj[size_t(v) + 1]; ++e) {
        conn[size_t(g.adj[size_t(e)])] += g.w[size_t(e)];
        toAssigned[size_t(g.adj[size_t(e)])] += g.w[size_t(e)];
      }
      if (taken + 1 < sizes[k]) v = pick(part, conn, seed);
    }
  }
  return part;
}

// balance-preserving refinement: for each vertex u, the swap with a vertex
// of another part that lowers the cut most, applied when it lowers it at all;
// passes until none does. ext[v * P + p] = weight from v into part p.
void refine(const Graph &g, int P, std::vector<int> &part, int maxPasses) {
  const int n = g.n;
  std::vector<int64_t> ext(size_t(n) * size_t(P), 0), wu(size_t(n), 0);
  for (int u = 0; u < n; ++u)
    for (int e = g.xadj[size_t(u)]; e < g.xadj[size_t(u) + 1]; ++e)
      ext[size_t(u) * P + size_t(part[size_t(g.adj[size_t(e)])])] += g.w[size_t(e)];
  for (int pass = 0; pass < maxPasses; ++pass) {
    bool improved = false;
    for (int u = 0; u < n; ++u) {
      const int a = part[size_t(u)];
      for (int e = g.xadj[size_t(u)]; e < g.xadj[size_t(u) + 1]; ++e) wu[size_t(g.adj[size_t(e)])] = g.w[size_t(e)];
      const int64_t *eu = &ext[size_t(u) * P];
      int64_t best = 0;
      int bv = -1;
      for (int v = 0; v < n; ++v) {
        const int b = part[size_t(v)];
        if (b == a) continue;
        const int64_t *ev = &ext[size_t(v) * P];
        const int64_t gain = eu[b] - eu[a] + ev[a] - ev[b] - 2 * wu[size_t(v)];
        if (gain > best) {
          best = gain;
          bv = v;
        }
      }
      for (int e = g.xadj[size_t(u)]; e < g.xadj[size_t(u) + 1]; ++e) wu[size_t(g.adj[size_t(e)])] = 0;
      if (bv < 0) continue;
      const int b = part[size_t(bv)];
      part[size_t(u)] = b;
      part[size_t(bv)] = a;
      for (int e = g.xadj[size_t(u)]; e < g.xadj[size_t(u) + 1]; ++e) {
        ext[size_t(g.adj[size_t(e)]) * P + size_t(a)] -= g.w[size_t(e)];
        ext[size_t(g.adj[size_t(e)]) * P + size_t(b)] += g.w[size_t(e)];
      }
      for (int e = g.xadj[size_t(bv)]; e < g.xadj[size_t(bv) + 1]; ++e) {
        ext[size_t(g.adj[size_t(e)]) * P + size_t(b)] -= g.w[size_t(e)];
        ext[size_t(g.adj[size_t(e)]) * P + size_t(a)] += g.w[size_t(e)];
      }
      improved = true;
    }
    if (!improved) break;
  }
}
} // namespace

Graph make_graph(int n, const std::vector<Edge> &edges) {
  std::map<std::pair<int, int>, int64_t> acc;
  for (const Edge &e : edges) {
    if (e.u == e.v || e.u < 0 || e.v < 0 || e.u >= n || e.v >= n) continue;
    acc[{std::min(e.u, e.v), std::max(e.u, e.v)}] += e.w;
  }
  Graph g;
  g.n = n;
  g.xadj.assign(size_t(n) + 1, 0);
  for (const auto &kv : acc) {
    ++g.xadj[size_t(kv.first.first) + 1];
    ++g.xadj[size_t(kv.first.second) + 1];
  }
  for (int v = 0; v < n; ++v) g.xadj[size_t(v) + 1] += g.xadj[size_t(v)];
  g.adj.resize(size_t(g.xadj[size_t(n)]));
  g.w.resize(g.adj.size());
  std::vector<int> fill(g.xadj.begin(), g.xadj.end() - 1);
  for (const auto &kv : acc) {
    const int u = kv.first.first, v = kv.first.second;
    g.adj[size_t(fill[size_t(u)])] = v;
    g.w[size_t(fill[size_t(u)]++)] = kv.second;
    g.adj[size_t(fill[size_t(v)])] = u;
    g.w[size_t(fill[size_t(v)]++)] = kv.second;
  }
  return g;
}

int64_t edge_cut(const Graph &g, const std::vector<int> &part) {
  int64_t cut = 0;
  for (int u = 0; u < g.n; ++u)
    for (int e = g.xadj[size_t(u)]; e < g.xadj[size_t(u) + 1]; ++e) {
      const int v = g.adj[size_t(e)];
      if (v > u && part[size_t(u)] != part[size_t(v)]) cut += g.w[size_t(e)];
    }
  return cut;
}

std::vector<int> partition(const Graph &g, const std::vector<int> &sizes) {
  const int n = g.n, P = int(sizes.size());
  if (P <= 1 || n == 0) return std::vector<int>(size_t(n), 0);
  // restarts from different seeds: cheap for the rank counts a placement
  // sees (each is O(n^2) per refinement pass)
  const int restarts = n <= 64 ? std::min(n, 16) : n <= 512 ? 8 : n <= 4096 ? 2 : 1;
  const int passes = n <= 4096 ? 20 : 4;
  std::vector<int> best;
  int64_t bestCut = std::numeric_limits<int64_t>::max();
  for (int r = 0; r < restarts; ++r) {
    std::vector<int> part = grow(g, sizes, int(int64_t(r) * n / restarts));
    refine(g, P, part, passes);
    const int64_t c = edge_cut(g, part);
    if (c < bestCut) {
      bestCut = c;
      best = std::move(part);
    }
  }
  return best;
}

std::vector<int> random_parts(const std::vector<int> &sizes) {
  std::vector<int> p;
  for (size_t k = 0; k < sizes.size(); ++k) p.insert(p.end(), size_t(std::max(0, sizes[k])), int(k));
  std::shuffle(p.begin(), p.end(), randomGen);
  return p;
}

bool create(MPI_Comm comm_old, int indegree, const int sources[], const int sourceweights[], int outdegree,
            const int destinations[], const int destweights[], MPI_Info info, int reorder,
            MPI_Comm *comm_dist_graph, int *rc) {
  if (env.placement == PlacementMethod::NONE || !reorder) return false;
  int size = 0, rank = 0;
  MPI_Comm_size(comm_old, &size);
  next.MPI_Comm_rank(comm_old, &rank);

  // the nodes of comm_old's ranks, numbered by first appearance, and each
  // node's ranks in order (topology.cpp:34-90 of the reference)
  int fake = 0;
  if (const char *s = std::getenv("TEMPI_FAKE_NODE_SIZE")) fake = std::max(0, std::atoi(s));
  std::map<int, int> label;
  std::vector<int> nodeOfRank(static_cast<size_t>(size));
  std::vector<std::vector<int>> ranksOfNode;
  for (int r = 0; r < size; ++r) {
    const int w = topology::world_rank(comm_old, r);
    const int key = fake > 0 ? w / fake : topology::node_of_world(w);
    auto it = label.find(key);
    if (it == label.end()) {
      it = label.emplace(key, int(ranksOfNode.size())).first;
      ranksOfNode.emplace_back();
    }
    nodeOfRank[size_t(r)] = it->second;
    ranksOfNode[size_t(it->second)].push_back(r);
  }
  const int nodes = int(ranksOfNode.size());
  if (nodes <= 1 || size / nodes <= 1) return false; // the reference's guard (:96-98)
  TEMPI_RANGE("placement");
  std::vector<int> sizes;
  for (const auto &v : ranksOfNode) sizes.push_back(int(v.size()));

  MPI_Comm priv;
  MPI_Comm_dup(comm_old, &priv);
  const bool weighted = sourceweights != MPI_UNWEIGHTED && destweights != MPI_UNWEIGHTED;
  auto wt = [&](const int *ws, int i) { return weighted && indegree + outdegree > 0 ? ws[i] : 1; };
  std::vector<int> part(static_cast<size_t>(size));
  int64_t cuts[2] = {0, 0};
  if (env.placement == PlacementMethod::RANDOM) {
    part = random_parts(sizes); // every rank draws the same (the reference does not broadcast it either)
  } else {
    // every rank's edges as (u, v, w) triples to rank 0 (:111-144)
    std::vector<int> mine;
    for (int i = 0; i < indegree; ++i) mine.insert(mine.end(), {sources[i], rank, wt(sourceweights, i)});
    for (int i = 0; i < outdegree; ++i) mine.insert(mine.end(), {rank, destinations[i], wt(destweights, i)});
    const int cnt = int(mine.size());
    std::vector<int> counts(static_cast<size_t>(size), 0), displs(static_cast<size_t>(size), 0), all;
    MPI_Gather(&cnt, 1, MPI_INT, counts.data(), 1, MPI_INT, 0, priv);
    if (rank == 0) {
      for (int r = 1; r < size; ++r) displs[size_t(r)] = displs[size_t(r) - 1] + counts[size_t(r) - 1];
      all.resize(size_t(displs[size_t(size) - 1] + counts[size_t(size) - 1]) + 1);
    }
    MPI_Gatherv(mine.data(), cnt, MPI_INT, all.data(), counts.data(), displs.data(), MPI_INT, 0, priv);
    if (rank == 0) {
      std::vector<Edge> edges;
      for (size_t i = 0; i + 2 < all.size(); i += 3) edges.push_back({all[i], all[i + 1], int64_t(all[i + 2])});
      const Graph g = make_graph(size, edges);
      part = partition(g, sizes);
      cuts[0] = edge_cut(g, nodeOfRank);
      cuts[1] = edge_cut(g, part);
      LOG_INFO("placement: " << nodes << " nodes, edge cut " << cuts[0] << " in library order, " << cuts[1]
                             << " placed");
    }
    MPI_Bcast(part.data(), size, MPI_INT, 0, priv);
    MPI_Bcast(cuts, 2, MPI_INT64_T, 0, priv);
  }

  // make_placement (topology.cpp:97-144): application rank ar runs on the
  // next unused process of node part[ar]
  std::vector<int> appRank(static_cast<size_t>(size)), libRank(static_cast<size_t>(size)), nextIdx(static_cast<size_t>(nodes), 0);
  for (int ar = 0; ar < size; ++ar) {
    const int node = part[size_t(ar)];
    const int cr = ranksOfNode[size_t(node)][size_t(nextIdx[size_t(node)]++)];
    appRank[size_t(cr)] = ar;
    libRank[size_t(ar)] = cr;
  }

  // this process becomes application rank q and presents old rank q's edges
  // (:400-431): they come from process q; its own go to the process that
  // becomes application rank `rank`
  const int q = appRank[size_t(rank)], to = libRank[size_t(rank)];
  int mineHdr[3] = {indegree, outdegree, weighted ? 1 : 0}, hdr[3] = {0, 0, 0};
  next.MPI_Sendrecv(mineHdr, 3, MPI_INT, to, 0, hdr, 3, MPI_INT, q, 0, priv, MPI_STATUS_IGNORE);
  std::vector<int> out(sources, sources + indegree);
  if (weighted) out.insert(out.end(), sourceweights, sourceweights + indegree);
  out.insert(out.end(), destinations, destinations + outdegree);
  if (weighted) out.insert(out.end(), destweights, destweights + outdegree);
  const int inQ = hdr[0], outQ = hdr[1], wQ = hdr[2];
  std::vector<int> in(size_t((inQ + outQ) * (wQ ? 2 : 1)) + 1);
  next.MPI_Sendrecv(out.data(), int(out.size()), MPI_INT, to, 1, in.data(), int(in.size()) - 1, MPI_INT, q, 1, priv,
                    MPI_STATUS_IGNORE);
  const int *src = in.data(), *srcW = src + inQ, *dst = srcW + (wQ ? inQ : 0), *dstW = dst + outQ;

  // the library builds the graph over comm_old reordered by application
  // rank, without reordering again: its ranks are the application's
  MPI_Comm byApp;
  MPI_Comm_split(priv, 0, q, &byApp);
  *rc = next.MPI_Dist_graph_create_adjacent(byApp, inQ, src, wQ ? (inQ ? srcW : MPI_WEIGHTS_EMPTY) : MPI_UNWEIGHTED,
                                            outQ, dst, wQ ? (outQ ? dstW : MPI_WEIGHTS_EMPTY) : MPI_UNWEIGHTED, info,
                                            0, comm_dist_graph);
  next.MPI_Comm_free(&byApp);
  next.MPI_Comm_free(&priv);
  lastInfo = Info{1, nodes, int(env.placement), q, cuts[0], cuts[1]};
  return true;
}

Info last() { return lastInfo; }

} // namespace placement
} // namespace tempi
