// tempi_amd/csrc/core/interpose_neighbor.cpp -- neighbourhood collectives on
// device buffers, and the communicator entry points of the reference's
// exported set.
//
//   MPI_Neighbor_alltoallw  reference: /root/reference/src/neighbor_alltoallw.cpp:11-18
//                           -> neighbor_alltoallw::isir
//                           (/root/reference/src/internal/neighbor_alltoallw.cpp:19-77):
//                           one MPI_Isend / MPI_Irecv per edge, so device
//                           buffers go through TEMPI's packers.
//   MPI_Neighbor_alltoallv  reference: /root/reference/src/neighbor_alltoallv.cpp:12-24
//                           (a pure passthrough there: a non-GPU-aware MPI then
//                           reads device memory from the host). Here it takes
//                           the same per-edge route as alltoallw when any block
//                           is on the GPU.
//   MPI_Dist_graph_create_adjacent  reference: src/dist_graph_create_adjacent.cpp:55-470
//                           -> placement::create (core/placement.hpp) when
//                           reorder = 1, TEMPI_PLACEMENT_* is set and the
//                           communicator spans several nodes.
//   MPI_Dist_graph_neighbors, MPI_Comm_rank
//                           reference: src/dist_graph_neighbors.cpp:13-49,
//                           src/comm_rank.cpp:13-27 translate library ranks to
//                           application ranks there. A placed communicator is
//                           created in the application's rank order here, so
//                           these forward unchanged.
//   MPI_Comm_free           reference: src/comm_free.cpp:13-19 -- drop the
//                           handle's cached state (world-rank map, private
//                           duplicate) before the library may reuse it.
//
// Differences from the reference's isir: receives are posted before sends
// (the transport then launches arrived messages' copies while sends are still
// being queued), completion goes through one MPI_Waitall, messages travel on
// a private duplicate of the communicator instead of a reserved tag, and
// Cartesian and (non-distributed) graph topologies are handled too, with
// MPI_PROC_NULL neighbours skipped. Edges between the same pair of ranks are
// matched in edge order, as the library's own implementation does.
#include "trace.hpp"
#include "counters.hpp"
#include "gpu.hpp"
#include "mt.hpp"
#include "next_mpi.hpp"
#include "p2p.hpp"
#include "placement.hpp"
#include "state.hpp"
#include "type_cache.hpp"

#include "tempi_mpi.h"

#include <cstdlib>
#include <cstring>
#include <list>
#include <unordered_map>
#include <vector>

#define TEMPI_EXPORT extern "C" __attribute__((visibility("default")))

namespace tempi {

MPI_Comm private_comm(MPI_Comm comm); // interpose_coll.cpp
void comm_release(MPI_Comm comm);

namespace {

// incoming / outgoing neighbours in MPI's canonical order; false when the
// communicator has no topology (the library then raises the error)
bool query_neighbours(MPI_Comm comm, std::vector<int> &in, std::vector<int> &out) {
  int topo = MPI_UNDEFINED;
  MPI_Topo_test(comm, &topo);
  in.clear();
  out.clear();
  if (topo == MPI_DIST_GRAPH) {
    int indeg = 0, outdeg = 0, weighted = 0;
    MPI_Dist_graph_neighbors_count(comm, &indeg, &outdeg, &weighted);
    in.resize(size_t(indeg));
    out.resize(size_t(outdeg));
    std::vector<int> iw(size_t(indeg) + 1), ow(size_t(outdeg) + 1);
    next.MPI_Dist_graph_neighbors(comm, indeg, in.data(), weighted ? iw.data() : MPI_UNWEIGHTED, outdeg, out.data(),
                                  weighted ? ow.data() : MPI_UNWEIGHTED);
    return true;
  }
  if (topo == MPI_CART) {
    int nd = 0;
    MPI_Cartdim_get(comm, &nd);
    for (int d = 0; d < nd; ++d) {
      int lo = MPI_PROC_NULL, hi = MPI_PROC_NULL;
      MPI_Cart_shift(comm, d, 1, &lo, &hi);
      in.push_back(lo);
      in.push_back(hi);
    }
    out = in;
    return true;
  }
  if (topo == MPI_GRAPH) {
    int rank = 0, n = 0;
    next.MPI_Comm_rank(comm, &rank);
    MPI_Graph_neighbors_count(comm, rank, &n);
    in.resize(size_t(n));
    MPI_Graph_neighbors(comm, rank, n, in.data());
    out = in;
    return true;
  }
  return false;
}

// a topology's neighbour lists never change: kept per communicator until it
// is freed (neighbourhood_forget)
struct Neighbours {
  std::vector<int> in, out;
};
std::unordered_map<MPI_Comm, Neighbours> neighbourCache;

const Neighbours *neighbours(MPI_Comm comm) {
  auto it = neighbourCache.find(comm);
  if (it != neighbourCache.end()) return &it->second;
  Neighbours n;
  if (!query_neighbours(comm, n.in, n.out)) return nullptr;
  return &neighbourCache.emplace(comm, std::move(n)).first->second;
}

// The per-call plan of a neighbourhood collective: which edges are self
// edges carried as strided -> strided copies, and those copies (descriptors
// resolved, pointers classified). The halo's MPI_Neighbor_alltoallw repeats
// the same few calls every iteration, and re-planning 26 self edges cost
// ~5 us of each ~63 us call. A plan is reused
// while the call is the same -- communicator, buffers, every count,
// displacement and type handle -- no type record was added or dropped since
// (type_generation), and both buffers still classify to the same device.
struct Plan {
  MPI_Comm comm;
  const void *sbuf;
  void *rbuf;
  std::vector<int> scounts, rcounts;
  std::vector<MPI_Aint> sdispls, rdispls;
  std::vector<MPI_Datatype> stypes, rtypes;
  uint64_t typeGen = 0;
  int sdev = -2, rdev = -2;
  MPI_Comm priv = MPI_COMM_NULL;
  int me = 0;
  std::vector<char> doneIn, doneOut;
  p2p::LocalCopies copies;
};
constexpr size_t kMaxPlans = 64;
std::list<Plan> plans; // most recently used first

int base_device(const void *p) {
  const gpu::Ptr q = gpu::classify(p);
  return q.device_accessible ? q.device : -1;
}

template <typename T> bool same(const std::vector<T> &v, const T *a, size_t n) {
  return v.size() == n && (n == 0 || std::memcmp(v.data(), a, n * sizeof(T)) == 0);
}

const Plan &plan_for(const void *sendbuf, const int *scounts, const MPI_Aint *sdispls, const MPI_Datatype *stypes,
                     void *recvbuf, const int *rcounts, const MPI_Aint *rdispls, const MPI_Datatype *rtypes,
                     MPI_Comm comm, const Neighbours &nb) {
  const size_t ni = nb.in.size(), no = nb.out.size();
  const uint64_t gen = type_generation();
  const int sdev = base_device(sendbuf), rdev = base_device(recvbuf);
  for (auto it = plans.begin(); it != plans.end(); ++it) {
    const Plan &p = *it;
    if (p.comm == comm && p.sbuf == sendbuf && p.rbuf == recvbuf && p.typeGen == gen && p.sdev == sdev &&
        p.rdev == rdev && same(p.scounts, scounts, no) && same(p.sdispls, sdispls, no) &&
        same(p.stypes, stypes, no) && same(p.rcounts, rcounts, ni) && same(p.rdispls, rdispls, ni) &&
        same(p.rtypes, rtypes, ni)) {
      plans.splice(plans.begin(), plans, it);
      return plans.front();
    }
  }
  Plan p;
  p.comm = comm;
  p.sbuf = sendbuf;
  p.rbuf = recvbuf;
  p.scounts.assign(scounts, scounts + no);
  p.sdispls.assign(sdispls, sdispls + no);
  p.stypes.assign(stypes, stypes + no);
  p.rcounts.assign(rcounts, rcounts + ni);
  p.rdispls.assign(rdispls, rdispls + ni);
  p.rtypes.assign(rtypes, rtypes + ni);
  p.typeGen = gen;
  p.sdev = sdev;
  p.rdev = rdev;
  p.priv = private_comm(comm);
  next.MPI_Comm_rank(p.priv, &p.me);
  // Self edges: the k-th edge to this rank meets the k-th edge from it (edge
  // order, as message matching would pair them). Each such pair whose blocks
  // are device objects is one strided -> strided copy, with no library
  // messages; the rest go as messages, still in edge order.
  p.doneIn.assign(ni, 0);
  p.doneOut.assign(no, 0);
  std::vector<size_t> selfIn, selfOut;
  for (size_t j = 0; j < ni; ++j)
    if (nb.in[j] == p.me) selfIn.push_back(j);
  for (size_t i = 0; i < no; ++i)
    if (nb.out[i] == p.me) selfOut.push_back(i);
  for (size_t k = 0; k < selfIn.size() && k < selfOut.size(); ++k) {
    const size_t i = selfOut[k], j = selfIn[k];
    if (p2p::plan_local_copy(static_cast<const char *>(sendbuf) + sdispls[i], scounts[i], stypes[i],
                             static_cast<char *>(recvbuf) + rdispls[j], rcounts[j], rtypes[j], &p.copies))
      p.doneOut[i] = p.doneIn[j] = 1;
  }
  plans.push_front(std::move(p));
  if (plans.size() > kMaxPlans) plans.pop_back();
  return plans.front();
}

// one Isend / Irecv per edge through the interposed entry points (device
// blocks -> TEMPI transport, host blocks -> library sends and
// descriptor-aware receives), receives first; self edges between device
// objects as one request of queued copies
int isir(const void *sendbuf, const int *scounts, const MPI_Aint *sdispls, const MPI_Datatype *stypes,
         void *recvbuf, const int *rcounts, const MPI_Aint *rdispls, const MPI_Datatype *rtypes, MPI_Comm comm,
         const Neighbours &nb) {
  const std::vector<int> &in = nb.in, &out = nb.out;
  const uint64_t t0 = tick();
  const Plan &plan = plan_for(sendbuf, scounts, sdispls, stypes, recvbuf, rcounts, rdispls, rtypes, comm, nb);
  const MPI_Comm c = plan.priv;
  const int tag = 0x4E41; // "NA": alone on the private communicator
  const std::vector<char> &doneIn = plan.doneIn, &doneOut = plan.doneOut;
  std::vector<MPI_Request> reqs;
  reqs.reserve(in.size() + out.size() + 1);
  // Receives, then sends (their gathers queue), then the self edges' copies:
  // one start launches the gathers first, so the peers' data leaves before
  // this rank's own copies run (on a GPU shared by several ranks, or a single
  // lane, a stream runs them in that order; profiles/r03/nbr_order_ab_s12.jsonl).
  for (size_t i = 0; i < in.size(); ++i) {
    if (in[i] == MPI_PROC_NULL || doneIn[i]) continue;
    MPI_Request r;
    const int rc = MPI_Irecv(static_cast<char *>(recvbuf) + rdispls[i], rcounts[i], rtypes[i], in[i], tag, c, &r);
    if (rc != MPI_SUCCESS) return rc;
    reqs.push_back(r);
  }
  // (no p2p::CollectiveScope here: the rendezvous would be deadlock-free, but
  // IPC COPY below the eager limit measured 15-20 % slower on the 2-rank
  // neighbourhood halo, tools/gpu_nbr_coll_ab.sh)
  for (size_t i = 0; i < out.size(); ++i) {
    if (out[i] == MPI_PROC_NULL || doneOut[i]) continue;
    MPI_Request r;
    const int rc =
        MPI_Isend(static_cast<const char *>(sendbuf) + sdispls[i], scounts[i], stypes[i], out[i], tag, c, &r);
    if (rc != MPI_SUCCESS) return rc;
    reqs.push_back(r);
  }
  if (!plan.copies.items.empty()) reqs.push_back(p2p::start_local_copies(plan.copies));
  p2p::start_queued();
  tock(counters.ns_nbr_post, t0);
  ScopedNs timer(counters.ns_nbr_wait);
  return MPI_Waitall(int(reqs.size()), reqs.data(), MPI_STATUSES_IGNORE);
}

} // namespace

// a communicator being freed: its handle may come back for another one
void neighbourhood_forget(MPI_Comm comm) {
  neighbourCache.erase(comm);
  for (auto it = plans.begin(); it != plans.end();)
    it = it->comm == comm ? plans.erase(it) : std::next(it);
}

// MPI_Finalize: drop every plan (they hold type records)
void neighbourhood_finalize() {
  plans.clear();
  neighbourCache.clear();
}

} // namespace tempi

using namespace tempi;

TEMPI_EXPORT int MPI_Neighbor_alltoallw(const void *sendbuf, const int sendcounts[], const MPI_Aint sdispls[],
                                        const MPI_Datatype sendtypes[], void *recvbuf, const int recvcounts[],
                                        const MPI_Aint rdispls[], const MPI_Datatype recvtypes[], MPI_Comm comm) {
  TEMPI_MT_ENTRY;
  resolve_next();
  TEMPI_RANGE("MPI_Neighbor_alltoallw");
  auto lib = [&] {
    return TEMPI_UNLOCKED(next.MPI_Neighbor_alltoallw(sendbuf, sendcounts, sdispls, sendtypes, recvbuf, recvcounts,
                                                      rdispls, recvtypes, comm));
  };
  // every rank takes the per-edge route, whatever memory its own blocks are
  // in: its neighbours' device blocks travel on the private duplicate, which
  // the library's own algorithm on `comm` would never match
  const Neighbours *nb = state.active && gpu::available() ? neighbours(comm) : nullptr;
  if (!nb) return lib();
  counters.neighbor_colls++;
  return isir(sendbuf, sendcounts, sdispls, sendtypes, recvbuf, recvcounts, rdispls, recvtypes, comm, *nb);
}

TEMPI_EXPORT int MPI_Neighbor_alltoallv(const void *sendbuf, const int sendcounts[], const int sdispls[],
                                        MPI_Datatype sendtype, void *recvbuf, const int recvcounts[],
                                        const int rdispls[], MPI_Datatype recvtype, MPI_Comm comm) {
  TEMPI_MT_ENTRY;
  resolve_next();
  TEMPI_RANGE("MPI_Neighbor_alltoallv");
  auto lib = [&] {
    return TEMPI_UNLOCKED(next.MPI_Neighbor_alltoallv(sendbuf, sendcounts, sdispls, sendtype, recvbuf, recvcounts,
                                                      rdispls, recvtype, comm));
  };
  const Neighbours *nb = state.active && gpu::available() ? neighbours(comm) : nullptr;
  if (!nb) return lib();
  const std::vector<int> &in = nb->in, &out = nb->out;
  // displacements are in extents of the one type: make the alltoallw form
  MPI_Aint lb, sext, rext;
  MPI_Type_get_extent(sendtype, &lb, &sext);
  MPI_Type_get_extent(recvtype, &lb, &rext);
  std::vector<MPI_Aint> sd(out.size()), rd(in.size());
  for (size_t i = 0; i < out.size(); ++i) sd[i] = MPI_Aint(sdispls[i]) * sext;
  for (size_t i = 0; i < in.size(); ++i) rd[i] = MPI_Aint(rdispls[i]) * rext;
  std::vector<MPI_Datatype> st(out.size(), sendtype), rt(in.size(), recvtype);
  counters.neighbor_colls++; // (every rank takes this route: see MPI_Neighbor_alltoallw)
  return isir(sendbuf, sendcounts, sd.data(), st.data(), recvbuf, recvcounts, rd.data(), rt.data(), comm, *nb);
}

TEMPI_EXPORT int MPI_Dist_graph_create_adjacent(MPI_Comm comm_old, int indegree, const int sources[],
                                                const int sourceweights[], int outdegree, const int destinations[],
                                                const int destweights[], MPI_Info info, int reorder,
                                                MPI_Comm *comm_dist_graph) {
  TEMPI_MT_ENTRY;
  resolve_next();
  TEMPI_RANGE("MPI_Dist_graph_create_adjacent");
  int rc = MPI_SUCCESS;
  if (state.active && placement::create(comm_old, indegree, sources, sourceweights, outdegree, destinations,
                                        destweights, info, reorder, comm_dist_graph, &rc))
    return rc;
  return TEMPI_UNLOCKED(next.MPI_Dist_graph_create_adjacent(comm_old, indegree, sources, sourceweights, outdegree,
                                                            destinations, destweights, info, reorder,
                                                            comm_dist_graph));
}

TEMPI_EXPORT int MPI_Dist_graph_neighbors(MPI_Comm comm, int maxindegree, int sources[], int sourceweights[],
                                          int maxoutdegree, int destinations[], int destweights[]) {
  TEMPI_MT_ENTRY;
  resolve_next();
  return next.MPI_Dist_graph_neighbors(comm, maxindegree, sources, sourceweights, maxoutdegree, destinations,
                                       destweights);
}

TEMPI_EXPORT int MPI_Comm_rank(MPI_Comm comm, int *rank) {
  TEMPI_MT_ENTRY;
  resolve_next();
  return next.MPI_Comm_rank(comm, rank);
}

TEMPI_EXPORT int MPI_Comm_free(MPI_Comm *comm) {
  TEMPI_MT_ENTRY;
  resolve_next();
  if (state.active && comm && *comm != MPI_COMM_NULL) comm_release(*comm);
  return next.MPI_Comm_free(comm);
}
