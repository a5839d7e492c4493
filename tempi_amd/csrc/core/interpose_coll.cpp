// tempi_amd/csrc/core/interpose_coll.cpp -- interposed MPI_Alltoallv for
// device buffers (config 5).
//
// Reference: /root/reference/src/alltoallv.cpp:14-68 dispatching to
// /root/reference/src/internal/alltoallv_impl.cpp:21-258 (host-staged library
// alltoallv; Isend/Irecv remote-first; host-staged Isend/Irecv; remote-staged
// / local-direct), restricted there to MPI_COMM_WORLD and byte counts, with
// buffer sizes computed as sdispls[last] + counts[last].
// Here: any intra-communicator and any datatype TEMPI knows (predefined or
// committed, strided or not), sizes from the true extent of every block.
//   AUTO / REMOTE_FIRST  per-peer MPI_Isend / MPI_Irecv through tempi::p2p,
//                        remote peers first then ranks in ring order: device
//                        to device over IPC (xGMI) between co-located ranks,
//                        ONESHOT (pinned host) otherwise
//   STAGED               device -> pinned host copy of the touched spans,
//                        library MPI_Alltoallv on host memory, copy back
//   ISIR_STAGED          per-peer Isend / Irecv, every transfer host-staged
//   ISIR_REMOTE_STAGED   IPC for co-located peers, STAGED for the others
// Messages travel on a private duplicate of the communicator, so they never
// match the application's own point-to-point traffic.
#include "trace.hpp"
#include "alloc.hpp"
#include "counters.hpp"
#include "env.hpp"
#include "gpu.hpp"
#include "log.hpp"
#include "mt.hpp"
#include "next_mpi.hpp"
#include "p2p.hpp"
#include "state.hpp"
#include "topology.hpp"
#include "type_cache.hpp"

#include "tempi_mpi.h"

#include <algorithm>
#include <map>
#include <vector>

#define TEMPI_EXPORT extern "C" __attribute__((visibility("default")))

namespace tempi {
namespace {

// [lo, hi) bytes from buf touched by blocks (counts[i] elements of t at
// displs[i] * extent)
bool span(const int *counts, const int *displs, int n, MPI_Datatype t, int64_t *lo, int64_t *hi) {
  MPI_Aint lb, ext, tlb, text;
  MPI_Type_get_extent(t, &lb, &ext);
  MPI_Type_get_true_extent(t, &tlb, &text);
  bool any = false;
  *lo = 0;
  *hi = 0;
  for (int i = 0; i < n; ++i) {
    if (counts[i] <= 0) continue;
    const int64_t b0 = int64_t(displs[i]) * ext;
    int64_t a = b0 + tlb, b = b0 + tlb + text;
    const int64_t d = int64_t(counts[i] - 1) * ext;
    if (d < 0) a += d; else b += d;
    if (!any || a < *lo) *lo = a;
    if (!any || b > *hi) *hi = b;
    any = true;
  }
  return any;
}

int staged(const void *sendbuf, const int *scounts, const int *sdispls, MPI_Datatype stype, void *recvbuf,
           const int *rcounts, const int *rdispls, MPI_Datatype rtype, MPI_Comm comm, int n) {
  int64_t slo, shi, rlo, rhi;
  const bool s = span(scounts, sdispls, n, stype, &slo, &shi);
  const bool r = span(rcounts, rdispls, n, rtype, &rlo, &rhi);
  Slab *hs = s ? pinned_pool().get(size_t(shi - slo), 0) : nullptr;
  Slab *hr = r ? pinned_pool().get(size_t(rhi - rlo), 0) : nullptr;
  if (s) gpu::check(tempi_hip_memcpy(hs->host, static_cast<const char *>(sendbuf) + slo, size_t(shi - slo)), "a2av D2H");
  if (r) gpu::check(tempi_hip_memcpy(hr->host, static_cast<char *>(recvbuf) + rlo, size_t(rhi - rlo)), "a2av D2H");
  const char *hsend = s ? static_cast<const char *>(hs->host) - slo : nullptr;
  char *hrecv = r ? static_cast<char *>(hr->host) - rlo : nullptr;
  const int rc =
      TEMPI_UNLOCKED(next.MPI_Alltoallv(hsend, scounts, sdispls, stype, hrecv, rcounts, rdispls, rtype, comm));
  if (r) gpu::check(tempi_hip_memcpy(static_cast<char *>(recvbuf) + rlo, hr->host, size_t(rhi - rlo)), "a2av H2D");
  if (hs) pinned_pool().put(hs);
  if (hr) pinned_pool().put(hr);
  return rc;
}

int isir(const void *sendbuf, const int *scounts, const int *sdispls, MPI_Datatype stype, void *recvbuf,
         const int *rcounts, const int *rdispls, MPI_Datatype rtype, MPI_Comm comm, int n, int rank, int local,
         int remote) {
  MPI_Aint lb, sext, rext;
  MPI_Type_get_extent(stype, &lb, &sext);
  MPI_Type_get_extent(rtype, &lb, &rext);
  // remote peers first (their transfers are the long pole), then ring order
  std::vector<int> order;
  for (int pass = 0; pass < 2; ++pass)
    for (int k = 1; k <= n; ++k) {
      const int p = (rank + k) % n;
      const bool co = topology::colocated(comm, p);
      if ((pass == 0) == !co) order.push_back(p);
    }
  const int tag = 0x3A2A;
  std::vector<MPI_Request> reqs;
  p2p::CollectiveScope scope; // every receive is posted before any wait
  // this rank's own block: one queued copy when both sides are device
  // objects (no library messages), else a message like the others
  bool selfDone = false;
  if (scounts[rank] > 0 && rcounts[rank] > 0) {
    MPI_Request r;
    if (p2p::local_copy(static_cast<const char *>(sendbuf) + int64_t(sdispls[rank]) * sext, scounts[rank], stype,
                        static_cast<char *>(recvbuf) + int64_t(rdispls[rank]) * rext, rcounts[rank], rtype, &r)) {
      reqs.push_back(r);
      selfDone = true;
      p2p::start_queued();
    }
  }
  for (int p : order)
    if (rcounts[p] > 0 && !(selfDone && p == rank)) {
      MPI_Request r;
      char *b = static_cast<char *>(recvbuf) + int64_t(rdispls[p]) * rext;
      p2p::Route route;
      if (p2p::handles(b, rcounts[p], rtype, p, &route))
        p2p::irecv(b, rcounts[p], rtype, p, tag, comm, &r, route);
      else if (p2p::host_recv_aware(p, tag, comm)) // a host block a peer's device send may reach as a descriptor
        p2p::irecv_host(b, rcounts[p], rtype, p, tag, comm, &r);
      else {
        p2p::self_spill(comm, p); // (a library receive from this rank: TEMPI's self channel hands over first)
        next.MPI_Irecv(b, rcounts[p], rtype, p, tag, comm, &r);
      }
      reqs.push_back(r);
    }
  for (int p : order)
    if (scounts[p] > 0 && !(selfDone && p == rank)) {
      MPI_Request r;
      const char *b = static_cast<const char *>(sendbuf) + int64_t(sdispls[p]) * sext;
      const int force = topology::colocated(comm, p) ? local : remote;
      p2p::Route route;
      if (p2p::handles(b, scounts[p], stype, p, &route))
        p2p::isend(b, scounts[p], stype, p, tag, comm, &r, route, force);
      else {
        p2p::self_spill(comm, p);
        next.MPI_Isend(b, scounts[p], stype, p, tag, comm, &r);
      }
      reqs.push_back(r);
    }
  int err = MPI_SUCCESS;
  for (MPI_Request &r : reqs) {
    const int rc = p2p::is_tempi_request(r) ? p2p::wait(&r, MPI_STATUS_IGNORE) : [&] {
      for (;;) {
        int flag = 0;
        const int e = next.MPI_Test(&r, &flag, MPI_STATUS_IGNORE);
        if (e != MPI_SUCCESS || flag) return e;
        p2p::progress();
        mt::yield();
      }
    }();
    if (rc != MPI_SUCCESS) err = rc;
  }
  return err;
}

// private duplicates of application communicators, one per communicator,
// made on first use and freed with it (MPI_Comm_free below) -- the
// reference instead reserves tags on the application's communicator
// (/root/reference/src/internal/tags.cpp)
std::map<MPI_Comm, MPI_Comm> privateComms;

} // namespace

MPI_Comm private_comm(MPI_Comm comm) {
  auto it = privateComms.find(comm);
  if (it != privateComms.end()) return it->second;
  MPI_Comm d;
  MPI_Comm_dup(comm, &d);
  privateComms[comm] = d;
  return d;
}

void coll_init() { private_comm(MPI_COMM_WORLD); }
void neighbourhood_finalize(); // interpose_neighbor.cpp
void coll_finalize() {
  neighbourhood_finalize();
  for (auto &kv : privateComms) next.MPI_Comm_free(&kv.second);
  privateComms.clear();
}

// the application frees `comm`: drop what TEMPI cached for the handle
void neighbourhood_forget(MPI_Comm comm); // interpose_neighbor.cpp

void comm_release(MPI_Comm comm) {
  p2p::self_forget(comm);
  neighbourhood_forget(comm);
  topology::uncache(comm);
  auto it = privateComms.find(comm);
  if (it != privateComms.end()) {
    next.MPI_Comm_free(&it->second);
    privateComms.erase(it);
  }
}

} // namespace tempi

using namespace tempi;

TEMPI_EXPORT int MPI_Alltoallv(const void *sendbuf, const int sendcounts[], const int sdispls[],
                               MPI_Datatype sendtype, void *recvbuf, const int recvcounts[], const int rdispls[],
                               MPI_Datatype recvtype, MPI_Comm comm) {
  TEMPI_MT_ENTRY;
  resolve_next();
  TEMPI_RANGE("MPI_Alltoallv");
  auto lib = [&] {
    return TEMPI_UNLOCKED(next.MPI_Alltoallv(sendbuf, sendcounts, sdispls, sendtype, recvbuf, recvcounts, rdispls,
                                             recvtype, comm));
  };
  if (!state.active || env.alltoallv == AlltoallvMethod::NONE || !gpu::available() || sendbuf == MPI_IN_PLACE)
    return lib();
  int inter = 0;
  MPI_Comm_test_inter(comm, &inter);
  if (inter) return lib();
  int n = 0, rank = 0;
  MPI_Comm_size(comm, &n);
  MPI_Comm_rank(comm, &rank);
  // Every rank takes TEMPI's route, whatever memory its own blocks are in:
  // a rank whose buffers are all on the host still exchanges with ranks
  // whose buffers are not, so the choice must be the same everywhere (the
  // library's alltoallv on `comm` cannot match TEMPI's messages on the
  // private duplicate). Only conditions every rank shares lead to the library.
  if (!type_lookup(sendtype) || !type_lookup(recvtype)) return lib(); // uncommitted: let MPI complain
  const MPI_Comm c = private_comm(comm);
  int rc;
  switch (env.alltoallv) {
  case AlltoallvMethod::STAGED:
    rc = staged(sendbuf, sendcounts, sdispls, sendtype, recvbuf, recvcounts, rdispls, recvtype, c, n);
    break;
  case AlltoallvMethod::ISIR_STAGED:
    rc = isir(sendbuf, sendcounts, sdispls, sendtype, recvbuf, recvcounts, rdispls, recvtype, c, n, rank, 1, 1);
    break;
  case AlltoallvMethod::ISIR_REMOTE_STAGED:
    rc = isir(sendbuf, sendcounts, sdispls, sendtype, recvbuf, recvcounts, rdispls, recvtype, c, n, rank, 3, 1);
    break;
  case AlltoallvMethod::AUTO:
  case AlltoallvMethod::REMOTE_FIRST:
  default:
    rc = isir(sendbuf, sendcounts, sdispls, sendtype, recvbuf, recvcounts, rdispls, recvtype, c, n, rank, -1, -1);
    break;
  }
  return rc;
}

// MPI_Barrier: not interposed by the reference. A rank blocked in the
// library's barrier makes no TEMPI progress, and a peer may be waiting on it:
// for the bytes of an IPC message it could not map (the NACK re-send), for an
// ack that frees a slab. While TEMPI has operations in flight the barrier is
// an MPI_Ibarrier completed under TEMPI's progress loop -- on every rank
// whenever TEMPI is active, since a blocking and a non-blocking barrier do
// not match each other (whether a rank is busy is its own business).
TEMPI_EXPORT int MPI_Barrier(MPI_Comm comm) {
  TEMPI_MT_ENTRY;
  resolve_next();
  TEMPI_RANGE("MPI_Barrier");
  if (!state.active) return TEMPI_UNLOCKED(next.MPI_Barrier(comm));
  MPI_Request r = MPI_REQUEST_NULL;
  int rc = MPI_Ibarrier(comm, &r);
  if (rc != MPI_SUCCESS) return rc;
  for (;;) {
    int flag = 0;
    rc = next.MPI_Test(&r, &flag, MPI_STATUS_IGNORE);
    if (rc != MPI_SUCCESS || flag) return rc;
    if (p2p::busy()) p2p::progress();
    mt::yield();
  }
}
