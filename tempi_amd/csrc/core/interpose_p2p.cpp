// tempi_amd/csrc/core/interpose_p2p.cpp -- interposed point-to-point calls
// (include/tempi_mpi.h): MPI_Send / MPI_Recv / MPI_Isend / MPI_Irecv /
// MPI_Wait as in the reference (/root/reference/src/send.cpp:12-17,
// recv.cpp:19-44, isend.cpp:11-16, irecv.cpp:11-16, wait.cpp:11-16), plus
// what the reference leaves to the library: the rest of the completion
// family, MPI_Sendrecv(_replace), the probe family, the other
// send modes and persistent requests. Device buffers go through tempi::p2p
// (p2p.hpp); host buffers go to the library, except where a receive could
// meet a descriptor; library waits keep TEMPI operations progressing.
#include "trace.hpp"
#include "counters.hpp"
#include "log.hpp"
#include "mt.hpp"
#include "next_mpi.hpp"
#include "p2p.hpp"
#include "gpu.hpp"
#include "state.hpp"

#include "tempi_mpi.h"

#include <vector>

#define TEMPI_EXPORT extern "C" __attribute__((visibility("default")))

using namespace tempi;

TEMPI_EXPORT int MPI_Send(const void *buf, int count, MPI_Datatype datatype, int dest, int tag,
                          MPI_Comm comm) {
  TEMPI_MT_ENTRY;
  resolve_next();
  TEMPI_RANGE("MPI_Send");
  p2p::Route route;
  if (!p2p::handles(buf, count, datatype, dest, &route)) {
    counters.lib_sends++;
    p2p::self_spill(comm, dest);
    if (state.active && p2p::send_gated(comm, dest)) p2p::drain_sends(comm, dest); // keep send order
    return TEMPI_UNLOCKED(next.MPI_Send(buf, count, datatype, dest, tag, comm));
  }
  counters.sends++;
  MPI_Request r;
  int rc = p2p::isend(buf, count, datatype, dest, tag, comm, &r, route, -1, /*blocking=*/true);
  if (rc != MPI_SUCCESS) return rc;
  return p2p::wait(&r, MPI_STATUS_IGNORE);
}

TEMPI_EXPORT int MPI_Recv(void *buf, int count, MPI_Datatype datatype, int source, int tag, MPI_Comm comm,
                          MPI_Status *status) {
  TEMPI_MT_ENTRY;
  resolve_next();
  TEMPI_RANGE("MPI_Recv");
  p2p::Route route;
  if (p2p::handles(buf, count, datatype, source, &route)) {
    counters.recvs++;
    MPI_Request r;
    int rc = p2p::irecv(buf, count, datatype, source, tag, comm, &r, route);
    if (rc != MPI_SUCCESS) return rc;
    return p2p::wait(&r, status);
  }
  bool handled = false;
  const int rc = p2p::recv_host_ipc_aware(buf, count, datatype, source, tag, comm, status, &handled);
  if (handled) return rc;
  counters.lib_recvs++;
  return TEMPI_UNLOCKED(next.MPI_Recv(buf, count, datatype, source, tag, comm, status));
}

TEMPI_EXPORT int MPI_Isend(const void *buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm,
                           MPI_Request *request) {
  TEMPI_MT_ENTRY;
  resolve_next();
  TEMPI_RANGE("MPI_Isend");
  p2p::Route route;
  if (p2p::handles(buf, count, datatype, dest, &route))
    return p2p::isend(buf, count, datatype, dest, tag, comm, request, route);
  if (state.active) {
    p2p::progress(false);
    p2p::self_spill(comm, dest);
    if (p2p::send_gated(comm, dest)) // behind a send still gathering: keep send order
      return p2p::isend_host(buf, count, datatype, dest, tag, comm, request);
  }
  counters.lib_sends++;
  return next.MPI_Isend(buf, count, datatype, dest, tag, comm, request);
}

TEMPI_EXPORT int MPI_Irecv(void *buf, int count, MPI_Datatype datatype, int source, int tag, MPI_Comm comm,
                           MPI_Request *request) {
  TEMPI_MT_ENTRY;
  resolve_next();
  TEMPI_RANGE("MPI_Irecv");
  p2p::Route route;
  if (p2p::handles(buf, count, datatype, source, &route))
    return p2p::irecv(buf, count, datatype, source, tag, comm, request, route);
  if (state.active) p2p::progress(false);
  // a host buffer: a co-located TEMPI device send may arrive as a descriptor
  if (p2p::host_recv_aware(source, tag, comm)) return p2p::irecv_host(buf, count, datatype, source, tag, comm, request);
  p2p::self_spill(comm, source);
  counters.lib_recvs++;
  return next.MPI_Irecv(buf, count, datatype, source, tag, comm, request);
}

TEMPI_EXPORT int MPI_Wait(MPI_Request *request, MPI_Status *status) {
  TEMPI_MT_ENTRY;
  resolve_next();
  TEMPI_RANGE("MPI_Wait");
  if (!state.active) return TEMPI_UNLOCKED(next.MPI_Wait(request, status));
  if (p2p::is_tempi_request(*request)) return p2p::wait(request, status);
  if (!p2p::busy()) return TEMPI_UNLOCKED(next.MPI_Wait(request, status));
  for (;;) { // a library request, while TEMPI operations are in flight
    int flag = 0;
    const int rc = next.MPI_Test(request, &flag, status);
    if (rc != MPI_SUCCESS || flag) return rc;
    p2p::progress();
    mt::yield();
  }
}

TEMPI_EXPORT int MPI_Test(MPI_Request *request, int *flag, MPI_Status *status) {
  TEMPI_MT_ENTRY;
  resolve_next();
  if (!state.active) return next.MPI_Test(request, flag, status);
  if (p2p::is_tempi_request(*request)) return p2p::test(request, flag, status);
  if (p2p::busy()) p2p::progress();
  return next.MPI_Test(request, flag, status);
}

TEMPI_EXPORT int MPI_Waitall(int count, MPI_Request requests[], MPI_Status statuses[]) {
  TEMPI_MT_ENTRY;
  resolve_next();
  TEMPI_RANGE("MPI_Waitall");
  if (!state.active) return TEMPI_UNLOCKED(next.MPI_Waitall(count, requests, statuses));
  bool any = false;
  for (int i = 0; i < count && !any; ++i) any = p2p::is_tempi_request(requests[i]);
  if (!any && !p2p::busy()) return TEMPI_UNLOCKED(next.MPI_Waitall(count, requests, statuses));
  std::vector<char> done(size_t(count), 0);
  int remaining = count;
  int err = MPI_SUCCESS;
  while (remaining) {
    p2p::progress();
    for (int i = 0; i < count; ++i) {
      if (done[size_t(i)]) continue;
      MPI_Status *st = statuses == MPI_STATUSES_IGNORE ? MPI_STATUS_IGNORE : &statuses[i];
      int flag = 0;
      const int rc = p2p::is_tempi_request(requests[i]) ? p2p::test(&requests[i], &flag, st)
                                                        : next.MPI_Test(&requests[i], &flag, st);
      if (rc != MPI_SUCCESS) {
        err = MPI_ERR_IN_STATUS;
        flag = 1;
      }
      if (flag) {
        done[size_t(i)] = 1;
        --remaining;
      }
    }
    if (remaining) mt::yield();
  }
  return err;
}

// ---------------------------------------------------------------------------
// The rest of the completion family. The reference interposes none of these
// (SURVEY F8), so a TEMPI request handed to them would reach the library;
// here they understand TEMPI requests and keep TEMPI operations moving.

namespace {

bool any_tempi(int count, const MPI_Request *requests) {
  for (int i = 0; i < count; ++i)
    if (p2p::is_tempi_request(requests[i])) return true;
  return false;
}

// one request, non-blocking: 1 = completed (request released, status set)
int test_one(MPI_Request *r, MPI_Status *st, int *err) {
  int flag = 0;
  const int rc = p2p::is_tempi_request(*r) ? p2p::test(r, &flag, st) : next.MPI_Test(r, &flag, st);
  if (rc != MPI_SUCCESS) {
    *err = rc;
    return 1;
  }
  return flag;
}

MPI_Status *at(MPI_Status *statuses, int i) {
  return statuses == MPI_STATUSES_IGNORE ? MPI_STATUS_IGNORE : &statuses[i];
}

} // namespace

TEMPI_EXPORT int MPI_Testall(int count, MPI_Request requests[], int *flag, MPI_Status statuses[]) {
  TEMPI_MT_ENTRY;
  resolve_next();
  if (!state.active || (!any_tempi(count, requests) && !p2p::busy()))
    return next.MPI_Testall(count, requests, flag, statuses);
  p2p::progress();
  // all or nothing: look first, complete only when every request is done
  for (int i = 0; i < count; ++i) {
    if (requests[i] == MPI_REQUEST_NULL) continue;
    int done = 0;
    if (p2p::is_tempi_request(requests[i]))
      done = p2p::peek(requests[i]);
    else
      next.MPI_Request_get_status(requests[i], &done, MPI_STATUS_IGNORE);
    if (!done) {
      *flag = 0;
      return MPI_SUCCESS;
    }
  }
  int err = MPI_SUCCESS;
  for (int i = 0; i < count; ++i) {
    if (requests[i] == MPI_REQUEST_NULL) continue;
    int e = MPI_SUCCESS;
    test_one(&requests[i], at(statuses, i), &e);
    if (e != MPI_SUCCESS) err = MPI_ERR_IN_STATUS;
  }
  *flag = 1;
  return err;
}

TEMPI_EXPORT int MPI_Testany(int count, MPI_Request requests[], int *index, int *flag, MPI_Status *status) {
  TEMPI_MT_ENTRY;
  resolve_next();
  if (!state.active || (!any_tempi(count, requests) && !p2p::busy()))
    return next.MPI_Testany(count, requests, index, flag, status);
  p2p::progress();
  bool anyActive = false;
  for (int i = 0; i < count; ++i) {
    if (requests[i] == MPI_REQUEST_NULL || p2p::inactive(requests[i])) continue;
    anyActive = true;
    int err = MPI_SUCCESS;
    if (test_one(&requests[i], status, &err)) {
      *index = i;
      *flag = 1;
      return err;
    }
  }
  *index = MPI_UNDEFINED;
  *flag = anyActive ? 0 : 1;
  if (!anyActive && status != MPI_STATUS_IGNORE) { // every request null or inactive: an empty status
    status->MPI_SOURCE = MPI_ANY_SOURCE;
    status->MPI_TAG = MPI_ANY_TAG;
    status->MPI_ERROR = MPI_SUCCESS;
    MPI_Status_set_elements(status, MPI_BYTE, 0);
    MPI_Status_set_cancelled(status, 0);
  }
  return MPI_SUCCESS;
}

TEMPI_EXPORT int MPI_Waitany(int count, MPI_Request requests[], int *index, MPI_Status *status) {
  TEMPI_MT_ENTRY;
  resolve_next();
  if (!state.active || (!any_tempi(count, requests) && !p2p::busy()))
    return TEMPI_UNLOCKED(next.MPI_Waitany(count, requests, index, status));
  for (;;) {
    int flag = 0;
    const int rc = MPI_Testany(count, requests, index, &flag, status);
    if (rc != MPI_SUCCESS || flag) return rc;
    mt::yield();
  }
}

TEMPI_EXPORT int MPI_Testsome(int incount, MPI_Request requests[], int *outcount, int indices[],
                              MPI_Status statuses[]) {
  TEMPI_MT_ENTRY;
  resolve_next();
  if (!state.active || (!any_tempi(incount, requests) && !p2p::busy()))
    return next.MPI_Testsome(incount, requests, outcount, indices, statuses);
  p2p::progress();
  bool anyActive = false;
  int n = 0, err = MPI_SUCCESS;
  for (int i = 0; i < incount; ++i) {
    if (requests[i] == MPI_REQUEST_NULL || p2p::inactive(requests[i])) continue;
    anyActive = true;
    int e = MPI_SUCCESS;
    if (test_one(&requests[i], at(statuses, n), &e)) {
      if (e != MPI_SUCCESS) err = MPI_ERR_IN_STATUS;
      indices[n++] = i;
    }
  }
  *outcount = anyActive ? n : MPI_UNDEFINED;
  return err;
}

TEMPI_EXPORT int MPI_Waitsome(int incount, MPI_Request requests[], int *outcount, int indices[],
                              MPI_Status statuses[]) {
  TEMPI_MT_ENTRY;
  resolve_next();
  if (!state.active || (!any_tempi(incount, requests) && !p2p::busy()))
    return TEMPI_UNLOCKED(next.MPI_Waitsome(incount, requests, outcount, indices, statuses));
  for (;;) {
    const int rc = MPI_Testsome(incount, requests, outcount, indices, statuses);
    if (rc != MPI_SUCCESS || *outcount != 0) return rc;
    mt::yield();
  }
}

TEMPI_EXPORT int MPI_Request_free(MPI_Request *request) {
  TEMPI_MT_ENTRY;
  resolve_next();
  if (state.active && p2p::is_tempi_request(*request)) {
    p2p::release(request);
    return MPI_SUCCESS;
  }
  return next.MPI_Request_free(request);
}

// MPI_Request_get_status and MPI_Cancel: not interposed by the reference (F8)
TEMPI_EXPORT int MPI_Request_get_status(MPI_Request request, int *flag, MPI_Status *status) {
  TEMPI_MT_ENTRY;
  resolve_next();
  if (state.active && p2p::is_tempi_request(request)) return p2p::get_status(request, flag, status);
  if (state.active && p2p::busy()) p2p::progress();
  return next.MPI_Request_get_status(request, flag, status);
}

TEMPI_EXPORT int MPI_Cancel(MPI_Request *request) {
  TEMPI_MT_ENTRY;
  resolve_next();
  if (state.active && p2p::is_tempi_request(*request)) return p2p::cancel(*request);
  return next.MPI_Cancel(request);
}

// MPI_Sendrecv: not interposed by the reference, so a device-buffer exchange
// would reach a library that cannot read GPU memory. When either side is a
// TEMPI object it is an MPI_Irecv + MPI_Isend through the interposed entry
// points and two waits (receive first, so a message to this same rank
// matches at once).
TEMPI_EXPORT int MPI_Sendrecv(const void *sendbuf, int sendcount, MPI_Datatype sendtype, int dest, int sendtag,
                              void *recvbuf, int recvcount, MPI_Datatype recvtype, int source, int recvtag,
                              MPI_Comm comm, MPI_Status *status) {
  TEMPI_MT_ENTRY;
  resolve_next();
  TEMPI_RANGE("MPI_Sendrecv");
  p2p::Route sr, rr;
  // TEMPI's when either side is a device object, or when the host receive
  // could meet a descriptor
  const bool mine = state.active && (p2p::handles(sendbuf, sendcount, sendtype, dest, &sr) ||
                                     p2p::handles(recvbuf, recvcount, recvtype, source, &rr) ||
                                     p2p::host_recv_aware(source, recvtag, comm));
  if (!mine) {
    p2p::self_spill(comm, dest);
    p2p::self_spill(comm, source);
    if (state.active && p2p::send_gated(comm, dest)) p2p::drain_sends(comm, dest); // keep send order
    return TEMPI_UNLOCKED(next.MPI_Sendrecv(sendbuf, sendcount, sendtype, dest, sendtag, recvbuf, recvcount,
                                            recvtype, source, recvtag, comm, status));
  }
  MPI_Request r = MPI_REQUEST_NULL, s = MPI_REQUEST_NULL;
  int rc = MPI_Irecv(recvbuf, recvcount, recvtype, source, recvtag, comm, &r);
  if (rc != MPI_SUCCESS) return rc;
  rc = MPI_Isend(sendbuf, sendcount, sendtype, dest, sendtag, comm, &s);
  if (rc != MPI_SUCCESS) return rc;
  rc = MPI_Wait(&r, status);
  const int rc2 = MPI_Wait(&s, MPI_STATUS_IGNORE);
  return rc != MPI_SUCCESS ? rc : rc2;
}

// The probe family and matched receives: not interposed by the reference,
// whose senders always send the packed bytes. Here a co-located device send
// may travel as a descriptor, so a probe reports the payload's size and a
// matched receive lands the payload (p2p.hpp).
TEMPI_EXPORT int MPI_Probe(int source, int tag, MPI_Comm comm, MPI_Status *status) {
  TEMPI_MT_ENTRY;
  resolve_next();
  TEMPI_RANGE("MPI_Probe");
  return p2p::probe(source, tag, comm, nullptr, status);
}

TEMPI_EXPORT int MPI_Iprobe(int source, int tag, MPI_Comm comm, int *flag, MPI_Status *status) {
  TEMPI_MT_ENTRY;
  resolve_next();
  return p2p::probe(source, tag, comm, flag, status);
}

TEMPI_EXPORT int MPI_Mprobe(int source, int tag, MPI_Comm comm, MPI_Message *message, MPI_Status *status) {
  TEMPI_MT_ENTRY;
  resolve_next();
  TEMPI_RANGE("MPI_Mprobe");
  return p2p::mprobe(source, tag, comm, nullptr, message, status);
}

TEMPI_EXPORT int MPI_Improbe(int source, int tag, MPI_Comm comm, int *flag, MPI_Message *message,
                             MPI_Status *status) {
  TEMPI_MT_ENTRY;
  resolve_next();
  return p2p::mprobe(source, tag, comm, flag, message, status);
}

TEMPI_EXPORT int MPI_Mrecv(void *buf, int count, MPI_Datatype datatype, MPI_Message *message, MPI_Status *status) {
  TEMPI_MT_ENTRY;
  resolve_next();
  TEMPI_RANGE("MPI_Mrecv");
  if (!state.active) return TEMPI_UNLOCKED(next.MPI_Mrecv(buf, count, datatype, message, status));
  return p2p::mrecv(buf, count, datatype, message, status);
}

TEMPI_EXPORT int MPI_Imrecv(void *buf, int count, MPI_Datatype datatype, MPI_Message *message,
                            MPI_Request *request) {
  TEMPI_MT_ENTRY;
  resolve_next();
  if (!state.active) return next.MPI_Imrecv(buf, count, datatype, message, request);
  return p2p::imrecv(buf, count, datatype, message, request);
}

// The send modes: the reference interposes only standard sends, so a
// device-buffer MPI_Ssend / MPI_Bsend / MPI_Rsend (and their I-forms) would
// reach a library that cannot read GPU memory. Here they take the TEMPI path
// with the matching library call (p2p.hpp: SendMode); host buffers keep the
// library's call, after the self channel spills and gated sends drain, as for
// MPI_Send.
namespace {
int mode_send(const void *buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm,
              MPI_Request *request, p2p::SendMode mode) {
  resolve_next();
  p2p::Route route;
  if (p2p::handles(buf, count, datatype, dest, &route)) {
    counters.sends++;
    MPI_Request r;
    const bool blocking = request == nullptr;
    const int rc = p2p::isend(buf, count, datatype, dest, tag, comm, request ? request : &r, route, -1, blocking,
                              mode);
    if (rc != MPI_SUCCESS || !blocking) return rc;
    return p2p::wait(&r, MPI_STATUS_IGNORE);
  }
  counters.lib_sends++;
  if (state.active) {
    if (request) p2p::progress(false);
    p2p::self_spill(comm, dest);
    if (p2p::send_gated(comm, dest)) p2p::drain_sends(comm, dest); // keep send order
  }
  using M = p2p::SendMode;
  if (request) {
    if (mode == M::SYNC) return next.MPI_Issend(buf, count, datatype, dest, tag, comm, request);
    if (mode == M::BUFFERED) return next.MPI_Ibsend(buf, count, datatype, dest, tag, comm, request);
    return next.MPI_Irsend(buf, count, datatype, dest, tag, comm, request);
  }
  if (mode == M::SYNC) return TEMPI_UNLOCKED(next.MPI_Ssend(buf, count, datatype, dest, tag, comm));
  if (mode == M::BUFFERED) return TEMPI_UNLOCKED(next.MPI_Bsend(buf, count, datatype, dest, tag, comm));
  return TEMPI_UNLOCKED(next.MPI_Rsend(buf, count, datatype, dest, tag, comm));
}
} // namespace

TEMPI_EXPORT int MPI_Ssend(const void *buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm) {
  TEMPI_MT_ENTRY;
  TEMPI_RANGE("MPI_Ssend");
  return mode_send(buf, count, datatype, dest, tag, comm, nullptr, p2p::SendMode::SYNC);
}
TEMPI_EXPORT int MPI_Bsend(const void *buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm) {
  TEMPI_MT_ENTRY;
  TEMPI_RANGE("MPI_Bsend");
  return mode_send(buf, count, datatype, dest, tag, comm, nullptr, p2p::SendMode::BUFFERED);
}
TEMPI_EXPORT int MPI_Rsend(const void *buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm) {
  TEMPI_MT_ENTRY;
  TEMPI_RANGE("MPI_Rsend");
  return mode_send(buf, count, datatype, dest, tag, comm, nullptr, p2p::SendMode::READY);
}
TEMPI_EXPORT int MPI_Issend(const void *buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm,
                            MPI_Request *request) {
  TEMPI_MT_ENTRY;
  return mode_send(buf, count, datatype, dest, tag, comm, request, p2p::SendMode::SYNC);
}
TEMPI_EXPORT int MPI_Ibsend(const void *buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm,
                            MPI_Request *request) {
  TEMPI_MT_ENTRY;
  return mode_send(buf, count, datatype, dest, tag, comm, request, p2p::SendMode::BUFFERED);
}
TEMPI_EXPORT int MPI_Irsend(const void *buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm,
                            MPI_Request *request) {
  TEMPI_MT_ENTRY;
  return mode_send(buf, count, datatype, dest, tag, comm, request, p2p::SendMode::READY);
}

// MPI_Buffer_detach waits until every buffered-mode message has been handed
// to the library: a device object's MPI_Ibsend reaches it only after its
// gather has run, and the attached buffer must still be there then (the
// library's own detach then waits for the library's copies to drain).
TEMPI_EXPORT int MPI_Buffer_detach(void *buffer_addr, int *size) {
  TEMPI_MT_ENTRY;
  resolve_next();
  if (state.active) p2p::drain_buffered();
  return TEMPI_UNLOCKED(next.MPI_Buffer_detach(buffer_addr, size));
}

// Persistent requests: TEMPI's while it is active beside a GPU (p2p.hpp:
// persistent_init; MPI_Start posts through the interposed non-blocking calls,
// so device objects take the transport and host buffers keep send order and
// see descriptors), the library's otherwise. Not interposed by the reference.
namespace {
int persistent_init(bool send, const void *buf, int count, MPI_Datatype datatype, int peer, int tag, MPI_Comm comm,
                    MPI_Request *request, p2p::SendMode mode) {
  if (state.active && gpu::available())
    return p2p::persistent_init(send, buf, count, datatype, peer, tag, comm, mode, request);
  if (state.active) p2p::self_spill(comm, peer);
  using M = p2p::SendMode;
  if (!send) return next.MPI_Recv_init(const_cast<void *>(buf), count, datatype, peer, tag, comm, request);
  if (mode == M::SYNC) return next.MPI_Ssend_init(buf, count, datatype, peer, tag, comm, request);
  if (mode == M::BUFFERED) return next.MPI_Bsend_init(buf, count, datatype, peer, tag, comm, request);
  if (mode == M::READY) return next.MPI_Rsend_init(buf, count, datatype, peer, tag, comm, request);
  return next.MPI_Send_init(buf, count, datatype, peer, tag, comm, request);
}
} // namespace

TEMPI_EXPORT int MPI_Send_init(const void *buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm,
                               MPI_Request *request) {
  TEMPI_MT_ENTRY;
  resolve_next();
  return persistent_init(true, buf, count, datatype, dest, tag, comm, request, p2p::SendMode::STANDARD);
}
TEMPI_EXPORT int MPI_Ssend_init(const void *buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm,
                                MPI_Request *request) {
  TEMPI_MT_ENTRY;
  resolve_next();
  return persistent_init(true, buf, count, datatype, dest, tag, comm, request, p2p::SendMode::SYNC);
}
TEMPI_EXPORT int MPI_Bsend_init(const void *buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm,
                                MPI_Request *request) {
  TEMPI_MT_ENTRY;
  resolve_next();
  return persistent_init(true, buf, count, datatype, dest, tag, comm, request, p2p::SendMode::BUFFERED);
}
TEMPI_EXPORT int MPI_Rsend_init(const void *buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm,
                                MPI_Request *request) {
  TEMPI_MT_ENTRY;
  resolve_next();
  return persistent_init(true, buf, count, datatype, dest, tag, comm, request, p2p::SendMode::READY);
}
TEMPI_EXPORT int MPI_Recv_init(void *buf, int count, MPI_Datatype datatype, int source, int tag, MPI_Comm comm,
                               MPI_Request *request) {
  TEMPI_MT_ENTRY;
  resolve_next();
  if (state.active && !gpu::available() && p2p::holds(source, tag, comm))
    LOG_WARN("MPI_Recv_init: a message it matches is held by an earlier MPI_Probe; the library's persistent "
             "receive will not see it");
  return persistent_init(false, buf, count, datatype, source, tag, comm, request, p2p::SendMode::STANDARD);
}

TEMPI_EXPORT int MPI_Start(MPI_Request *request) {
  TEMPI_MT_ENTRY;
  resolve_next();
  if (state.active && p2p::is_tempi_request(*request)) return p2p::start(request);
  return next.MPI_Start(request);
}

TEMPI_EXPORT int MPI_Startall(int count, MPI_Request requests[]) {
  TEMPI_MT_ENTRY;
  resolve_next();
  if (!state.active || !any_tempi(count, requests)) return next.MPI_Startall(count, requests);
  int err = MPI_SUCCESS;
  for (int i = 0; i < count; ++i) { // (a burst of starts shares the transport's launches)
    const int rc = MPI_Start(&requests[i]);
    if (rc != MPI_SUCCESS && err == MPI_SUCCESS) err = rc;
  }
  return err;
}

#define TEMPI_SPILL_THEN(peer, call)                                                               \
  resolve_next();                                                                                  \
  if (state.active) p2p::self_spill(comm, peer);                                                   \
  return call;

// MPI_Sendrecv_replace: when the receive is TEMPI's (a device object, or a
// host buffer a descriptor or a held message may reach: p2p::host_recv_aware)
// the outgoing element is packed into a host buffer first and the exchange
// is MPI_Sendrecv through the interposed entry point (MPI_PACKED matches any
// receive type); otherwise the library's.
TEMPI_EXPORT int MPI_Sendrecv_replace(void *buf, int count, MPI_Datatype datatype, int dest, int sendtag, int source,
                                      int recvtag, MPI_Comm comm, MPI_Status *status) {
  TEMPI_MT_ENTRY;
  resolve_next();
  p2p::Route rr;
  if (state.active && count > 0 &&
      (p2p::handles(buf, count, datatype, source, &rr) || p2p::handles(buf, count, datatype, dest, &rr) ||
       p2p::host_recv_aware(source, recvtag, comm))) {
    int size = 0, pos = 0;
    MPI_Pack_size(count, datatype, comm, &size);
    std::vector<char> tmp(size_t(size > 0 ? size : 1));
    int rc = tempi::pack(buf, count, datatype, tmp.data(), size, &pos, comm); // (device objects too)
    if (rc != MPI_SUCCESS) return rc;
    return MPI_Sendrecv(tmp.data(), pos, MPI_PACKED, dest, sendtag, buf, count, datatype, source, recvtag, comm,
                        status);
  }
  if (state.active) p2p::self_spill(comm, source);
  TEMPI_SPILL_THEN(dest, TEMPI_UNLOCKED(next.MPI_Sendrecv_replace(buf, count, datatype, dest, sendtag, source,
                                                                   recvtag, comm, status)))
}
#undef TEMPI_SPILL_THEN
