// tempi_amd/csrc/core/p2p_probe.cpp -- the probe family, held messages and
// host receives that may meet a descriptor (p2p.hpp, p2p_internal.hpp)
#include "p2p_internal.hpp"

#include "alloc.hpp"
#include "counters.hpp"
#include "env.hpp"
#include "gpu.hpp"
#include "log.hpp"
#include "mt.hpp"
#include "next_mpi.hpp"
#include "packer.hpp"
#include "perf_model.hpp"
#include "state.hpp"
#include "topology.hpp"
#include "trace.hpp"
#include "type_cache.hpp"

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <unistd.h>

namespace tempi {
namespace p2p {
namespace detail {
namespace {
std::deque<std::unique_ptr<Probed>> probed;
std::unordered_map<uint32_t, std::unique_ptr<Probed>> probedMsgs; // MPI_Mprobe handles
// the communicator of each library message an MPI_Mprobe / MPI_Improbe here
// returned: a matched receive of it raises errors on that communicator's
// error handler
std::unordered_map<MPI_Message, MPI_Comm> libMsgComm;
uint32_t nextMsgHandle = 1;

bool probed_matches(const Probed &p, int source, int tag, MPI_Comm comm) {
  return p.comm == comm && (source == MPI_ANY_SOURCE || source == p.st.MPI_SOURCE) &&
         (tag == MPI_ANY_TAG || tag == p.st.MPI_TAG);
}
} // namespace

// the earliest kept message a receive (source, tag, comm) matches, taken out
std::unique_ptr<Probed> take_probed(int source, int tag, MPI_Comm comm) {
  if (probed.empty()) return nullptr;
  for (auto it = probed.begin(); it != probed.end(); ++it)
    if (probed_matches(**it, source, tag, comm)) {
      std::unique_ptr<Probed> p = std::move(*it);
      probed.erase(it);
      return p;
    }
  return nullptr;
}

} // namespace detail

using namespace detail;

int recv_host_ipc_aware(void *buf, int count, MPI_Datatype dt, int source, int tag, MPI_Comm comm,
                        MPI_Status *status, bool *handled) {
  *handled = false;
  if (!state.active || !gpu::available() || source == MPI_PROC_NULL) return MPI_SUCCESS;
  self_spill(comm, source);
  *handled = true;
  auto land = [&](const char *msg, int n, MPI_Status st) {
    int64_t got = 0;
    const int e = land_host(msg, n, buf, count, dt, comm, &got);
    if (status != MPI_STATUS_IGNORE) {
      *status = st;
      status->MPI_ERROR = e;
      set_received(status, got);
    }
    return e == MPI_SUCCESS ? MPI_SUCCESS : raise_error(comm, e);
  };
  if (std::unique_ptr<Probed> p = take_probed(source, tag, comm)) // a probe already received it
    return land(p->bytes.data(), int(p->bytes.size()), p->st);
  MPI_Message msg;
  MPI_Status st;
  // keep TEMPI operations moving while we wait for the message
  for (;;) {
    int flag = 0;
    const int rc = next.MPI_Improbe(source, tag, comm, &flag, &msg, &st);
    if (rc != MPI_SUCCESS) return rc;
    if (flag) break;
    progress();
    mt::yield();
    // at MPI_THREAD_MULTIPLE another thread's probe may have taken this
    // message (with the source's earlier ones) out of the library while the
    // lock was handed over: it is kept here, never again in the library
    // 
    if (std::unique_ptr<Probed> p = take_probed(source, tag, comm))
      return land(p->bytes.data(), int(p->bytes.size()), p->st);
  }
  int n = 0;
  MPI_Get_count(&st, MPI_BYTE, &n);
  if (size_t(n) != sizeof(IpcDesc) && size_t(n) != sizeof(DirectDesc) && size_t(n) != sizeof(IpcCopyDesc))
    return TEMPI_UNLOCKED(next.MPI_Mrecv(buf, count, dt, &msg, status));
  alignas(16) char raw[kDescCap];
  TEMPI_UNLOCKED(next.MPI_Mrecv(raw, n, MPI_BYTE, &msg, &st));
  return land(raw, n, st);
}

bool holds(int source, int tag, MPI_Comm comm) {
  for (const auto &p : probed)
    if (probed_matches(*p, source, tag, comm)) return true;
  return false;
}

bool host_recv_aware(int source, int tag, MPI_Comm comm) {
  if (!state.active || !gpu::available() || source == MPI_PROC_NULL) return false;
  if (holds(source, tag, comm)) return true; // a probe holds a message it may match
  return source == MPI_ANY_SOURCE || topology::colocated(comm, source);
}

int irecv_host(void *buf, int count, MPI_Datatype dt, int source, int tag, MPI_Comm comm, MPI_Request *req) {
  counters.lib_recvs++;
  self_spill(comm, source);
  *req = add(new_host_irecv(buf, count, dt, source, tag, comm, take_probed(source, tag, comm)));
  return MPI_SUCCESS;
}

namespace {
// receive a library message of a descriptor's size to look at it
std::unique_ptr<Probed> receive_probed(MPI_Message *m, int n, MPI_Comm comm) {
  auto p = std::make_unique<Probed>();
  p->comm = comm;
  p->bytes.resize(size_t(n));
  next.MPI_Mrecv(p->bytes.data(), n, MPI_BYTE, m, &p->st);
  p->st.MPI_ERROR = MPI_SUCCESS;
  p->payload = descriptor_payload(p->bytes.data(), n);
  return p;
}

// A probe found a message of a descriptor's size from `src` with tag `tag`
// and must receive it to look at it. Messages of `src` earlier than it (other
// tags) would then be overtaken by a later receive that matches both (MPI's
// non-overtaking rule), so they are received first, in order, and
// kept too: the kept messages of a source are always its earliest, in send
// order, and every TEMPI receive takes from them before the library.
//
// At MPI_THREAD_MULTIPLE the blocking MPI_Probe that found the message ran
// without TEMPI's lock, so another thread may have received it (or the
// source's earlier ones) since: the library then has nothing (more) of src,
// and the caller simply probes again -- as the library's own
// probe information would be stale in that race too.
void hold_through(int src, int tag, MPI_Comm comm) {
  for (;;) {
    MPI_Message m = MPI_MESSAGE_NULL;
    MPI_Status st;
    int g = 0;
    next.MPI_Improbe(src, MPI_ANY_TAG, comm, &g, &m, &st); // the earliest message of src
    if (!g) {
      if (!mt::on) LOG_FATAL("a probed message could not be matched");
      return; // taken by another thread: probe again
    }
    int n = 0;
    MPI_Get_count(&st, MPI_BYTE, &n);
    probed.push_back(receive_probed(&m, n, comm));
    if (st.MPI_TAG == tag) return; // the probed message: the first of src with its tag
  }
}

void report(const Probed &p, MPI_Status *status) {
  if (status == MPI_STATUS_IGNORE) return;
  *status = p.st;
  set_received(status, p.payload);
}
} // namespace

int probe(int source, int tag, MPI_Comm comm, int *flag, MPI_Status *status) {
  if (source == MPI_PROC_NULL || !state.active || !gpu::available()) // no descriptors can arrive
    return flag ? next.MPI_Iprobe(source, tag, comm, flag, status)
                : TEMPI_UNLOCKED(next.MPI_Probe(source, tag, comm, status));
  self_spill(comm, source);
  if (flag && busy()) progress(false);
  for (;;) {
    for (const auto &p : probed)
      if (probed_matches(*p, source, tag, comm)) {
        report(*p, status);
        if (flag) *flag = 1;
        return MPI_SUCCESS;
      }
    int f = 0;
    MPI_Status st;
    int rc;
    if (!flag && !busy()) { // nothing of TEMPI's to keep moving: the library may block
      rc = TEMPI_UNLOCKED(next.MPI_Probe(source, tag, comm, &st));
      f = 1;
    } else {
      rc = next.MPI_Iprobe(source, tag, comm, &f, &st);
    }
    if (rc != MPI_SUCCESS) return rc;
    if (f) {
      int n = 0;
      MPI_Get_count(&st, MPI_BYTE, &n);
      // only a co-located sender (this process included) can send a
      // descriptor: anything else is reported as the library sees it
      if (!descriptor_sized(n) || !topology::colocated(comm, st.MPI_SOURCE)) {
        if (status != MPI_STATUS_IGNORE) *status = st;
        if (flag) *flag = 1;
        return MPI_SUCCESS;
      }
      // The earliest message from that source with that tag is the one just
      // probed (the library keeps one sender's messages in order, and any
      // earlier one would have matched the probe first): take it out to look
      // at it -- with the source's earlier messages, in order -- and keep it
      // for the receive that will match it.
      hold_through(st.MPI_SOURCE, st.MPI_TAG, comm);
      continue;
    }
    if (flag) {
      *flag = 0;
      return MPI_SUCCESS;
    }
    progress();
    mt::yield();
  }
}

int mprobe(int source, int tag, MPI_Comm comm, int *flag, MPI_Message *msg, MPI_Status *status) {
  if (source == MPI_PROC_NULL || !state.active || !gpu::available()) // no descriptors can arrive
    return flag ? next.MPI_Improbe(source, tag, comm, flag, msg, status)
                : TEMPI_UNLOCKED(next.MPI_Mprobe(source, tag, comm, msg, status));
  self_spill(comm, source);
  if (flag && busy()) progress(false);
  auto claim = [&](std::unique_ptr<Probed> p) { // a TEMPI message handle, outside the library's handle space
    report(*p, status);
    while (probedMsgs.count(nextMsgHandle) || nextMsgHandle == 0) nextMsgHandle = (nextMsgHandle + 1) % kHandleSpace;
    const uint32_t h = nextMsgHandle;
    nextMsgHandle = (nextMsgHandle + 1) % kHandleSpace;
    probedMsgs.emplace(h, std::move(p));
    *msg = MPI_Message(h);
    if (flag) *flag = 1;
    return MPI_SUCCESS;
  };
  for (;;) {
    if (std::unique_ptr<Probed> p = take_probed(source, tag, comm)) return claim(std::move(p));
    int f = 0;
    MPI_Status st;
    MPI_Message m = MPI_MESSAGE_NULL;
    int rc;
    if (!flag && !busy()) {
      rc = TEMPI_UNLOCKED(next.MPI_Mprobe(source, tag, comm, &m, &st));
      f = 1;
    } else {
      rc = next.MPI_Improbe(source, tag, comm, &f, &m, &st);
    }
    if (rc != MPI_SUCCESS) return rc;
    if (f) {
      int n = 0;
      MPI_Get_count(&st, MPI_BYTE, &n);
      // (a matched message leaves the matching order, so nothing before it
      // needs keeping; only a co-located sender can send a descriptor)
      if (!descriptor_sized(n) || !topology::colocated(comm, st.MPI_SOURCE)) { // the library's message, as it is
        *msg = m;
        libMsgComm[m] = comm;
        if (status != MPI_STATUS_IGNORE) *status = st;
        if (flag) *flag = 1;
        return MPI_SUCCESS;
      }
      return claim(receive_probed(&m, n, comm));
    }
    if (flag) {
      *flag = 0;
      return MPI_SUCCESS;
    }
    progress();
    mt::yield();
  }
}

int imrecv(void *buf, int count, MPI_Datatype dt, MPI_Message *msg, MPI_Request *req) {
  Route route;
  auto it = probedMsgs.find(uint32_t(*msg));
  if (it == probedMsgs.end()) { // the library's message
    MPI_Comm mc = MPI_COMM_WORLD; // (a message probed before TEMPI was active)
    auto lc = libMsgComm.find(*msg);
    if (lc != libMsgComm.end()) {
      mc = lc->second;
      libMsgComm.erase(lc);
    }
    if (*msg == MPI_MESSAGE_NULL || *msg == MPI_MESSAGE_NO_PROC || !handles(buf, count, dt, 0, &route))
      return next.MPI_Imrecv(buf, count, dt, msg, req);
    counters.irecvs++;
    if (!route.rec->packer) {
      *req = add(new_lib_irecv(buf, count, dt, MPI_ANY_SOURCE, MPI_ANY_TAG, mc, msg));
    } else {
      const int64_t bytes = packed_bytes(route.rec, count, dt, mc);
      char *origin = static_cast<char *>(route.ptr.dptr) - route.rec->desc.start;
      *req = add(new_irecv(route.rec, origin, count, dt, MPI_ANY_SOURCE, MPI_ANY_TAG, mc, route.ptr.device, bytes, msg));
    }
    *msg = MPI_MESSAGE_NULL;
    return MPI_SUCCESS;
  }
  std::unique_ptr<Probed> p = std::move(it->second);
  probedMsgs.erase(it);
  *msg = MPI_MESSAGE_NULL;
  const MPI_Comm comm = p->comm;
  if (!handles(buf, count, dt, 0, &route)) {
    *req = add(new_host_irecv(buf, count, dt, MPI_ANY_SOURCE, MPI_ANY_TAG, comm, std::move(p)));
    return MPI_SUCCESS;
  }
  counters.irecvs++;
  if (!route.rec->packer) {
    *req = add(new_lib_irecv(buf, count, dt, MPI_ANY_SOURCE, MPI_ANY_TAG, comm, nullptr, std::move(p)));
    return MPI_SUCCESS;
  }
  const int64_t bytes = packed_bytes(route.rec, count, dt, comm);
  char *origin = static_cast<char *>(route.ptr.dptr) - route.rec->desc.start;
  *req = add(new_irecv(route.rec, origin, count, dt, MPI_ANY_SOURCE, MPI_ANY_TAG, comm, route.ptr.device, bytes, nullptr,
                          std::move(p)));
  return MPI_SUCCESS;
}

int mrecv(void *buf, int count, MPI_Datatype dt, MPI_Message *msg, MPI_Status *status) {
  Route route;
  if (!probedMsgs.count(uint32_t(*msg)) && !handles(buf, count, dt, 0, &route)) {
    libMsgComm.erase(*msg);
    return TEMPI_UNLOCKED(next.MPI_Mrecv(buf, count, dt, msg, status)); // the library's message into host memory
  }
  MPI_Request r = MPI_REQUEST_NULL;
  const int rc = imrecv(buf, count, dt, msg, &r);
  if (rc != MPI_SUCCESS) return rc;
  return is_tempi_request(r) ? wait(&r, status) : TEMPI_UNLOCKED(next.MPI_Wait(&r, status));
}

} // namespace p2p
} // namespace tempi
