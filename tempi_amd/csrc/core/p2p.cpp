// tempi_amd/csrc/core/p2p.cpp -- see p2p.hpp; the request table, routing of
// isend / irecv, progress and the waits (the rest: p2p_internal.hpp)
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
// The operations in flight, by request handle. Handles are handed out in
// sequence (mod kHandleSpace, never 0) and the table is direct-mapped: handle
// h lives in slot h & mask, so finding a request is one index and one compare
// (a halo substep waits on 416 requests, most of them already complete: three
// hash lookups each were a third of its tail, profiles/r05/halo_tl*). A
// handle whose slot is still taken by an older operation is skipped; the
// table doubles when half full (entries never collide after doubling: equal
// low bits under the new mask would mean equal slots under the old one).
class OpTable {
  struct Slot {
    uint32_t h = 0;
    std::unique_ptr<Op> op;
  };
  std::vector<Slot> slots_ = std::vector<Slot>(4096);
  size_t mask_ = 4095, n_ = 0;

  void grow() {
    std::vector<Slot> old(slots_.size() * 2);
    old.swap(slots_);
    mask_ = slots_.size() - 1;
    for (Slot &s : old)
      if (s.op) slots_[s.h & mask_] = std::move(s);
  }

public:
  Op *get(uint32_t h) const {
    const Slot &s = slots_[h & mask_];
    return h && s.h == h ? s.op.get() : nullptr;
  }
  bool slot_free(uint32_t h) const { return !slots_[h & mask_].op; }
  void put(uint32_t h, std::unique_ptr<Op> op) {
    if (2 * (n_ + 1) > slots_.size()) grow();
    Slot &s = slots_[h & mask_];
    s.h = h;
    s.op = std::move(op);
    ++n_;
  }
  // the slot is cleared before the operation is destroyed (a destructor may
  // free or add other requests)
  void erase(uint32_t h) {
    Slot &s = slots_[h & mask_];
    if (!h || s.h != h || !s.op) return;
    std::unique_ptr<Op> dead = std::move(s.op);
    s.h = 0;
    --n_;
  }
  size_t size() const { return n_; }
  bool all_done() const {
    for (const Slot &s : slots_)
      if (s.op && !s.op->done) return false;
    return true;
  }
  void clear() {
    std::vector<Slot> old(slots_.size());
    old.swap(slots_);
    n_ = 0;
  }
};
OpTable active;
uint32_t nextHandle = 1;
std::vector<uint32_t> detachedOps; // freed by the application, still running
} // namespace

MPI_Request add(std::unique_ptr<Op> op) {
  uint32_t h = nextHandle;
  while (h == 0 || !active.slot_free(h)) h = (h + 1) % kHandleSpace; // (a free slot holds no live handle)
  nextHandle = (h + 1) % kHandleSpace;
  active.put(h, std::move(op));
  return MPI_Request(h);
}

namespace {
// scratch for progress()
std::vector<MPI_Request> pollReqs;
std::vector<Op *> pollOps;   // nullptr: a pending ack
std::vector<PendingAck *> pollAck; // the pending ack of each request (nullptr: an op's)
int progressDepth = 0;             // progress() passes on the stack
std::vector<int> pollIdx;
std::vector<MPI_Status> pollSt;
} // namespace
} // namespace detail

using namespace detail;

int collectiveDepth = 0;

void init() {
  gpu::choose_lanes(topology::ranks_on_node());
  gpuAwareLibrary = std::getenv("TEMPI_MPI_GPU_AWARE") != nullptr;
  directEnabled = std::getenv("TEMPI_NO_DIRECT") == nullptr;
  selfChannelEnabled = directEnabled && std::getenv("TEMPI_NO_SELF_CHANNEL") == nullptr; // it carries direct sends
  clear_channels();
  faultCanary = std::getenv("TEMPI_FAULT_CANARY") != nullptr;
  clear_canary();
  ipcCopyEnabled = std::getenv("TEMPI_NO_IPC_COPY") == nullptr;
  if (const char *s = std::getenv("TEMPI_IPC_COPY_MIN_BYTES")) ipcCopyMinBytes = std::atoll(s);
  if (const char *s = std::getenv("TEMPI_IPC_COPY_MIN_BLOCK")) ipcCopyMinBlock = std::atoll(s);
  scattersInFlight = 0;
  batchesInFlight = 0;
  directShared.clear();
  directShared.reserve(512);
  systemPerformanceLoaded = import_system_performance(&systemPerformance);
  clear_model_cache();
  MPI_Comm_dup(MPI_COMM_WORLD, &ctrlComm);
  int flag = 0;
  int *ub = nullptr;
  MPI_Comm_get_attr(MPI_COMM_WORLD, MPI_TAG_UB, &ub, &flag);
  if (flag && ub) tagUb = *ub;
  board_init();
  boardOps.clear();
}

void reload_perf_model() {
  systemPerformanceLoaded = import_system_performance(&systemPerformance);
  clear_model_cache();
}

void finalize() {
  // complete everything the application left behind, then wait (bounded) for
  // the acks that let us release IPC slabs
  const auto t0 = std::chrono::steady_clock::now();
  auto all_done = [] { return active.all_done(); };
  while (!all_done()) {
    progress();
    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(30)) {
      LOG_WARN("request(s) left incomplete at MPI_Finalize");
      break;
    }
  }
  clear_channels(); // (receives still waiting there die with `active`)
  active.clear();
  detachedOps.clear();
  clear_gates();
  libWatch.clear();
  boardOps.clear(); // (their ops died with `active`)
  for (auto &b : batches)
    if (b->event) tempi_hip_event_destroy(b->event);
  batches.clear();
  scattersInFlight = 0;
  batchesInFlight = 0;
  while (!pendingAcks.empty()) {
    progress();
    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(30)) {
      LOG_WARN(pendingAcks.size() << " IPC slab(s) never acknowledged; abandoning");
      for (auto &pa : pendingAcks)
        if (pa->req != MPI_REQUEST_NULL) MPI_Cancel(&pa->req);
      pendingAcks.clear();
    }
  }
  destroy_events();
  close_mappings();
  if (ctrlComm != MPI_COMM_NULL) MPI_Comm_free(&ctrlComm);
  board_finalize();
  device_pool().release_all();
  pinned_pool().release_all();
}

bool handles(const void *buf, int count, MPI_Datatype dt, int peer, Route *route) {
  if (!state.active || !gpu::available() || count <= 0 || peer == MPI_PROC_NULL) return false;
  const TypeRecord *rec = type_lookup(dt);
  if (!rec || rec->desc.size == 0) return false;
  const int64_t first = rec->desc.valid ? rec->desc.start : 0;
  const gpu::Ptr p = gpu::classify(static_cast<const char *>(buf) + first);
  if (!p.device_accessible) return false;
  route->rec = rec;
  route->ptr = p;
  return true;
}


int isend(const void *buf, int count, MPI_Datatype dt, int dest, int tag, MPI_Comm comm, MPI_Request *req,
          const Route &route, int force, bool blocking, SendMode mode) {
  const TypeRecord *rec = route.rec;
  ScopedNs timer(counters.ns_isend);
  if (pendingPack.size() >= kMaxPending) flush(); // (no progress(): consecutive Isends share a launch)
  counters.isends++;
  if (!rec->packer) {
    self_spill(comm, dest);
    *req = add(new_lib_isend(buf, count, dt, dest, tag, comm, mode));
    return MPI_SUCCESS;
  }
  const gpu::Ptr &p = route.ptr;
  const int64_t bytes = packed_bytes(rec, count, dt, comm);
  const char *origin = static_cast<const char *>(p.dptr) - rec->desc.start;
  const int destWorld = topology::world_rank(comm, dest);
  // a non-blocking send to this same process: the receiver copies directly
  tempi_hip_desc flat;
  if (directEnabled && !blocking && mode != SendMode::SYNC && mode != SendMode::BUFFERED && force < 0 && destWorld == state.worldRank &&
      rec->flat(count, &flat)) {
    counters.send_direct++;
    counters.bytes_direct += uint64_t(bytes);
    *req = add(new_isend_direct(rec, origin, count, dt, dest, tag, comm, p.device, bytes, flat));
    return MPI_SUCCESS;
  }
  if (destWorld == state.worldRank) spill_channel(comm); // a message to this rank the self channel cannot carry
  const bool colocated = topology::colocated_world(destWorld);
  modelBlock = std::min<int64_t>(std::max<int64_t>(1, rec->desc.block), 512);
  Method m = choose(bytes, colocated, blocking);
  if (force >= 0) m = Method(force);
  if (m == Method::IPC && (!colocated || ipc_broken(destWorld))) m = Method::ONESHOT;
  if (m == Method::DEVICE && !gpuAwareLibrary) m = colocated ? Method::IPC : Method::STAGED;
  // a buffered send must fit the buffer the application attached for its bytes
  if (mode == SendMode::BUFFERED && m == Method::IPC && bytes < int64_t(sizeof(IpcDesc))) m = Method::ONESHOT;
  switch (m) {
  case Method::ONESHOT:
    counters.send_oneshot++;
    counters.bytes_oneshot += uint64_t(bytes);
    break;
  case Method::STAGED:
    counters.send_staged++;
    counters.bytes_staged += uint64_t(bytes);
    break;
  case Method::DEVICE:
    counters.send_device++;
    counters.bytes_device += uint64_t(bytes);
    break;
  case Method::IPC:
    counters.send_ipc++;
    counters.bytes_ipc += uint64_t(bytes);
    break;
  default: break;
  }
  // IPC COPY: a large message of wide rows is copied by the receiver straight
  // out of this process's object (no gather, no slab)
  const int64_t copyMin = collectiveDepth > 0 ? 1 : ipcCopyMinBytes;
  if (m == Method::IPC && ipcCopyEnabled && mode != SendMode::BUFFERED && bytes >= copyMin && rec->flat(count, &flat) &&
      flat.ndims <= 3 && flat.block >= ipcCopyMinBlock && bytes < (int64_t(1) << 31)) {
    IpcCopyDesc d{};
    d.magic[0] = kMagicCopy;
    d.magic[1] = kMagic1;
    d.bytes = bytes;
    d.senderWorld = state.worldRank;
    d.senderPid = state.pid;
    d.device = p.device;
    d.rawFirst = reinterpret_cast<uint64_t>(origin + rec->desc.start);
    d.desc = flat;
    d.gpu = gpu::identity(p.device);
    const int half = std::max(1, tagUb / 2);
    d.ackTag = half + int32_t(nextCopyTag++ % uint32_t(half)); // slab ids (the IPC acks) stay below
    if (export_object(origin + rec->desc.start, &d)) {
      counters.send_ipc_copy++;
      counters.bytes_ipc_copy += uint64_t(bytes);
      *req = add(new_isend_copy(rec, origin, count, dt, dest, tag, comm, p.device, bytes, destWorld, d));
      return MPI_SUCCESS;
    }
  }
  int cur = 0;
  tempi_hip_get_device(&cur);
  if (cur != p.device) tempi_hip_set_device(p.device);
  *req = add(new_isend(rec, origin, count, dt, dest, tag, comm, p.device, m, bytes, mode));
  if (cur != p.device) tempi_hip_set_device(cur);
  return MPI_SUCCESS;
}

int irecv(void *buf, int count, MPI_Datatype dt, int source, int tag, MPI_Comm comm, MPI_Request *req,
          const Route &route) {
  const TypeRecord *rec = route.rec;
  // start queued gathers (a burst of Isends shares this launch); the rest of
  // progress is left to the waits, so a burst of Irecvs stays O(1) each
  if (!pendingPack.empty()) flush_list(pendingPack, true);
  const uint64_t t0 = tick();
  counters.irecvs++;
  std::unique_ptr<Probed> pre = take_probed(source, tag, comm); // a probe already received it
  if (source == MPI_ANY_SOURCE || !rec->packer) self_spill(comm, source); // (receives from this rank: the channel's)
  if (!rec->packer) {
    *req = add(new_lib_irecv(buf, count, dt, source, tag, comm, nullptr, std::move(pre)));
    return MPI_SUCCESS;
  }
  const gpu::Ptr &p = route.ptr;
  const int64_t bytes = packed_bytes(rec, count, dt, comm);
  char *origin = static_cast<char *>(p.dptr) - rec->desc.start;
  *req = add(new_irecv(rec, origin, count, dt, source, tag, comm, p.device, bytes, nullptr, std::move(pre)));
  // keep the GPU busy while the caller is still posting: launch arrived
  // messages' copies / unpacks once a launch's worth has queued up
  // (sooner while the GPU has no scatter work: the first batch starts early)
  if (pendingUnpack.size() >= (scattersInFlight ? kEarlyFlush : kFirstFlush)) flush_list(pendingUnpack, false);
  tock(counters.ns_irecv, t0);
  return MPI_SUCCESS;
}

bool local_copy(const void *sbuf, int scount, MPI_Datatype stype, void *rbuf, int rcount, MPI_Datatype rtype,
                MPI_Request *req) {
  LocalCopies plan;
  if (!plan_local_copy(sbuf, scount, stype, rbuf, rcount, rtype, &plan)) return false;
  *req = start_local_copies(plan);
  return true;
}

MPI_Request start_local_copies(const LocalCopies &plan) {
  counters.send_direct += plan.items.size();
  counters.bytes_direct += uint64_t(plan.bytes);
  return add(new_local_copies(plan));
}

bool plan_local_copy(const void *sbuf, int scount, MPI_Datatype stype, void *rbuf, int rcount, MPI_Datatype rtype,
                     LocalCopies *plan) {
  if (!directEnabled) return false;
  Route sr, rr;
  if (!handles(sbuf, scount, stype, 0, &sr) || !handles(rbuf, rcount, rtype, 0, &rr)) return false;
  if (!sr.rec->packer || !rr.rec->packer || !sr.rec->desc.valid || !rr.rec->desc.valid) return false;
  if (sr.ptr.device != rr.ptr.device) return false;
  const int64_t bytes = sr.rec->desc.size * int64_t(scount);
  if (bytes != rr.rec->desc.size * int64_t(rcount) || bytes <= 0) return false;
  tempi_hip_desc sflat, rflat;
  if (!sr.rec->flat(scount, &sflat) || !rr.rec->flat(rcount, &rflat) || !copy_ok(rflat, sflat)) return false;
  tempi_hip_copy_item c{};
  c.src_first = sr.ptr.dptr;
  c.dst_first = rr.ptr.dptr;
  c.src = sflat;
  c.dst = rflat;
  if (plan->device >= 0 && plan->device != rr.ptr.device) return false; // one request, one device
  plan->device = rr.ptr.device;
  plan->items.push_back(c);
  plan->recs.push_back(sr.rec->ref());
  plan->recs.push_back(rr.rec->ref());
  plan->bytes += bytes;
  return true;
}

void start_queued() {
  if (!pendingPack.empty()) flush_list(pendingPack, true);
  if (!pendingUnpack.empty()) flush_list(pendingUnpack, false);
}

bool send_gated(MPI_Comm comm, int dest) { return gate_busy(gate_key(comm, dest)); }

void self_spill(MPI_Comm comm, int peer) {
  if (!state.active || !selfChannelEnabled || peer == MPI_PROC_NULL) return;
  if (peer != MPI_ANY_SOURCE && topology::world_rank(comm, peer) != state.worldRank) return;
  spill_channel(comm);
}

void self_forget(MPI_Comm comm) { forget_channel(comm); }

int isend_host(const void *buf, int count, MPI_Datatype dt, int dest, int tag, MPI_Comm comm, MPI_Request *req) {
  counters.lib_sends++;
  *req = add(new_host_isend(buf, count, dt, dest, tag, comm));
  return MPI_SUCCESS;
}

void drain_sends(MPI_Comm comm, int dest) {
  const uint64_t key = gate_key(comm, dest);
  while (gate_busy(key)) {
    progress();
    mt::yield();
  }
}

void drain_buffered() {
  while (bufferedUnposted > 0) {
    progress();
    mt::yield();
  }
}

bool is_tempi_request(MPI_Request r) {
  const uint32_t h = uint32_t(r);
  return h < kHandleSpace && active.get(h) != nullptr;
}

namespace detail {
Op *find_op(MPI_Request r) {
  const uint32_t h = uint32_t(r);
  return h < kHandleSpace ? active.get(h) : nullptr;
}
} // namespace detail

bool peek(MPI_Request r) {
  Op *op = find_op(r);
  if (!op) return false;
  if (PersistentOp *p = op->persistent()) return persistent_peek(p);
  return op->done;
}

void release(MPI_Request *req) {
  const uint32_t h = uint32_t(*req);
  if (Op *op = find_op(*req)) {
    if (PersistentOp *p = op->persistent()) {
      persistent_free(p);
      active.erase(h);
    } else if (op->done) {
      active.erase(h);
    } else {
      op->detached = true;
      detachedOps.push_back(h);
    }
  }
  *req = MPI_REQUEST_NULL;
}

int get_status(MPI_Request r, int *flag, MPI_Status *status) {
  Op *op = find_op(r);
  if (!op) return next.MPI_Request_get_status(r, flag, status);
  if (PersistentOp *p = op->persistent()) return persistent_get_status(p, flag, status);
  progress();
  *flag = op->done ? 1 : 0; // (progress never frees an application-visible request)
  if (*flag) op->status(status);
  return MPI_SUCCESS;
}

int cancel(MPI_Request r) {
  Op *op = find_op(r);
  if (!op) return MPI_SUCCESS;
  if (PersistentOp *p = op->persistent()) return persistent_cancel(p);
  op->cancel();
  return MPI_SUCCESS;
}

namespace {
// Queued scatters / copies are launched by a waiting pass only while a
// scatter lane is free, or once a launch's worth has queued: with every lane
// busy the GPU has work either way, and messages arriving one at a time then
// share a launch instead of each taking one (a cheap pass -- no library
// request to test -- would otherwise launch every arrival on its own).
bool scatter_flush_due() {
  return scattersInFlight < std::max(1, gpu::lanes() - 1) || pendingUnpack.size() >= kEarlyFlush;
}
} // namespace

bool progress(bool full) {
  bool moved = false;
  counters.progress_passes++;
  // a pass run from inside a callback of an outer pass (a wait inside it)
  // leaves finished detached operations to the outer pass, whose recorded
  // completions may still name them
  struct Depth {
    int &d;
    explicit Depth(int &x) : d(++x) {}
    ~Depth() { --d; }
  } depth(progressDepth);
  // 0. launch queued gathers (one launch per batch group); scatters too when
  //    the caller is about to wait
  if (!pendingPack.empty()) {
    flush_list(pendingPack, true);
    moved = true;
  }
  if (full && !pendingUnpack.empty() && scatter_flush_due()) {
    flush_list(pendingUnpack, false);
    moved = true;
  }
  // 1. GPU events, in launch order (a later event of the same stream cannot
  //    complete before an earlier one)
  uint64_t t0 = tick();
  uint64_t blocked = 0; // streams (bit per device x lane) with an incomplete batch
  for (auto &b : batches) {
    const uint64_t bit = uint64_t(1) << ((b->device * gpu::kMaxLanes + b->lane) & 63);
    if (b->complete || (blocked & bit)) continue;
    if (b->flag) { // the batch's last launch stores its ticket (tickets of a stream ascend)
      if (int32_t(__atomic_load_n(b->flag, __ATOMIC_ACQUIRE) - b->ticket) < 0) {
        // not yet: now and then ask the stream, so that a faulted launch (which
        // would never store the ticket) ends in its error instead of a hang
        if ((++b->polls & 255) == 0) {
          const int q = tempi_hip_stream_query(b->stream);
          if (q == 0 && int32_t(__atomic_load_n(b->flag, __ATOMIC_ACQUIRE) - b->ticket) < 0)
            LOG_FATAL("a batch's stream is idle but its completion ticket was never stored");
          if (q != 1) gpu::check(q, "stream query");
        }
        if (int32_t(__atomic_load_n(b->flag, __ATOMIC_ACQUIRE) - b->ticket) < 0) {
          blocked |= bit;
          continue;
        }
      }
    } else {
      const int q = tempi_hip_event_query(b->event);
      if (q == 1) {
        blocked |= bit;
        continue;
      }
      gpu::check(q, "event query");
      put_event(b->event);
      b->event = nullptr;
    }
    b->complete = true;
    batch_observed_done();
    if (trace::timelineOn) trace::mark(b->scatter ? "batch done (scatter)" : "batch done (gather)", 2);
    if (b->scatter) --scattersInFlight;
    std::vector<Op *> ops;
    ops.swap(b->ops);
    for (Op *op : ops) op->gpu_done();
    moved = true;
  }
  while (!batches.empty() && batches.front()->complete) batches.pop_front();
  tock(counters.ns_events, t0);
  t0 = tick();
  // 2. acks on this rank's board, then every outstanding library request in
  //    one MPI_Testsome. Completions are recorded -- requests cleared, the
  //    watch list compacted, acknowledged slabs released -- before any
  //    operation's callback runs: a callback may wait for something (a
  //    descriptor landing in a host buffer does), and so run a nested pass,
  //    which must not test a request the library has already completed and
  //    freed.
  if (!boardOps.empty()) {
    size_t w = 0;
    for (size_t i = 0; i < boardOps.size(); ++i) {
      Op *op = boardOps[i];
      const int code = board_poll(op->boardSlot);
      if (code < 0) {
        boardOps[w++] = op;
        continue;
      }
      op->boardSlot = -1;
      op->acked(code);
      moved = true;
    }
    boardOps.resize(w);
  }
  std::vector<PendingAck *> acked;
  pollReqs.clear();
  pollOps.clear();
  pollAck.clear();
  for (Op *op : libWatch) {
    pollReqs.push_back(op->lib);
    pollOps.push_back(op);
    pollAck.push_back(nullptr);
  }
  for (auto &p : pendingAcks) {
    PendingAck &pa = *p;
    if (!pa.onBoard) {
      pollReqs.push_back(pa.req);
      pollOps.push_back(nullptr);
      pollAck.push_back(&pa);
    } else if ((pa.code = board_poll(pa.tag)) >= 0) {
      acked.push_back(&pa);
    }
  }
  std::vector<std::pair<Op *, MPI_Status>> completed;
  if (!pollReqs.empty()) {
    const int n = int(pollReqs.size());
    pollIdx.resize(size_t(n));
    pollSt.resize(size_t(n));
    int outcount = 0;
    const int trc = next.MPI_Testsome(n, pollReqs.data(), &outcount, pollIdx.data(), pollSt.data());
    if (outcount == MPI_UNDEFINED) outcount = 0;
    if (trc != MPI_ERR_IN_STATUS) // the statuses' MPI_ERROR fields are set only with this code
      for (int k = 0; k < outcount; ++k) pollSt[size_t(k)].MPI_ERROR = MPI_SUCCESS;
    for (int k = 0; k < outcount; ++k) {
      const size_t i = size_t(pollIdx[size_t(k)]);
      if (Op *op = pollOps[i]) {
        op->lib = MPI_REQUEST_NULL;
        completed.emplace_back(op, pollSt[size_t(k)]);
      } else {
        pollAck[i]->req = MPI_REQUEST_NULL;
        acked.push_back(pollAck[i]);
      }
    }
    if (!completed.empty()) { // drop completed requests from the watch list
      size_t w = 0;
      for (Op *op : libWatch) {
        if (op->lib != MPI_REQUEST_NULL)
          libWatch[w++] = op;
        else
          op->watched = false;
      }
      libWatch.resize(w);
    }
  }
  // release acknowledged slabs
  for (PendingAck *pa : acked) {
    if (pa->code == 1) { // the receiver could not map the slab: send the bytes through the host
      mark_ipc_broken(pa->peer);
      Slab *h = pinned_pool().get(size_t(pa->bytes), pa->slab->device);
      gpu::check(tempi_hip_memcpy(h->host, pa->slab->dev, size_t(pa->bytes)), "ipc fallback D2H");
      next.MPI_Send(h->host, int(pa->bytes), MPI_PACKED, pa->peer, pa->tag, ctrlComm); // receive already posted
      pinned_pool().put(h);
    }
    device_pool().put(pa->slab);
    pa->slab = nullptr;
  }
  if (!acked.empty()) {
    pendingAcks.erase(std::remove_if(pendingAcks.begin(), pendingAcks.end(),
                                     [](const std::unique_ptr<PendingAck> &p) { return !p->slab; }),
                      pendingAcks.end());
    moved = true;
  }
  // the callbacks of the completed library requests, last
  for (auto &c : completed) c.first->lib_done(c.second);
  if (!completed.empty()) moved = true;
  tock(counters.ns_testsome, t0);
  // 3. unpacks of messages that arrived: launched together when the caller
  //    is about to wait for them (light passes from MPI_Isend / MPI_Irecv
  //    only queue them, so a burst of receives shares one launch)
  if (!pendingUnpack.empty() && (full || pendingUnpack.size() >= kMaxPending) && scatter_flush_due())
    flush_list(pendingUnpack, false);
  // 4. operations the application freed with MPI_Request_free
  if (!detachedOps.empty() && progressDepth == 1) {
    size_t w = 0;
    for (uint32_t h : detachedOps) {
      Op *op = active.get(h);
      if (!op) continue;
      if (op->done)
        active.erase(h);
      else
        detachedOps[w++] = h;
    }
    detachedOps.resize(w);
  }
  return moved;
}

// (idle persistent requests are not work; started ones have an inner request)
int progress_depth() { return progressDepth; }

bool busy() { return active.size() > size_t(persistent_count) || !pendingAcks.empty(); }

namespace {
// a completed operation's error, raised on its communicator's handler (as
// the library does for its own requests) and returned
int finish_error(int err, MPI_Comm comm) {
  if (err == MPI_SUCCESS) return MPI_SUCCESS;
  return raise_error(comm == MPI_COMM_NULL ? MPI_COMM_WORLD : comm, err);
}
} // namespace

int wait(MPI_Request *req, MPI_Status *status) {
  const uint32_t h = uint32_t(*req);
  Op *op = find_op(*req);
  if (!op) return TEMPI_UNLOCKED(next.MPI_Wait(req, status));
  if (PersistentOp *p = op->persistent()) return persistent_wait(p, status);
  if (!op->done) {
    ScopedNs timer(counters.ns_wait);
    while (!op->done) {
      progress();
      if (!op->done) op->stalled();
      if (!op->done) mt::yield();
    }
  }
  op->status(status);
  const int err = op->err;
  const MPI_Comm ec = op->errComm;
  active.erase(h);
  *req = MPI_REQUEST_NULL;
  return finish_error(err, ec);
}

int test(MPI_Request *req, int *flag, MPI_Status *status) {
  const uint32_t h = uint32_t(*req);
  Op *op = find_op(*req);
  if (!op) return next.MPI_Test(req, flag, status);
  if (PersistentOp *p = op->persistent()) return persistent_test(p, flag, status);
  progress();
  if (!op->done) op->stalled();
  *flag = op->done ? 1 : 0;
  if (*flag) {
    op->status(status);
    const int err = op->err;
    const MPI_Comm ec = op->errComm;
    active.erase(h);
    *req = MPI_REQUEST_NULL;
    return finish_error(err, ec);
  }
  return MPI_SUCCESS;
}


} // namespace p2p
} // namespace tempi
