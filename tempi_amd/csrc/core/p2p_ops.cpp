// tempi_amd/csrc/core/p2p_ops.cpp -- operation plumbing and the send state
// machines (p2p_internal.hpp)
#include "p2p_internal.hpp"

#include "alloc.hpp"
#include "counters.hpp"
#include "env.hpp"
#include "gpu.hpp"
#include "log.hpp"
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

std::pmr::unsynchronized_pool_resource &op_pool() {
  static auto *pool = new std::pmr::unsynchronized_pool_resource();
  return *pool;
}

// ---------------------------------------------------------------- operations
//
// Every operation is a small state machine with at most one GPU event and at
// most one library request outstanding. progress() polls GPU events in
// creation order, skipping the rest of a stream (device x lane) once one of
// its events is incomplete (each lane is an in-order stream, so its later
// events cannot be complete either), then tests every outstanding library
// request with a single MPI_Testsome. A pass therefore costs O(newly completed) HIP queries
// plus one library call, instead of one query and one MPI_Test per operation
// (the reference's try_progress wakes every operation: async_operation.cpp:
// 501-513).

void fail_post(Op *op, int rc, MPI_Comm comm) {
  op->lib = MPI_REQUEST_NULL;
  op->err = rc;
  op->errComm = comm;
  op->done = true;
}

std::vector<void *> eventPool;

void *get_event() {
  if (!eventPool.empty()) {
    void *e = eventPool.back();
    eventPool.pop_back();
    return e;
  }
  void *e = nullptr;
  gpu::check(tempi_hip_event_create(&e, 0), "event create");
  return e;
}

void put_event(void *e) {
  if (e) eventPool.push_back(e);
}

void destroy_events() {
  for (void *e : eventPool) tempi_hip_event_destroy(e);
  eventPool.clear();
}

std::deque<std::shared_ptr<GpuBatch>> batches;

// ops waiting for an ack on this rank's board (polled by progress())
std::vector<Op *> boardOps;

// ops with a library request outstanding (tested together by progress()).
// Every post of Op::lib is followed by watch(op).
std::vector<Op *> libWatch;
void watch(Op *op) {
  if (!op->watched && op->lib != MPI_REQUEST_NULL) {
    op->watched = true;
    libWatch.push_back(op);
  }
}
void unwatch(Op *op) {
  if (!op->watched) return;
  libWatch.erase(std::find(libWatch.begin(), libWatch.end(), op));
  op->watched = false;
}

// MPI's non-overtaking rule: sends from this process to one (comm, dest) reach
// the library in call order. An IsendOp reaches it only when its gather has
// run (gpu_done), so while one is still gathering, any later send to the same
// peer -- even one that could go at once (a direct descriptor, a
// library-packed type, a host buffer) -- queues behind it in that peer's gate
// and is posted when everything ahead of it has been. Gates are keyed by
// (comm, dest); ops never leave a gate before posting, and nothing waits on a
// receiver to post, so a gate always drains. (The reference lets such sends
// overtake; SURVEY F-list.)
namespace {
struct SendGate {
  std::vector<Op *> q;
  size_t head = 0;
  bool busy() const { return head < q.size(); }
};
std::unordered_map<uint64_t, SendGate> gates;
size_t gatedOps = 0; // ops in any gate: 0 means every send may post at once
} // namespace

uint64_t gate_key(MPI_Comm comm, int dest) {
  uint64_t c = 0;
  std::memcpy(&c, &comm, std::min(sizeof comm, sizeof c));
  return (c * 0x9e3779b97f4a7c15ull) ^ uint64_t(uint32_t(dest));
}

bool gate_busy(uint64_t key) {
  if (!gatedOps) return false;
  auto it = gates.find(key);
  return it != gates.end() && it->second.busy();
}

void gate_enter(uint64_t key, Op *op) {
  gates[key].q.push_back(op);
  ++gatedOps;
}

// post every op at the head of the gate that may go
void gate_advance(uint64_t key) {
  SendGate &g = gates[key];
  while (g.busy() && g.q[g.head]->ready) {
    Op *op = g.q[g.head++];
    --gatedOps;
    op->posted = true;
    op->post();
  }
  if (!g.busy()) {
    g.q.clear();
    g.head = 0;
  }
}

// a send that could post at once: now, unless an earlier send to the same
// peer is still gathering
void post_or_queue(uint64_t key, Op *op) {
  op->ready = true;
  if (gate_busy(key)) {
    gate_enter(key, op);
  } else {
    op->posted = true;
    op->post();
  }
}

void clear_gates() {
  gates.clear();
  gatedOps = 0;
}

void PendingList::add_items(const Op *op, const Packer &pk, void *packed, const void *origin, int64_t count) {
  pk.items(packed, origin, count, items);
  itemDev.resize(items.size(), op->device);
}

PendingList pendingPack, pendingUnpack;
int64_t bufferedUnposted = 0;

void Op::count_buffered() {
  if (!unpostedBuffered) ++bufferedUnposted;
  unpostedBuffered = true;
}

void Op::settle_buffered() {
  if (unpostedBuffered) --bufferedUnposted;
  unpostedBuffered = false;
}
int scattersInFlight = 0;
int batchesInFlight = 0;
uint64_t inflightSince = 0; // (ns) the first of the batches now in flight was launched

void batch_launched() {
  if (batchesInFlight++ == 0) inflightSince = now_ns();
}

void batch_observed_done() {
  if (batchesInFlight > 0 && --batchesInFlight == 0) counters.ns_gpu_inflight += now_ns() - inflightSince;
}

namespace {
template <typename T> const T *select(const std::vector<T> &v, const std::vector<int> &dev, int d, bool all,
                                      std::vector<T> &tmp) {
  if (all) return v.data();
  tmp.clear();
  for (size_t i = 0; i < v.size(); ++i)
    if (dev[i] == d) tmp.push_back(v[i]);
  return tmp.data();
}

int nextLane = 0; // round robin over the scatter lanes
} // namespace

void flush_list(PendingList &list, bool pack) {
  if (list.empty()) return;
  TEMPI_RANGE(pack ? "tempi::launch gathers" : "tempi::launch scatters/copies");
  ScopedNs timer(counters.ns_flush);
  // gathers (and anything ordered after one) run on lane 0; scatters and
  // copies take the other lanes in turn, so consecutive batches overlap
  int lane = 0;
  if (!pack && list.afterPack) flush_list(pendingPack, true); // that gather goes first
  if (!pack && !list.afterPack && gpu::lanes() > 1) {
    lane = 1 + nextLane;
    nextLane = (nextLane + 1) % (gpu::lanes() - 1);
  }
  // group by device (almost always one)
  int devices[64];
  int ndev = 0;
  for (const Op *op : list.ops) {
    int k = 0;
    while (k < ndev && devices[k] != op->device) ++k;
    if (k == ndev && ndev < 64) devices[ndev++] = op->device;
  }
  const bool all = ndev == 1;
  std::vector<tempi_hip_batch_item> itmp;
  std::vector<tempi_hip_copy_item> ctmp;
  for (int di = 0; di < ndev; ++di) {
    const int dev = devices[di];
    const tempi_hip_batch_item *items = select(list.items, list.itemDev, dev, all, itmp);
    const size_t nitems = all ? list.items.size() : itmp.size();
    const tempi_hip_copy_item *copies = select(list.copies, list.copyDev, dev, all, ctmp);
    const size_t ncopies = all ? list.copies.size() : ctmp.size();
    void *s = gpu::stream(dev, lane);
    int cur = 0;
    tempi_hip_get_device(&cur);
    if (cur != dev) tempi_hip_set_device(dev);
    counters.batches++;
    counters.batched_items += nitems + ncopies;
    // the last launch of the batch may store a completion ticket itself
    // (never after a staged copy, which is not a kernel)
    bool staged = false;
    for (const PendingList::Stage &st : list.stages) staged |= st.dev == dev;
    const bool ticketed = !staged;
    const uint32_t *flag = nullptr;
    uint32_t ticket = 0;
    if (nitems) {
      const bool last = ticketed && !ncopies;
      const int e = pack ? (last ? tempi_hip_pack_batch_ticket(items, int(nitems), s, &flag, &ticket)
                                 : tempi_hip_pack_batch(items, int(nitems), s))
                         : (last ? tempi_hip_unpack_batch_ticket(items, int(nitems), s, &flag, &ticket)
                                 : tempi_hip_unpack_batch(items, int(nitems), s));
      gpu::check(e, pack ? "batched pack" : "batched unpack");
    }
    if (ncopies)
      gpu::check(ticketed ? tempi_hip_copy_batch_ticket(copies, int(ncopies), s, &flag, &ticket)
                          : tempi_hip_copy_batch(copies, int(ncopies), s),
                 "batched direct copy");
    for (const PendingList::Stage &st : list.stages)
      if (st.dev == dev) gpu::check(tempi_hip_memcpy_async(st.dst, st.src, st.n, s), "staged D2H");
    auto b = std::make_shared<GpuBatch>();
    b->device = dev;
    b->lane = lane;
    b->scatter = !pack;
    b->stream = s;
    if (!pack) {
      ++scattersInFlight;
    }
    if (flag) {
      counters.ticket_batches++;
      b->flag = flag;
      b->ticket = ticket;
    } else {
      b->event = get_event();
      gpu::check(tempi_hip_event_record(b->event, s), "event record");
    }
    if (cur != dev) tempi_hip_set_device(cur);
    for (Op *op : list.ops)
      if (op->device == dev) {
        op->queued = false;
        b->ops.push_back(op);
      }
    batches.push_back(b);
    batch_launched();
  }
  list.clear();
}

void flush() {
  flush_list(pendingPack, true);
  flush_list(pendingUnpack, false);
}

namespace {

struct IsendOp : Op {
  RecordRef rec;      // the type (kept alive: MPI_Type_free may come first)
  const char *origin; // GPU-visible
  int count, dest, tag;
  MPI_Datatype dt;
  MPI_Comm comm;
  Method method;
  int64_t bytes;
  Slab *dslab = nullptr, *hslab = nullptr;
  IpcDesc desc{};

  uint64_t key;

  SendMode mode;

  IsendOp(const TypeRecord *r, const char *o, int c, MPI_Datatype d, int de, int t, MPI_Comm cm, int dev,
          Method m, int64_t b, SendMode md)
      : rec(r->ref()), origin(o), count(c), dest(de), tag(t), dt(d), comm(cm), method(m), bytes(b),
        key(gate_key(cm, de)), mode(md) {
    device = dev;
    if (mode == SendMode::BUFFERED) count_buffered();
    gate_enter(key, this);
    if (method == Method::ONESHOT) {
      hslab = pinned_pool().get(size_t(bytes), device);
      pendingPack.add_items(this, *rec->packer, hslab->dev, origin, count);
    } else {
      dslab = device_pool().get(size_t(bytes), device);
      pendingPack.add_items(this, *rec->packer, dslab->dev, origin, count);
      if (method == Method::STAGED) {
        hslab = pinned_pool().get(size_t(bytes), device);
        pendingPack.stages.push_back({hslab->host, dslab->dev, size_t(bytes), device});
      }
    }
    pendingPack.queue(this);
  }

  void gpu_done() override { // packed: hand it to the library (in order)
    ready = true;
    gate_advance(key);
  }
  // the library refused the send (MPI_Ibsend with too small an attached
  // buffer, ...): the op completes with that error, its slabs released
  void post_failed(int rc) {
    lib = MPI_REQUEST_NULL;
    err = rc;
    errComm = comm;
    lib_done(MPI_Status{});
  }
  void post() override {
    settle_buffered();
    int rc = MPI_SUCCESS;
    switch (method) {
    case Method::ONESHOT:
    case Method::STAGED: rc = lib_isend(mode, hslab->host, int(bytes), MPI_PACKED, dest, tag, comm, &lib); break;
    case Method::DEVICE: rc = lib_isend(mode, dslab->dev, int(bytes), MPI_PACKED, dest, tag, comm, &lib); break;
    case Method::IPC: {
      desc.magic[0] = kMagic0;
      desc.magic[1] = kMagic1;
      desc.slabId = dslab->id;
      desc.offset = 0;
      desc.bytes = bytes;
      desc.senderWorld = state.worldRank;
      desc.senderPid = state.pid;
      desc.rawPtr = reinterpret_cast<uint64_t>(dslab->dev);
      desc.gpu = gpu::identity(device);
      std::memcpy(desc.handle, slab_ipc_handle(dslab), sizeof desc.handle);
      // the slab is reused once the receiver acknowledges: in a board slot,
      // or as a library message on the private communicator (those tags take
      // [board.slots, tagUb/2); IPC COPY's the upper half). The ack's receive
      // is posted after the descriptor's send (the library holds an early ack
      // as an unexpected message), so a refused send leaves nothing behind.
      const int peer = topology::world_rank(comm, dest);
      const int slot = board_take(peer);
      const uint32_t span = uint32_t(std::max(1, tagUb / 2 - board.slots));
      desc.ackTag = slot >= 0 ? slot : board.slots + int32_t(dslab->id % span);
      rc = lib_isend(mode, &desc, int(sizeof desc), MPI_PACKED, dest, tag, comm, &lib);
      if (rc != MPI_SUCCESS) {
        if (slot >= 0) board_give(slot);
        break;
      }
      pendingAcks.push_back(
          std::unique_ptr<PendingAck>(new PendingAck{MPI_REQUEST_NULL, dslab, peer, desc.ackTag, bytes, -1, slot >= 0}));
      PendingAck &pa = *pendingAcks.back();
      if (slot < 0) next.MPI_Irecv(&pa.code, 1, MPI_INT, peer, desc.ackTag, ctrlComm, &pa.req);
      dslab = nullptr;
      break;
    }
    default:
      return;
    }
    if (rc != MPI_SUCCESS)
      post_failed(rc);
    else
      watch(this);
  }
  void lib_done(const MPI_Status &) override {
    if (dslab) device_pool().put(dslab);
    if (hslab) pinned_pool().put(hslab);
    dslab = hslab = nullptr;
    done = true;
  }
  void status(MPI_Status *s) const override {
    if (s != MPI_STATUS_IGNORE) {
      s->MPI_SOURCE = MPI_ANY_SOURCE;
      s->MPI_TAG = MPI_ANY_TAG;
      s->MPI_ERROR = err;
      MPI_Status_set_elements(s, MPI_BYTE, 0);
    }
  }
};

struct IsendDirectOp : Op {
  RecordRef rec;
  const char *origin;
  int count;
  MPI_Datatype dt;
  int64_t bytes;
  std::shared_ptr<DirectShared> sh;
  bool packDone = false;

  IsendDirectOp(const TypeRecord *r, const char *o, int c, MPI_Datatype d, int dest, int tag, MPI_Comm comm,
                int dev, int64_t b, const tempi_hip_desc &flat)
      : rec(r->ref()), origin(o), count(c), dt(d), bytes(b) {
    device = dev;
    sh = std::allocate_shared<DirectShared>(std::pmr::polymorphic_allocator<DirectShared>(&op_pool()));
    sh->device = dev;
    sh->sender = this;
    const uint64_t token = nextDirectToken++;
    DirectDesc &desc = sh->desc;
    desc.magic[0] = kMagicDirect;
    desc.magic[1] = kMagic1;
    desc.token = token;
    desc.bytes = b;
    desc.senderWorld = state.worldRank;
    desc.senderPid = state.pid;
    desc.device = dev;
    desc.first = reinterpret_cast<uint64_t>(o + rec->desc.start);
    desc.desc = flat;
    this->dest = dest;
    this->tag = tag;
    this->comm = comm;
    post_or_queue(gate_key(comm, dest), this);
  }
  int dest, tag;
  MPI_Comm comm;
  void post() override {
    if (self_send(sh, comm, tag)) {
      maybe_done();
      return;
    }
    directShared[sh->desc.token] = sh; // claimed by the receive that matches the descriptor
    // the library may hold a send to this same process open until its
    // receive is posted (MPICH does), so the send's completion cannot wait for
    // it: the request is released now and the descriptor outlives it in `sh`
    MPI_Request sreq;
    const int rc = next.MPI_Isend(&sh->desc, int(sizeof sh->desc), MPI_PACKED, dest, tag, comm, &sreq);
    if (rc != MPI_SUCCESS) {
      directShared.erase(sh->desc.token);
      return fail_post(this, rc, comm);
    }
    next.MPI_Request_free(&sreq);
    maybe_done();
  }
  ~IsendDirectOp() override {
    if (sh) sh->sender = nullptr;
  }
  void maybe_done() {
    done = posted && (sh->state == DirectShared::DONE || (sh->state == DirectShared::PACKED && packDone));
  }
  void gpu_done() override {
    packDone = true;
    sh->gathered = true;
    maybe_done();
  }
  void peer_done() override { maybe_done(); }
  void stalled() override {
    if (sh->state != DirectShared::PENDING) return;
    // waited on before its receive exists: gather into a slab the receiver
    // will unpack, so the send can complete on its own
    counters.direct_fallbacks++;
    gather();
  }
  void gather() {
    sh->state = DirectShared::PACKED;
    sh->slab = device_pool().get(size_t(bytes), device);
    pendingPack.add_items(this, *rec->packer, sh->slab->dev, origin, count);
    pendingPack.queue(this);
  }
  void status(MPI_Status *s) const override {
    if (s != MPI_STATUS_IGNORE) {
      s->MPI_SOURCE = MPI_ANY_SOURCE;
      s->MPI_TAG = MPI_ANY_TAG;
      s->MPI_ERROR = err; // set by fail_post when the library refused the post
      MPI_Status_set_elements(s, MPI_BYTE, 0);
    }
  }
};

// IPC COPY sender: posts the descriptor, then waits for the receiver's ack
// (its copy out of this process's memory has run). A NACK (the receiver
// cannot copy this shape, or cannot map the memory) is answered by gathering
// the object into pinned host memory here and sending those bytes on
// (ctrlComm, ackTag), where the receiver has already posted for them.
struct IsendCopyOp : Op {
  RecordRef rec;
  const char *origin; // GPU-visible
  int count, dest, tag, peer;
  MPI_Datatype dt;
  MPI_Comm comm;
  int64_t bytes;
  IpcCopyDesc desc{};
  int ack = -1;

  uint64_t key;

  IsendCopyOp(const TypeRecord *r, const char *o, int c, MPI_Datatype d, int de, int t, MPI_Comm cm, int dev,
              int64_t b, int peerWorld, const IpcCopyDesc &filled)
      : rec(r->ref()), origin(o), count(c), dest(de), tag(t), peer(peerWorld), dt(d), comm(cm), bytes(b),
        desc(filled), key(gate_key(cm, de)) {
    device = dev;
    // The application's last writes to the object may still sit in this
    // GPU's L2, invisible to a reader on another GPU. The descriptor leaves
    // only after a batch event (a system-scope release: the L2 is written
    // back) has completed -- an empty batch on lane 0, queued like a gather.
    gate_enter(key, this);
    pendingPack.queue(this);
  }
  void gpu_done() override {
    ready = true;
    gate_advance(key);
  }
  // With a board slot the library request is the descriptor's send (tested
  // until it is delivered, which keeps the library progressing it) and the
  // ack arrives on the board; the send completes once both have. Otherwise
  // the library request is the ack's receive, and the descriptor's send is
  // freed (the ack follows its delivery).
  bool boardAck = false, descSent = false;
  void post() override {
    const int slot = board_take(peer);
    if (slot >= 0) {
      desc.ackTag = slot;
      boardSlot = slot;
      const int rc = next.MPI_Isend(&desc, int(sizeof desc), MPI_PACKED, dest, tag, comm, &lib);
      if (rc != MPI_SUCCESS) {
        board_give(slot);
        boardSlot = -1;
        return fail_post(this, rc, comm);
      }
      boardAck = true;
      boardOps.push_back(this);
      watch(this);
      return;
    }
    MPI_Request r; // the descriptor lives in this op until the ack, which follows its delivery
    const int rc = next.MPI_Isend(&desc, int(sizeof desc), MPI_PACKED, dest, tag, comm, &r);
    if (rc != MPI_SUCCESS) return fail_post(this, rc, comm);
    next.MPI_Irecv(&ack, 1, MPI_INT, peer, desc.ackTag, ctrlComm, &lib); // (the ack follows the delivery)
    watch(this);
    next.MPI_Request_free(&r);
  }
  void lib_done(const MPI_Status &) override {
    if (boardAck) {
      descSent = true;
      if (ack >= 0 && !done) finish();
      return;
    }
    finish();
  }
  void acked(int code) override {
    ack = code;
    // the receiver has the descriptor, so the library is done with this
    // op's copy of it: a send still under test is let go (its completion may
    // also be recorded already, with the callback still to come)
    if (!descSent && lib != MPI_REQUEST_NULL) {
      unwatch(this);
      next.MPI_Request_free(&lib);
    }
    descSent = true;
    finish();
  }
  void finish() {
    if (ack != kCopyDone) {
      if (ack == kCopyUnmapped) mark_ipc_broken(peer);
      counters.copy_resends++;
      Slab *h = pinned_pool().get(size_t(std::max<int64_t>(bytes, 1)), device);
      void *s = gpu::stream(device);
      int cur = 0;
      tempi_hip_get_device(&cur);
      if (cur != device) tempi_hip_set_device(device);
      gpu::check(rec->packer->pack_async(h->dev, origin, count, s), "ipc copy fallback gather");
      gpu::check(tempi_hip_stream_synchronize(s), "ipc copy fallback sync");
      if (cur != device) tempi_hip_set_device(cur);
      next.MPI_Send(h->host, int(bytes), MPI_PACKED, peer, desc.ackTag, ctrlComm); // receive already posted
      pinned_pool().put(h);
    }
    done = true;
  }
  void status(MPI_Status *s) const override {
    if (s != MPI_STATUS_IGNORE) {
      s->MPI_SOURCE = MPI_ANY_SOURCE;
      s->MPI_TAG = MPI_ANY_TAG;
      s->MPI_ERROR = err; // set by fail_post when the library refused the post
      MPI_Status_set_elements(s, MPI_BYTE, 0);
    }
  }
};

// library-packed transfer of a device buffer whose type TEMPI cannot pack
// (the touched span is staged through host memory by tempi::pack / unpack)
struct LibIsendOp : Op {
  std::vector<char> buf;
  MPI_Datatype dt;
  int n = 0, dest, tag;
  MPI_Comm comm;
  SendMode mode;
  LibIsendOp(const void *b, int c, MPI_Datatype d, int de, int t, MPI_Comm cm, SendMode md)
      : dt(d), dest(de), tag(t), comm(cm), mode(md) {
    buf.resize(size_t(std::max<int64_t>(pack_size(c, d, comm), 1)));
    tempi::pack(b, c, d, buf.data(), int(buf.size()), &n, comm);
    if (mode == SendMode::BUFFERED) count_buffered();
    post_or_queue(gate_key(comm, dest), this);
  }
  void post() override {
    settle_buffered();
    const int rc = lib_isend(mode, buf.data(), n, MPI_PACKED, dest, tag, comm, &lib);
    if (rc == MPI_SUCCESS) {
      watch(this);
      return;
    }
    lib = MPI_REQUEST_NULL;
    err = rc;
    errComm = comm;
    done = true;
  }
  void lib_done(const MPI_Status &) override { done = true; }
  void status(MPI_Status *s) const override {
    if (s != MPI_STATUS_IGNORE) {
      s->MPI_ERROR = err;
      MPI_Status_set_elements(s, MPI_BYTE, 0);
    }
  }
};

// a host-buffer send queued behind a gathering send to the same peer
struct HostIsendOp : Op {
  const void *buf;
  int count, dest, tag;
  MPI_Datatype dt;
  MPI_Comm comm;
  HostIsendOp(const void *b, int c, MPI_Datatype d, int de, int t, MPI_Comm cm)
      : buf(b), count(c), dest(de), tag(t), dt(hold_type(d)), comm(cm) {
    ready = true;
    gate_enter(gate_key(comm, dest), this);
  }
  ~HostIsendOp() override { drop_type(dt); }
  void post() override {
    const int rc = next.MPI_Isend(buf, count, dt, dest, tag, comm, &lib);
    if (rc != MPI_SUCCESS) return fail_post(this, rc, comm);
    watch(this);
  }
  void lib_done(const MPI_Status &) override { done = true; }
  void status(MPI_Status *s) const override {
    if (s != MPI_STATUS_IGNORE) {
      s->MPI_ERROR = err; // set by fail_post when the library refused the post
      MPI_Status_set_elements(s, MPI_BYTE, 0);
    }
  }
};

// self edges of a collective: the copies alone, one request for all of
// them (see p2p::local_copy, p2p::start_local_copies)
struct LocalCopyOp : Op {
  std::vector<RecordRef> recs;
  int64_t bytes;
  explicit LocalCopyOp(const LocalCopies &plan) : recs(plan.recs), bytes(plan.bytes) {
    device = plan.device;
    for (const tempi_hip_copy_item &c : plan.items) pendingUnpack.add_copy(this, c);
    pendingUnpack.queue(this);
  }
  void gpu_done() override { done = true; }
  void status(MPI_Status *s) const override {
    if (s != MPI_STATUS_IGNORE) {
      s->MPI_SOURCE = state.worldRank;
      s->MPI_TAG = MPI_ANY_TAG;
      s->MPI_ERROR = err; // set by fail_post when the library refused the post
      set_received(s, bytes);
    }
  }
};

} // namespace

std::unique_ptr<Op> new_isend(const TypeRecord *r, const char *origin, int count, MPI_Datatype dt, int dest, int tag,
                              MPI_Comm comm, int dev, Method m, int64_t bytes, SendMode mode) {
  return std::make_unique<IsendOp>(r, origin, count, dt, dest, tag, comm, dev, m, bytes, mode);
}
std::unique_ptr<Op> new_isend_direct(const TypeRecord *r, const char *origin, int count, MPI_Datatype dt, int dest,
                                     int tag, MPI_Comm comm, int dev, int64_t bytes, const tempi_hip_desc &flat) {
  return std::make_unique<IsendDirectOp>(r, origin, count, dt, dest, tag, comm, dev, bytes, flat);
}
std::unique_ptr<Op> new_isend_copy(const TypeRecord *r, const char *origin, int count, MPI_Datatype dt, int dest,
                                   int tag, MPI_Comm comm, int dev, int64_t bytes, int peerWorld,
                                   const IpcCopyDesc &filled) {
  return std::make_unique<IsendCopyOp>(r, origin, count, dt, dest, tag, comm, dev, bytes, peerWorld, filled);
}
std::unique_ptr<Op> new_lib_isend(const void *buf, int count, MPI_Datatype dt, int dest, int tag, MPI_Comm comm,
                                  SendMode mode) {
  return std::make_unique<LibIsendOp>(buf, count, dt, dest, tag, comm, mode);
}

int lib_isend(SendMode mode, const void *buf, int count, MPI_Datatype dt, int dest, int tag, MPI_Comm comm,
              MPI_Request *req) {
  switch (mode) {
  case SendMode::SYNC: return next.MPI_Issend(buf, count, dt, dest, tag, comm, req);
  case SendMode::BUFFERED: return next.MPI_Ibsend(buf, count, dt, dest, tag, comm, req);
  default: return next.MPI_Isend(buf, count, dt, dest, tag, comm, req);
  }
}
std::unique_ptr<Op> new_host_isend(const void *buf, int count, MPI_Datatype dt, int dest, int tag, MPI_Comm comm) {
  return std::make_unique<HostIsendOp>(buf, count, dt, dest, tag, comm);
}
std::unique_ptr<Op> new_local_copies(const LocalCopies &plan) { return std::make_unique<LocalCopyOp>(plan); }

} // namespace detail
} // namespace p2p
} // namespace tempi
