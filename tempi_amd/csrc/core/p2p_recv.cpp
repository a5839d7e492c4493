// tempi_amd/csrc/core/p2p_recv.cpp -- the receive state machines and the
// self channel (p2p_internal.hpp)
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

bool selfChannelEnabled = true;

namespace {

struct IrecvOp;
bool self_recv(IrecvOp *r, int source, int tag); // the self channel took this receive

struct IrecvOp : Op {
  RecordRef rec;
  char *origin; // GPU-visible
  int count;
  MPI_Datatype dt;
  MPI_Comm comm;
  int64_t bytes;
  Slab *hslab = nullptr;
  MPI_Status libStatus{};
  IpcDesc desc{};
  bool ipc = false;
  bool fallback = false; // waiting for the bytes the peer re-sends through the host
  int64_t elems = 0;
  std::shared_ptr<DirectShared> direct; // a same-process send being copied / unpacked
  bool arrived = false;   // the library receive matched
  bool cancelled = false; // MPI_Cancel took effect
  bool xcopy = false;     // an IPC COPY out of the sender's memory: ack it when done
  int copyWorld = -1, copyTag = 0;
  bool selfPending = false; // waiting in the self channel (no library receive posted)
  int selfSource = 0, selfTag = 0;

  // msg: receive this library message (MPI_Mrecv); pre: a message a probe
  // already received (it is delivered at once)
  IrecvOp(const TypeRecord *r, char *o, int c, MPI_Datatype d, int source, int tag, MPI_Comm cm, int dev,
          int64_t b, MPI_Message *msg = nullptr, std::unique_ptr<Probed> pre = nullptr)
      : rec(r->ref()), origin(o), count(c), dt(d), comm(cm), bytes(b) {
    device = dev;
    errComm = cm;
    // from this same process: matched inside TEMPI when the channel allows
    if (!msg && !pre && source >= 0 && self_recv(this, source, tag)) return;
    const size_t cap = std::max<size_t>(size_t(bytes), kDescCap);
    hslab = pinned_pool().get(cap, device);
    if (pre) {
      std::memcpy(hslab->host, pre->bytes.data(), std::min(cap, pre->bytes.size()));
      lib_done(pre->st);
      return;
    }
    const int rc = msg ? next.MPI_Imrecv(hslab->host, int(cap), MPI_PACKED, msg, &lib)
                       : next.MPI_Irecv(hslab->host, int(cap), MPI_PACKED, source, tag, comm, &lib);
    if (rc != MPI_SUCCESS) {
      pinned_pool().put(hslab);
      hslab = nullptr;
      fail_post(this, rc, comm);
      return;
    }
    // a message from this same process is matched as the receive is posted:
    // take it now, so its copy can start while the caller posts more
    if (!msg && source >= 0 && topology::world_rank(comm, source) == state.worldRank) {
      int flag = 0;
      MPI_Status st;
      next.MPI_Test(&lib, &flag, &st);
      if (flag) {
        lib = MPI_REQUEST_NULL;
        st.MPI_ERROR = MPI_SUCCESS; // (MPI_Test leaves it unset)
        lib_done(st);
      }
    }
    watch(this);
  }

  // (the self channel spills) post the library receive this op skipped
  void post_library() {
    selfPending = false;
    const size_t cap = std::max<size_t>(size_t(bytes), kDescCap);
    hslab = pinned_pool().get(cap, device);
    next.MPI_Irecv(hslab->host, int(cap), MPI_PACKED, selfSource, selfTag, comm, &lib);
    watch(this);
  }
  // a direct send of this process, matched by the self channel
  void take_self(const std::shared_ptr<DirectShared> &sh, int tag, int sourceRank) {
    selfPending = false;
    arrived = true;
    libStatus = MPI_Status{};
    libStatus.MPI_SOURCE = sourceRank;
    libStatus.MPI_TAG = tag;
    libStatus.MPI_ERROR = MPI_SUCCESS;
    counters.self_matched++;
    on_direct(sh);
  }
  void cancel() override;
  // the message is larger than the receive allows: the wait returns
  // MPI_ERR_TRUNCATE (on the communicator's error handler); nothing is
  // written, and the sender has already been released
  void truncate(int64_t got) {
    LOG_DEBUG("message truncated: " << got << " B into " << bytes);
    err = MPI_ERR_TRUNCATE;
    elems = 0;
    pinned_pool().put(hslab);
    hslab = nullptr;
    done = true;
  }
  void lib_done(const MPI_Status &st) override { // arrived: queue its unpack
    const Packer &packer = *rec->packer;
    if (!arrived) {
      int c = 0;
      MPI_Test_cancelled(&st, &c);
      if (c) {
        cancelled = done = true;
        libStatus = st;
        pinned_pool().put(hslab);
        hslab = nullptr;
        return;
      }
      if (st.MPI_ERROR != MPI_SUCCESS) { // the library's own error (e.g. its truncation)
        libStatus = st;
        err = st.MPI_ERROR;
        pinned_pool().put(hslab);
        hslab = nullptr;
        done = true;
        return;
      }
    }
    arrived = true;
    if (fallback) { // the host copy of an IPC message we could not map
      elems = packer.desc().size ? desc.bytes / packer.desc().size : 0;
      pendingUnpack.add_items(this, packer, hslab->dev, origin, elems);
      pendingUnpack.queue(this);
      return;
    }
    libStatus = st;
    int n = 0;
    MPI_Get_count(&libStatus, MPI_PACKED, &n);
    IpcDesc d;
    std::memcpy(&d, hslab->host, std::min<size_t>(sizeof d, size_t(n)));
    if (is_direct(hslab->host, n)) {
      DirectDesc dd;
      std::memcpy(&dd, hslab->host, sizeof dd);
      return on_direct(claim_direct(dd));
    }
    lib_done_rest(n, d);
  }
  // a direct send's bytes (its descriptor came through the library, or the
  // self channel handed it over): one copy kernel when it can, else the
  // sender's gather unpacked, else the bytes fetched through the host
  void on_direct(std::shared_ptr<DirectShared> sh) {
    const Packer &packer = *rec->packer;
    const int64_t size = packer.desc().size;
    direct = std::move(sh);
    const DirectDesc &dd = direct->desc;
    {
      if (dd.bytes > bytes) {
        const int64_t got = dd.bytes;
        direct_finish(direct);
        return truncate(got);
      }
      elems = size ? dd.bytes / size : 0;
      const bool sameDevice = direct->device == device;
      tempi_hip_desc mine;
      char *first = origin + packer.desc().start;
      if (direct->state == DirectShared::PENDING && sameDevice && elems * size == dd.bytes &&
          rec->flat(elems, &mine) && copy_ok(mine, dd.desc)) {
        direct->state = DirectShared::CLAIMED;
        tempi_hip_copy_item c{};
        c.dst_first = first;
        c.src_first = reinterpret_cast<const void *>(dd.first);
        c.dst = mine;
        c.src = dd.desc;
        pendingUnpack.add_copy(this, c);
      } else if (direct->state == DirectShared::PACKED && sameDevice) {
        // the sender's gather runs on lane 0: so does this scatter, after it
        // (unless that gather is already seen complete)
        pendingUnpack.add_items(this, packer, direct->slab->dev, origin, elems);
        if (!direct->gathered) pendingUnpack.afterPack = true;
      } else { // another device, or a shape the copy kernel does not take
        if (!hslab) hslab = pinned_pool().get(std::max<size_t>(size_t(bytes), kDescCap), device);
        const DirectDesc copy = dd; // (materialise_direct releases the shared state)
        materialise_direct(direct, copy, hslab);
        pendingUnpack.add_items(this, packer, hslab->dev, origin, elems);
      }
      pendingUnpack.queue(this);
    }
  }
  void lib_done_rest(int n, const IpcDesc &d) {
    const Packer &packer = *rec->packer;
    const int64_t size = packer.desc().size;
    if (is_ipc_copy(hslab->host, n)) {
      IpcCopyDesc xd;
      std::memcpy(&xd, hslab->host, sizeof xd);
      if (xd.bytes > bytes) {
        send_ack(xd.senderWorld, xd.ackTag, kCopyDone);
        return truncate(xd.bytes);
      }
      elems = size ? xd.bytes / size : 0;
      const bool local = xd.senderPid == state.pid;
      if (!local) recycle_alloc_maps();
      const char *src = (local && xd.device != device) ? nullptr : peer_object(xd);
      if (src && !local && xd.gpu != gpu::identity(device) &&
          !canary(xd.senderWorld, src, std::min(xd.desc.block, xd.bytes), device))
        src = nullptr; // (the peer is now marked: the NACK below says so)
      tempi_hip_desc mine;
      if (src && elems * size == xd.bytes && rec->flat(elems, &mine) && copy_ok(mine, xd.desc)) {
        xcopy = true;
        copyWorld = xd.senderWorld;
        copyTag = xd.ackTag;
        tempi_hip_copy_item c{};
        c.dst_first = origin + packer.desc().start;
        c.src_first = src;
        c.dst = mine;
        c.src = xd.desc;
        // another GPU's memory, reused by its owner between messages: read it
        // with system-scope loads. (Memory of this same GPU is read through
        // its own L2, which holds the sender's latest writes: measured, the
        // system-scope loads could return stale bytes there.)
        if (!local && xd.gpu != gpu::identity(device)) c.flags = TEMPI_HIP_ITEM_REMOTE;
        pendingUnpack.add_copy(this, c);
        pendingUnpack.queue(this);
        return;
      }
      // a shape the copy kernel does not take, or memory we cannot map: the
      // sender gathers and sends the bytes through the host
      fallback = true;
      desc.bytes = xd.bytes;
      next.MPI_Irecv(hslab->host, int(xd.bytes), MPI_PACKED, xd.senderWorld, xd.ackTag, ctrlComm, &lib);
      watch(this);
      send_ack(xd.senderWorld, xd.ackTag, (src || local) ? kCopyResend : kCopyUnmapped);
      return;
    }
    if (size_t(n) == sizeof(IpcDesc) && d.magic[0] == kMagic0 && d.magic[1] == kMagic1) {
      ipc = true;
      desc = d;
      if (d.bytes > bytes) {
        send_ack(d);
        return truncate(d.bytes);
      }
      void *base = peer_pointer(d);
      if (base && d.senderPid != state.pid && d.gpu != gpu::identity(device) &&
          !canary(d.senderWorld, static_cast<const char *>(base) + d.offset, d.bytes, device))
        base = nullptr;
      if (!base) { // cannot map (or trust) the sender's slab: ask for the bytes via the host
        ipc = false;
        fallback = true;
        next.MPI_Irecv(hslab->host, int(d.bytes), MPI_PACKED, d.senderWorld, d.ackTag, ctrlComm, &lib);
        watch(this);
        send_ack(d, 1);
        return;
      }
      const char *peer = static_cast<const char *>(base) + d.offset;
      elems = size ? d.bytes / size : 0;
      const size_t first = pendingUnpack.items.size();
      pendingUnpack.add_items(this, packer, const_cast<char *>(peer), origin, elems);
      if (d.gpu != gpu::identity(device)) // another GPU's slab, reused between messages
        for (size_t i = first; i < pendingUnpack.items.size(); ++i) pendingUnpack.items[i].flags |= TEMPI_HIP_ITEM_REMOTE;
    } else {
      if (int64_t(n) > bytes) return truncate(n);
      elems = size ? n / size : 0;
      pendingUnpack.add_items(this, packer, hslab->dev, origin, elems);
    }
    pendingUnpack.queue(this);
  }
  void gpu_done() override {
    if (ipc) send_ack(desc);
    if (xcopy) send_ack(copyWorld, copyTag, kCopyDone);
    direct_finish(direct);
    pinned_pool().put(hslab);
    hslab = nullptr;
    done = true;
  }
  void status(MPI_Status *s) const override {
    if (s != MPI_STATUS_IGNORE) {
      *s = libStatus;
      s->MPI_ERROR = err;
      set_received(s, elems * rec->desc.size);
      if (cancelled) MPI_Status_set_cancelled(s, 1);
    }
  }
};

// ------------------------------------------------------------- self channel
//
// Messages a process sends to itself on a communicator (every neighbour of a
// one-rank halo, the x and y faces at two ranks) are matched inside TEMPI:
// a direct send is queued per communicator and a device receive from the same
// rank takes the earliest one whose tag matches (or waits, in post order, for
// the next). No descriptor, library message, pinned slab or library test per
// message -- on the one-rank 512^3 halo these were ~0.55 us of the ~1 us of
// host time each of its 624 messages per iteration cost.
//
// MPI matching stays exact because the channel of a communicator carries
// either ALL of its self-traffic or none: the first self-message operation
// the channel cannot carry (a send to this rank that is not a direct send --
// host buffer, blocking, library-packed -- a receive from this rank or from
// MPI_ANY_SOURCE into anything but a TEMPI device receive, a probe of this
// rank or of any source, a send mode TEMPI does not carry (MPI_Ssend ...))
// SPILLS it: the receives it holds are posted to the library in post order,
// the sends it holds are posted as descriptors in send order (none of them
// matches any of those receives, or they would have been paired), and the
// communicator's self-traffic goes through the library from then on.
// TEMPI_NO_SELF_CHANNEL turns it off.
struct SelfSend {
  std::shared_ptr<DirectShared> sh;
  int tag;
};
struct SelfChannel {
  bool spilled = false;
  int myRank = 0; // this process's rank in the communicator
  std::deque<SelfSend> sends;  // unmatched, send order
  std::deque<IrecvOp *> recvs; // unmatched, post order
};
std::unordered_map<uint64_t, SelfChannel> selfChannels;

uint64_t comm_key(MPI_Comm c) {
  uint64_t k = 0;
  std::memcpy(&k, &c, std::min(sizeof c, sizeof k));
  return k;
}

SelfChannel &self_channel(MPI_Comm comm) {
  auto it = selfChannels.find(comm_key(comm));
  if (it != selfChannels.end()) return it->second;
  SelfChannel &ch = selfChannels[comm_key(comm)];
  next.MPI_Comm_rank(comm, &ch.myRank);
  return ch;
}

bool tags_match(int want, int got) { return want == MPI_ANY_TAG || want == got; }

bool self_recv(IrecvOp *r, int source, int tag) {
  if (!selfChannelEnabled || topology::world_rank(r->comm, source) != state.worldRank) return false;
  SelfChannel &ch = self_channel(r->comm);
  if (ch.spilled) return false;
  r->selfSource = source;
  r->selfTag = tag;
  for (auto it = ch.sends.begin(); it != ch.sends.end(); ++it)
    if (tags_match(tag, it->tag)) {
      SelfSend e = std::move(*it);
      ch.sends.erase(it);
      r->take_self(e.sh, e.tag, ch.myRank);
      return true;
    }
  r->selfPending = true;
  ch.recvs.push_back(r);
  return true;
}

void IrecvOp::cancel() {
  if (selfPending) { // nothing matched it yet: drop it from the channel
    SelfChannel &ch = self_channel(comm);
    ch.recvs.erase(std::remove(ch.recvs.begin(), ch.recvs.end(), this), ch.recvs.end());
    selfPending = false;
    cancelled = done = true;
    return;
  }
  if (!arrived && lib != MPI_REQUEST_NULL) next.MPI_Cancel(&lib);
}

struct LibIrecvOp : Op {
  std::vector<char> buf;
  void *user;
  int count;
  MPI_Datatype dt;
  MPI_Comm comm;
  MPI_Status libStatus{};
  int64_t cap = 0; // packed bytes the receive allows
  int elems = 0;
  int received = 0; // bytes
  LibIrecvOp(void *b, int c, MPI_Datatype d, int source, int tag, MPI_Comm cm, MPI_Message *msg = nullptr,
             std::unique_ptr<Probed> pre = nullptr)
      : user(b), count(c), dt(hold_type(d)), comm(cm) {
    errComm = cm;
    cap = pack_size(c, d, cm);
    buf.resize(std::max<size_t>(size_t(std::max<int64_t>(cap, 1)), kDescCap));
    if (pre) {
      std::memcpy(buf.data(), pre->bytes.data(), std::min(buf.size(), pre->bytes.size()));
      lib_done(pre->st);
      return;
    }
    const int rc = msg ? next.MPI_Imrecv(buf.data(), int(buf.size()), MPI_PACKED, msg, &lib)
                       : next.MPI_Irecv(buf.data(), int(buf.size()), MPI_PACKED, source, tag, comm, &lib);
    if (rc != MPI_SUCCESS) {
      fail_post(this, rc, comm);
      return;
    }
    watch(this);
  }
  bool cancelled = false;
  void cancel() override {
    if (lib != MPI_REQUEST_NULL) next.MPI_Cancel(&lib);
  }
  void lib_done(const MPI_Status &st) override {
    libStatus = st;
    int c = 0;
    MPI_Test_cancelled(&st, &c);
    if (c) {
      cancelled = done = true;
      return;
    }
    if (st.MPI_ERROR != MPI_SUCCESS) { // the library's own error (e.g. its truncation)
      err = st.MPI_ERROR;
      done = true;
      return;
    }
    int n = 0, size = 0;
    MPI_Get_count(&libStatus, MPI_PACKED, &n);
    if (is_descriptor(buf.data(), n)) { // a TEMPI descriptor
      std::vector<char> bytes;
      land_descriptor(buf.data(), n, bytes);
      buf.swap(bytes);
      n = int(buf.size());
    }
    if (int64_t(n) > cap) { // larger than the receive allows: nothing written
      err = MPI_ERR_TRUNCATE;
      done = true;
      return;
    }
    MPI_Type_size(dt, &size);
    elems = size ? n / size : 0;
    received = elems * size;
    int pos = 0;
    tempi::unpack(buf.data(), n, &pos, user, elems, dt, comm);
    done = true;
  }
  ~LibIrecvOp() override { drop_type(dt); }
  void status(MPI_Status *s) const override {
    if (s != MPI_STATUS_IGNORE) {
      *s = libStatus;
      s->MPI_ERROR = err;
      set_received(s, received);
      if (cancelled) MPI_Status_set_cancelled(s, 1);
    }
  }
};

// Staging buffers of host receives, reused: a fresh buffer per receive costs
// its zeroing (std::vector) or its first-touch page faults (new[]) on every
// message, which on the host-buffer halo was most of TEMPI's overhead over
// the library (tools/gpu_host_ab.sh). Power-of-two classes from 4 KiB; at
// most kStageCache bytes kept.
class StagePool {
public:
  struct Buf {
    char *p = nullptr;
    size_t cap = 0;
  };
  Buf get(size_t n) {
    int c = 12;
    while ((size_t(1) << c) < n) ++c;
    auto &l = free_[size_t(c)];
    Buf b;
    if (!l.empty()) {
      b = l.back();
      l.pop_back();
      held_ -= b.cap;
      return b;
    }
    b.cap = size_t(1) << c;
    b.p = new char[b.cap];
    return b;
  }
  void put(Buf b) {
    if (!b.p) return;
    if (held_ + b.cap > kStageCache) {
      delete[] b.p;
      return;
    }
    int c = 12;
    while ((size_t(1) << c) < b.cap) ++c;
    free_[size_t(c)].push_back(b);
    held_ += b.cap;
  }

private:
  static constexpr size_t kStageCache = size_t(256) << 20;
  std::vector<Buf> free_[64];
  size_t held_ = 0;
};
StagePool &stage_pool() {
  static auto *p = new StagePool(); // (never destroyed: ops may outlive statics)
  return *p;
}

// A receive into host memory (p2p::irecv_host) that a co-located TEMPI send
// may reach with a descriptor. Contiguous receives of at least kDescCap bytes
// are posted in place with the buffer's first kDescCap bytes saved: a
// descriptor that lands there is recognised (size + magic), the saved bytes
// are put back and what it names is fetched and copied in. Other receives
// land in a staging buffer as MPI_PACKED and are unpacked from it.
struct HostIrecvOp : Op {
  void *user;
  int count;
  MPI_Datatype dt = MPI_DATATYPE_NULL; // held for staged receives (unpacked with it)
  MPI_Comm comm;
  int64_t cap = 0; // bytes the receive allows
  bool inPlace = false;
  StagePool::Buf stage;
  alignas(16) char saved[kDescCap];
  MPI_Status libStatus{};
  int64_t received = 0;
  bool cancelled = false;

  HostIrecvOp(void *b, int c, MPI_Datatype d, int source, int tag, MPI_Comm cm, std::unique_ptr<Probed> pre)
      : user(b), count(c), comm(cm) {
    errComm = cm;
    int size = 0;
    MPI_Type_size(d, &size);
    cap = int64_t(size) * c;
    MPI_Aint lb = 0, ext = 0, tlb = 0, text = 0;
    MPI_Type_get_extent(d, &lb, &ext);
    MPI_Type_get_true_extent(d, &tlb, &text);
    inPlace = !pre && tlb == 0 && text == size && (c == 1 || ext == size) && cap >= int64_t(kDescCap);
    if (inPlace) {
      std::memcpy(saved, b, kDescCap);
      const int rc = next.MPI_Irecv(b, c, d, source, tag, cm, &lib);
      if (rc != MPI_SUCCESS) {
        fail_post(this, rc, cm);
        return;
      }
      watch(this);
      return;
    }
    dt = hold_type(d);
    if (pre) {
      libStatus = pre->st;
      deliver(pre->bytes.data(), int(pre->bytes.size()));
      return;
    }
    const size_t n = std::max({size_t(std::max<int64_t>(cap, 1)), size_t(pack_size(c, d, cm)), kDescCap});
    stage = stage_pool().get(n);
    const int rc = next.MPI_Irecv(stage.p, int(n), MPI_PACKED, source, tag, cm, &lib);
    if (rc != MPI_SUCCESS) {
      fail_post(this, rc, cm);
      return;
    }
    watch(this);
  }
  ~HostIrecvOp() override {
    drop_type(dt);
    if (lib == MPI_REQUEST_NULL) stage_pool().put(stage); // (else the library may still write it: kept)
  }
  void cancel() override {
    if (lib != MPI_REQUEST_NULL) next.MPI_Cancel(&lib);
  }
  void deliver(const char *msg, int n) {
    err = land_host(msg, n, user, count, dt, comm, &received);
    done = true;
    if (msg == stage.p) {
      stage_pool().put(stage);
      stage = StagePool::Buf();
    }
  }
  void lib_done(const MPI_Status &st) override {
    libStatus = st;
    int c = 0;
    MPI_Test_cancelled(&st, &c);
    if (c || st.MPI_ERROR != MPI_SUCCESS) {
      cancelled = c;
      err = c ? MPI_SUCCESS : st.MPI_ERROR;
      done = true;
      return;
    }
    int n = 0;
    MPI_Get_count(&st, MPI_BYTE, &n);
    if (!inPlace) return deliver(stage.p, n);
    received = n;
    if (is_descriptor(user, n)) {
      alignas(16) char raw[kDescCap];
      std::memcpy(raw, user, size_t(n));
      std::memcpy(user, saved, size_t(n)); // the application's bytes under the descriptor
      std::vector<char> fetched;
      land_descriptor(raw, n, fetched);
      received = 0;
      if (int64_t(fetched.size()) > cap) {
        err = MPI_ERR_TRUNCATE;
      } else {
        std::memcpy(user, fetched.data(), fetched.size());
        received = int64_t(fetched.size());
      }
    }
    done = true;
  }
  void status(MPI_Status *s) const override {
    if (s != MPI_STATUS_IGNORE) {
      *s = libStatus;
      s->MPI_ERROR = err;
      set_received(s, received);
      if (cancelled) MPI_Status_set_cancelled(s, 1);
    }
  }
};

} // namespace

void spill_channel(MPI_Comm comm) {
  SelfChannel &ch = self_channel(comm);
  if (ch.spilled) return;
  ch.spilled = true;
  if (!ch.recvs.empty() || !ch.sends.empty())
    LOG_DEBUG("self channel spills " << ch.recvs.size() << " receive(s), " << ch.sends.size() << " send(s)");
  for (IrecvOp *r : ch.recvs) r->post_library();
  ch.recvs.clear();
  for (SelfSend &e : ch.sends) {
    directShared[e.sh->desc.token] = e.sh;
    MPI_Request r;
    next.MPI_Isend(&e.sh->desc, int(sizeof e.sh->desc), MPI_PACKED, ch.myRank, e.tag, comm, &r);
    next.MPI_Request_free(&r);
  }
  ch.sends.clear();
}

bool self_send(const std::shared_ptr<DirectShared> &sh, MPI_Comm comm, int tag) {
  if (!selfChannelEnabled) return false;
  SelfChannel &ch = self_channel(comm);
  if (ch.spilled) return false;
  for (auto it = ch.recvs.begin(); it != ch.recvs.end(); ++it)
    if (tags_match((*it)->selfTag, tag)) {
      IrecvOp *r = *it;
      ch.recvs.erase(it);
      r->take_self(sh, tag, ch.myRank);
      return true;
    }
  ch.sends.push_back({sh, tag});
  return true;
}

bool forget_channel(MPI_Comm comm) {
  auto it = selfChannels.find(comm_key(comm));
  if (it == selfChannels.end()) return false;
  spill_channel(comm);
  selfChannels.erase(it);
  return true;
}

void clear_channels() { selfChannels.clear(); }

std::unique_ptr<Op> new_irecv(const TypeRecord *r, char *origin, int count, MPI_Datatype dt, int source, int tag,
                              MPI_Comm comm, int dev, int64_t bytes, MPI_Message *msg, std::unique_ptr<Probed> pre) {
  return std::make_unique<IrecvOp>(r, origin, count, dt, source, tag, comm, dev, bytes, msg, std::move(pre));
}
std::unique_ptr<Op> new_lib_irecv(void *buf, int count, MPI_Datatype dt, int source, int tag, MPI_Comm comm,
                                  MPI_Message *msg, std::unique_ptr<Probed> pre) {
  return std::make_unique<LibIrecvOp>(buf, count, dt, source, tag, comm, msg, std::move(pre));
}
std::unique_ptr<Op> new_host_irecv(void *buf, int count, MPI_Datatype dt, int source, int tag, MPI_Comm comm,
                                   std::unique_ptr<Probed> pre) {
  return std::make_unique<HostIrecvOp>(buf, count, dt, source, tag, comm, std::move(pre));
}

} // namespace detail
} // namespace p2p
} // namespace tempi
