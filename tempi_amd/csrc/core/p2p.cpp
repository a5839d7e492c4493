// tempi_amd/csrc/core/p2p.cpp -- see p2p.hpp
#include "trace.hpp"
#include "p2p.hpp"

#include "alloc.hpp"
#include "counters.hpp"
#include "env.hpp"
#include "gpu.hpp"
#include "log.hpp"
#include "next_mpi.hpp"
#include "perf_model.hpp"
#include "state.hpp"
#include "topology.hpp"
#include "type_cache.hpp"

#include <chrono>
#include <cstddef>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <deque>
#include <map>
#include <tuple>
#include <unordered_map>
#include <memory>
#include <memory_resource>
#include <unistd.h>
#include <vector>

namespace tempi {
namespace p2p {

enum class Method { ONESHOT, STAGED, DEVICE, IPC, LIBPACK };

namespace {

constexpr uint64_t kMagic0 = 0x54454d5049495043ull; // "TEMPIIPC"
constexpr uint64_t kMagic1 = 0x9e3779b97f4a7c15ull;

struct IpcDesc {
  uint64_t magic[2];
  uint64_t slabId;
  uint64_t offset;
  int64_t bytes;
  int32_t senderWorld;
  int32_t senderPid;
  int32_t ackTag;
  uint32_t gpu;    // gpu::identity of the slab's GPU
  uint64_t rawPtr; // valid inside the sender's own process
  unsigned char handle[TEMPI_HIP_IPC_HANDLE_BYTES];
};
static_assert(sizeof(IpcDesc) == 128, "descriptor size");

// DIRECT (a send to this same process): the descriptor names the sender's
// object itself, and the receiver copies it strided -> strided into its own
// object with one kernel (tempi_hip_copy_batch): no packed intermediate, half
// the HBM traffic of pack + unpack. The sender completes once the receiver's
// copy has run. If the sender is waited on before the matching receive has
// been posted, it falls back to gathering into a slab (so a wait on a send
// never depends on a later receive), and the receiver unpacks that slab.
constexpr uint64_t kMagicDirect = 0x54454d5049445254ull; // "TEMPIDRT"

struct DirectDesc {
  uint64_t magic[2];
  uint64_t token; // key of the DirectShared below
  int64_t bytes;
  int32_t senderWorld;
  int32_t senderPid;
  int32_t device; // the sender object's GPU
  int32_t pad;
  uint64_t first;      // the sender object's first byte
  tempi_hip_desc desc; // its shape, element count folded in
  uint64_t reserved;
};
static_assert(sizeof(DirectDesc) == 160 && sizeof(DirectDesc) != sizeof(IpcDesc), "descriptor size");

// IPC COPY (a large message between processes, wide rows): the descriptor
// names the sender's own object through an IPC handle of its allocation, and
// the receiver copies it strided -> strided straight out of the sender's
// memory (tempi_hip_copy_batch, source read with system-scope loads). No
// gather on the sender, no packed slab: the payload crosses xGMI once and
// each HBM sees it once. The send completes when the receiver acknowledges
// its copy (rendezvous), so only messages of at least TEMPI_IPC_COPY_MIN_BYTES
// take this route: larger than MPICH's eager limit, i.e. messages the library
// itself would not buffer either (a program waiting on such a send before
// posting the matching receive deadlocks with MPICH alone too). Narrow rows (< TEMPI_IPC_COPY_MIN_BLOCK)
// are gathered on the sender instead: a 24-byte row read across xGMI costs a
// whole remote line.
constexpr uint64_t kMagicCopy = 0x54454d5049585043ull; // "TEMPIXPC"

struct IpcCopyDesc {
  uint64_t magic[2];
  int64_t bytes;
  int32_t senderWorld;
  int32_t senderPid;
  int32_t ackTag;
  int32_t device;
  uint64_t bufferId; // the sender allocation's id: the receiver's mapping cache key
  uint64_t offset;   // of the object's first byte from the allocation base
  uint64_t rawFirst; // the first byte, in the sender's address space
  unsigned char handle[TEMPI_HIP_IPC_HANDLE_BYTES];
  tempi_hip_desc desc; // the object's shape, element count folded in
  uint32_t gpu;        // gpu::identity of the object's GPU
  uint32_t pad;
};
static_assert(sizeof(IpcCopyDesc) == 232, "descriptor size");

// Operation objects, the shared state of direct sends and the request table
// are carved from one unsynchronised pool (the transport runs on the MPI
// thread only), so a message's bookkeeping costs no malloc / free. The pool
// is never destroyed: objects that outlive MPI_Finalize (statics torn down at
// exit) still return their memory to it.
std::pmr::unsynchronized_pool_resource &op_pool() {
  static auto *pool = new std::pmr::unsynchronized_pool_resource();
  return *pool;
}

struct Op;
struct DirectShared {
  DirectDesc desc{}; // the library's send buffer: alive until the receiver claims it
  enum State { PENDING, CLAIMED, PACKED, DONE } state = PENDING;
  Slab *slab = nullptr; // PACKED: the sender's gather (released by the receiver)
  int device = 0;
  Op *sender = nullptr; // while the send is incomplete
};
std::unordered_map<uint64_t, std::shared_ptr<DirectShared>> directShared; // sent, not yet matched
uint64_t nextDirectToken = 1;
bool directEnabled = true;
bool ipcSystemLoads = true; // TEMPI_IPC_PLAIN_LOADS=1 turns off TEMPI_HIP_ITEM_REMOTE (A/B only)
bool hostRecvAware = true;  // TEMPI_NO_HOST_RECV=1: host receives go straight to the library (A/B only)

MPI_Comm ctrlComm = MPI_COMM_NULL; // private duplicate of MPI_COMM_WORLD for acks
int tagUb = 32767;
bool gpuAwareLibrary = false;
int64_t ipcMinBytes = 4 * 1024;

// Acks between the ranks of one node go through shared memory: each rank
// exposes `slots` 32-bit slots (MPI_Win_allocate_shared over its
// MPI_COMM_TYPE_SHARED communicator). A sender takes a free slot of its own
// board for each message whose ack it waits for (IPC slab, IPC COPY) and names
// it as the descriptor's ackTag; the receiver stores code + 1 into that slot
// (release) and the sender polls its outstanding slots on each progress pass
// (acquire). No library message per ack, and no library request in the
// sender's MPI_Testsome for it. Tags below `slots` are board slots; acks that
// travel as library messages (a peer outside the node communicator, no free
// slot, TEMPI_NO_SHM_ACKS) keep tags at or above it.
struct AckBoard {
  MPI_Comm node = MPI_COMM_NULL;
  MPI_Win win = MPI_WIN_NULL;
  std::vector<uint32_t *> of; // per world rank: its slots (nullptr: not on this board)
  std::vector<int> freeSlots;
  int slots = 0; // 0: off
};
AckBoard board;

// a free slot of this rank's board for a message to world rank `peer`, or -1
int board_take(int peer) {
  if (!board.slots || peer < 0 || size_t(peer) >= board.of.size() || !board.of[size_t(peer)] ||
      board.freeSlots.empty())
    return -1;
  const int s = board.freeSlots.back();
  board.freeSlots.pop_back();
  return s;
}

// the ack code in this rank's slot (and the slot freed), or -1 until it arrives
int board_poll(int slot) {
  uint32_t *p = board.of[size_t(state.worldRank)] + slot;
  const uint32_t v = __atomic_load_n(p, __ATOMIC_ACQUIRE);
  if (!v) return -1;
  __atomic_store_n(p, 0u, __ATOMIC_RELAXED);
  board.freeSlots.push_back(slot);
  return int(v) - 1;
}

void board_init() {
  board = AckBoard();
  if (std::getenv("TEMPI_NO_SHM_ACKS")) return;
  const int half = std::max(1, tagUb / 2);
  const int slots = std::min(16384, half / 2); // (library-message ack tags stay above)
  if (slots < 64) return;
  MPI_Comm_split_type(MPI_COMM_WORLD, MPI_COMM_TYPE_SHARED, state.worldRank, MPI_INFO_NULL, &board.node);
  MPI_Comm_set_errhandler(board.node, MPI_ERRORS_RETURN); // no shared window: library acks, not an abort
  uint32_t *mine = nullptr;
  if (MPI_Win_allocate_shared(MPI_Aint(slots) * MPI_Aint(sizeof(uint32_t)), int(sizeof(uint32_t)), MPI_INFO_NULL,
                              board.node, &mine, &board.win) != MPI_SUCCESS) {
    next.MPI_Comm_free(&board.node);
    return;
  }
  std::memset(mine, 0, size_t(slots) * sizeof(uint32_t));
  int n = 0;
  MPI_Comm_size(board.node, &n);
  MPI_Group g, wg;
  MPI_Comm_group(board.node, &g);
  MPI_Comm_group(MPI_COMM_WORLD, &wg);
  std::vector<int> local(static_cast<size_t>(n)), world(static_cast<size_t>(n));
  for (int i = 0; i < n; ++i) local[size_t(i)] = i;
  MPI_Group_translate_ranks(g, n, local.data(), wg, world.data());
  MPI_Group_free(&g);
  MPI_Group_free(&wg);
  board.of.assign(size_t(state.worldSize), nullptr);
  for (int i = 0; i < n; ++i) {
    MPI_Aint size = 0;
    int unit = 0;
    uint32_t *base = nullptr;
    MPI_Win_shared_query(board.win, i, &size, &unit, &base);
    if (world[size_t(i)] >= 0) board.of[size_t(world[size_t(i)])] = base;
  }
  board.freeSlots.reserve(size_t(slots));
  for (int i = slots - 1; i >= 0; --i) board.freeSlots.push_back(i);
  board.slots = slots;
  MPI_Barrier(board.node); // every board is zeroed before any rank writes to one
}

void board_finalize() {
  if (board.win != MPI_WIN_NULL) MPI_Win_free(&board.win);
  if (board.node != MPI_COMM_NULL) next.MPI_Comm_free(&board.node);
  board = AckBoard();
}

// acks the sender is waiting for before reusing a device slab
struct PendingAck {
  MPI_Request req; // the library receive of the ack (not on the board)
  Slab *slab;   // nullptr once released
  int peer;     // world rank of the receiver
  int tag;      // ack tag (a board slot when onBoard)
  int64_t bytes;
  int code;     // received ack payload
  bool onBoard; // the ack arrives in board slot `tag`
};
std::vector<std::unique_ptr<PendingAck>> pendingAcks; // stable addresses: Irecv targets

// peer slabs mapped into this process: (world rank, slab id) -> base
std::map<std::pair<int, uint64_t>, void *> ipcOpen;
// peer allocations mapped for IPC COPY: (world rank, buffer id) -> mapping
struct AllocMap {
  void *base;                // the mapping in this process
  uint64_t senderBase;       // the allocation's base in the sender's address space
  unsigned char handle[TEMPI_HIP_IPC_HANDLE_BYTES];
};
std::map<std::pair<int, uint64_t>, AllocMap> ipcAllocOpen;
// this process's allocations exported for IPC COPY: base -> (buffer id, handle)
struct Export {
  uint64_t id;
  unsigned char handle[TEMPI_HIP_IPC_HANDLE_BYTES];
};
std::unordered_map<uintptr_t, Export> ipcExports;
bool ipcCopyEnabled = true;             // TEMPI_NO_IPC_COPY
// Inside MPI_Alltoallv every receive is posted before any send is waited on,
// so a rendezvous send cannot deadlock there: IPC COPY takes messages of any
// size (TEMPI_NO_COLL_COPY keeps the point-to-point threshold)
bool collCopyEnabled = true;
// above MPICH's own eager limit (MPIR_CVAR_CH3_EAGER_MAX_MSG_SIZE, 128 KiB):
// a program that works with the library's rendezvous works with this one
int64_t ipcCopyMinBytes = 128 * 1024 + 1; // TEMPI_IPC_COPY_MIN_BYTES
int64_t ipcCopyMinBlock = 256;          // TEMPI_IPC_COPY_MIN_BLOCK
uint32_t nextCopyTag = 0;

// A datatype handle that stays valid while an operation still needs it:
// the application may MPI_Type_free its type right after MPI_Isend /
// MPI_Irecv returns. Derived types are duplicated (the duplicate of a
// committed type is committed); named types are returned as they are.
bool named_type(MPI_Datatype t) {
  int ni = 0, na = 0, nd = 0, comb = 0;
  MPI_Type_get_envelope(t, &ni, &na, &nd, &comb);
  return comb == MPI_COMBINER_NAMED;
}
MPI_Datatype hold_type(MPI_Datatype t) {
  if (named_type(t)) return t;
  MPI_Datatype d = MPI_DATATYPE_NULL;
  MPI_Type_dup(t, &d);
  return d;
}
void drop_type(MPI_Datatype t) {
  if (t != MPI_DATATYPE_NULL && !named_type(t)) next.MPI_Type_free(&t);
}

// the status of a completed receive: `bytes` received (MPI_Get_count with
// the receive's datatype then gives whole elements), without touching the
// application's datatype handle, which may have been freed meanwhile
void set_received(MPI_Status *s, int64_t bytes) { MPI_Status_set_elements_x(s, MPI_BYTE, MPI_Count(bytes)); }

int64_t pack_size(int count, MPI_Datatype dt, MPI_Comm comm) {
  int s = 0;
  MPI_Pack_size(count, dt, comm, &s);
  return s;
}

// AUTO with a measured perf.json: the cheapest modelled method, cached per
// (colocated, bytes, block) as in the reference (/root/reference/src/internal/
// sender.cpp:251-290, async_operation.cpp:334-389). The DEVICE curve is
// carried out by IPC between co-located ranks when the library is not
// GPU-aware (the intra-node GPU-GPU curve is measured through that path).
std::map<std::tuple<bool, int64_t, int64_t>, Method> modelCache;

bool model_choice(int64_t bytes, bool colocated, int64_t block, Method *out) {
  if (!systemPerformanceLoaded) return false;
  const auto key = std::make_tuple(colocated, bytes, block);
  auto it = modelCache.find(key);
  if (it != modelCache.end()) {
    *out = it->second;
    return true;
  }
  const SystemPerformance &sp = systemPerformance;
  const Opt o = model_oneshot(sp, colocated, bytes, block);
  const Opt d = model_device(sp, colocated, bytes, block, !gpuAwareLibrary);
  const Opt s = model_staged(sp, colocated, bytes, block);
  Method best = Method::ONESHOT;
  double t = o.ok ? o.v : 1e300;
  const Method dev = gpuAwareLibrary ? Method::DEVICE : (colocated ? Method::IPC : Method::STAGED);
  if (d.ok && d.v < t) {
    best = dev;
    t = d.v;
  }
  if (s.ok && s.v < t) best = Method::STAGED;
  if (!o.ok && !d.ok && !s.ok) return false;
  modelCache[key] = best;
  *out = best;
  return true;
}

int64_t modelBlock = 512; // block length of the type being sent (set per call)

Method choose(int64_t bytes, bool colocated) {
  switch (env.datatype) {
  case DatatypeMethod::ONESHOT:
    return Method::ONESHOT;
  case DatatypeMethod::STAGED:
    return Method::STAGED;
  case DatatypeMethod::DEVICE:
    if (gpuAwareLibrary) return Method::DEVICE;
    return colocated ? Method::IPC : Method::STAGED;
  case DatatypeMethod::IPC:
    return colocated ? Method::IPC : Method::ONESHOT;
  case DatatypeMethod::AUTO:
  default: {
    Method m;
    if (model_choice(bytes, colocated, modelBlock, &m)) return m;
    if (colocated && bytes >= ipcMinBytes) return Method::IPC;
    return Method::ONESHOT;
  }
  }
}

// peers whose memory could not be mapped: no more IPC to or from them
std::vector<char> ipcBroken;

bool ipc_broken(int world) { return world >= 0 && size_t(world) < ipcBroken.size() && ipcBroken[size_t(world)]; }

void mark_ipc_broken(int world) {
  if (world < 0) return;
  if (ipcBroken.size() <= size_t(world)) ipcBroken.resize(size_t(world) + 1, 0);
  if (!ipcBroken[size_t(world)]) LOG_WARN("IPC with rank " << world << " unavailable; using host-staged transfers");
  ipcBroken[size_t(world)] = 1;
}

// the sender's slab mapped into this process, or nullptr when it cannot be
void *peer_pointer(const IpcDesc &d) {
  if (d.senderPid == int32_t(getpid())) return reinterpret_cast<void *>(d.rawPtr);
  auto key = std::make_pair(int(d.senderWorld), d.slabId);
  auto it = ipcOpen.find(key);
  if (it != ipcOpen.end()) return it->second;
  void *p = nullptr;
  // fault injection (tests): TEMPI_FAULT_IPC_OPEN makes every mapping fail
  static const bool injectFault = std::getenv("TEMPI_FAULT_IPC_OPEN") != nullptr;
  const int e = injectFault ? 1 : tempi_hip_ipc_open_handle(&p, d.handle);
  if (e != 0) {
    LOG_WARN("cannot map rank " << d.senderWorld << "'s slab: " << tempi_hip_error_string(e));
    mark_ipc_broken(d.senderWorld);
    return nullptr;
  }
  ipcOpen[key] = p;
  return p;
}

// First contact with a peer on ANOTHER GPU. This pool's boxes have one GPU,
// so the cross-GPU IPC path is first met on the driver's 8-GPU node: before
// the transport trusts a mapping of that peer's memory, the first bytes a
// descriptor names are read twice -- by a DMA copy (hipMemcpy) and by the
// remote-load copy kernel the receiver uses (TEMPI_HIP_ITEM_REMOTE,
// system-scope loads) -- and compared on the host. The kernel runs only after
// the DMA read succeeded and when HIP reports that this GPU can load from the
// mapping's GPU, so a mapping the fabric cannot serve fails as a HIP error,
// never as a faulting kernel. A failed read or a mismatch turns IPC with that
// peer off: this message and every later one go through the host (the NACK
// path). Once per peer; at most 64 KiB.
std::vector<signed char> canaryVerdict; // per world rank: 0 untested, 1 passed, -1 failed
bool faultCanary = false;               // TEMPI_FAULT_CANARY: the comparison fails (tests)

bool canary(int world, const void *peerBytes, int64_t n, int device) {
  if (world < 0) return true;
  if (canaryVerdict.size() <= size_t(world)) canaryVerdict.resize(size_t(world) + 1, 0);
  signed char &v = canaryVerdict[size_t(world)];
  if (v) return v > 0;
  n = std::min<int64_t>(n, 64 * 1024);
  if (n <= 0) return true; // nothing to read yet: decide on a later message
  int cur = 0;
  tempi_hip_get_device(&cur);
  if (cur != device) tempi_hip_set_device(device);
  std::vector<unsigned char> viaKernel(size_t(n), 0), viaDma(size_t(n), 1);
  bool ok = tempi_hip_memcpy(viaDma.data(), peerBytes, size_t(n)) == 0;
  if (ok) {
    tempi_hip_ptrinfo info;
    if (tempi_hip_pointer_info(peerBytes, &info) == 0 && info.device >= 0 &&
        !tempi_hip_can_access_peer(device, info.device)) {
      LOG_WARN("canary: GPU " << device << " cannot load from GPU " << info.device << " (rank " << world << ")");
      ok = false;
    }
  }
  void *scratch = nullptr;
  ok = ok && tempi_hip_malloc(&scratch, size_t(n)) == 0;
  if (ok) {
    tempi_hip_copy_item c{};
    c.dst_first = scratch;
    c.src_first = peerBytes;
    c.dst.block = n;
    c.dst.ndims = 0;
    c.src = c.dst;
    c.flags = TEMPI_HIP_ITEM_REMOTE;
    void *s = gpu::stream(device);
    ok = tempi_hip_copy_batch(&c, 1, s) == 0 && tempi_hip_stream_synchronize(s) == 0 &&
         tempi_hip_memcpy(viaKernel.data(), scratch, size_t(n)) == 0;
  }
  if (scratch) tempi_hip_free(scratch);
  if (cur != device) tempi_hip_set_device(cur);
  if (ok && faultCanary) viaDma[0] ^= 0xFF;
  ok = ok && viaKernel == viaDma;
  v = ok ? 1 : -1;
  if (ok) {
    counters.canary_ok++;
    LOG_DEBUG("canary: rank " << world << "'s GPU memory reads back right (" << n << " B)");
  } else {
    counters.canary_fail++;
    LOG_WARN("canary: rank " << world << "'s GPU memory does not read back right through IPC");
    mark_ipc_broken(world);
  }
  return ok;
}

// ack payload: 0 = pulled, release the slab; 1 = could not map it, send the
// bytes through the host on (ctrlComm, ackTag)
int ackCodes[3] = {0, 1, 2};

void send_ack(int world, int tag, int code) {
  if (tag < board.slots && world >= 0 && size_t(world) < board.of.size() && board.of[size_t(world)]) {
    __atomic_store_n(board.of[size_t(world)] + tag, uint32_t(code + 1), __ATOMIC_RELEASE);
    return;
  }
  MPI_Request r;
  next.MPI_Isend(&ackCodes[code], 1, MPI_INT, world, tag, ctrlComm, &r);
  next.MPI_Request_free(&r);
}
void send_ack(const IpcDesc &d, int code = 0) { send_ack(d.senderWorld, d.ackTag, code); }

// IPC COPY acks: 0 = copied; 1 = cannot copy this shape, send the packed
// bytes through the host on (ctrlComm, ackTag); 2 = the same, and the
// sender's memory could not be mapped (no more IPC with that rank)
enum { kCopyDone = 0, kCopyResend = 1, kCopyUnmapped = 2 };

// A new allocation of a sender at the base of one we hold mapped, or with the
// same handle bytes, means that sender freed the old one (its sends from it
// have completed, so no copy of ours still reads it). Close those mappings
// first: the runtime may hand back its cached import for identical handle
// bytes -- the freed allocation's pages, not the new one's.
void forget_freed_allocs(const IpcCopyDesc &d) {
  const uint64_t senderBase = d.rawFirst - d.offset;
  bool synced = false;
  for (auto it = ipcAllocOpen.begin(); it != ipcAllocOpen.end();) {
    const AllocMap &m = it->second;
    if (it->first.first == int(d.senderWorld) &&
        (m.senderBase == senderBase || std::memcmp(m.handle, d.handle, sizeof m.handle) == 0)) {
      if (!synced) {
        gpu::check(tempi_hip_device_synchronize(), "ipc mapping replace");
        synced = true;
      }
      LOG_DEBUG("ipc copy unmap: rank " << d.senderWorld << " id " << it->first.second << " (replaced by id "
                                        << d.bufferId << ")");
      tempi_hip_ipc_close_handle(m.base);
      counters.ipc_maps_replaced++;
      it = ipcAllocOpen.erase(it);
    } else {
      ++it;
    }
  }
}

// the sender's allocation mapped into this process (its first byte), or
// nullptr when it cannot be
const char *peer_object(const IpcCopyDesc &d) {
  if (d.senderPid == int32_t(getpid())) return reinterpret_cast<const char *>(d.rawFirst);
  auto key = std::make_pair(int(d.senderWorld), d.bufferId);
  auto it = ipcAllocOpen.find(key);
  if (it == ipcAllocOpen.end()) {
    forget_freed_allocs(d);
    void *p = nullptr;
    static const bool injectFault = std::getenv("TEMPI_FAULT_IPC_OPEN") != nullptr;
    const int e = injectFault ? 1 : tempi_hip_ipc_open_handle(&p, d.handle);
    if (e != 0) {
      LOG_WARN("cannot map rank " << d.senderWorld << "'s buffer: " << tempi_hip_error_string(e));
      mark_ipc_broken(d.senderWorld);
      return nullptr;
    }
    AllocMap m;
    m.base = p;
    m.senderBase = d.rawFirst - d.offset;
    std::memcpy(m.handle, d.handle, sizeof m.handle);
    it = ipcAllocOpen.emplace(key, m).first;
    LOG_DEBUG("ipc copy map: rank " << d.senderWorld << " id " << d.bufferId << " -> " << p);
  }
  return static_cast<const char *>(it->second.base) + d.offset;
}

// this process's allocation holding `first` exported for IPC COPY: fills the
// descriptor's handle / buffer id / offset; false when it cannot be exported
// (not hipMalloc memory, or the export fails)
bool export_object(const void *first, IpcCopyDesc *d) {
  void *base = nullptr;
  size_t size = 0;
  uint64_t id = 0;
  if (tempi_hip_mem_info(first, &base, &size, &id) != 0 || !base) return false;
  const uintptr_t b = reinterpret_cast<uintptr_t>(base);
  auto it = ipcExports.find(b);
  if (it == ipcExports.end() || it->second.id != id) { // new, or freed and replaced at the same address
    Export x;
    x.id = id;
    if (tempi_hip_ipc_get_handle(x.handle, base) != 0) return false;
    it = ipcExports.insert_or_assign(b, x).first;
    LOG_DEBUG("ipc copy export: base " << base << " size " << size << " id " << id);
  } else {
    LOG_DEBUG("ipc copy export reused: base " << base << " size " << size << " id " << id);
  }
  d->bufferId = id;
  d->offset = uint64_t(reinterpret_cast<uintptr_t>(first) - b);
  std::memcpy(d->handle, it->second.handle, sizeof d->handle);
  return true;
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

// one batched launch (+ its trailing copies) and the event that follows it
struct Op;
struct GpuBatch {
  void *event = nullptr;
  int device = 0;
  int lane = 0;
  bool scatter = false;
  bool complete = false;
  std::vector<Op *> ops; // whose GPU work this batch carries (alive until gpu_done)
};
std::deque<std::shared_ptr<GpuBatch>> batches; // launch order

struct Op {
  virtual ~Op() {}
  static void *operator new(size_t n) { return op_pool().allocate(n, alignof(std::max_align_t)); }
  // (virtual destructor: `n` is the size of the object's dynamic type)
  static void operator delete(void *p, size_t n) { op_pool().deallocate(p, n, alignof(std::max_align_t)); }
  virtual void gpu_done() {}                   // its GPU work completed
  virtual void lib_done(const MPI_Status &) {} // library request completed
  virtual void status(MPI_Status *s) const = 0;
  virtual void stalled() {}                    // waited on and still incomplete after a pass
  virtual void peer_done() {}                  // (direct sends) the receiver's copy ran
  virtual void post() {}                       // (sends) hand the message to the library
  virtual void cancel() {}                     // MPI_Cancel (receives not yet matched)
  bool queued = false;                         // GPU work not launched yet
  bool ready = false;                          // (sends in a gate) post() may run
  bool posted = false;                         // (sends) post() has run
  int device = 0;
  MPI_Request lib = MPI_REQUEST_NULL;          // outstanding library request
  bool watched = false;                        // in libWatch
  bool detached = false;                       // MPI_Request_free'd: dropped when done
  bool done = false;
  int err = MPI_SUCCESS;                       // completed with this error (MPI_ERR_TRUNCATE, ...)
  MPI_Comm errComm = MPI_COMM_NULL;            // whose error handler the wait raises it on
  int boardSlot = -1;                          // waiting for an ack in this board slot (boardOps)
  virtual void acked(int) {}                   // that ack arrived with this code
};

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
struct SendGate {
  std::vector<Op *> q;
  size_t head = 0;
  bool busy() const { return head < q.size(); }
};
std::unordered_map<uint64_t, SendGate> gates;
size_t gatedOps = 0; // ops in any gate: 0 means every send may post at once

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

// GPU work waiting for the next flush: gathers of Isends, scatters and direct
// copies of Irecvs. Flat arrays (no per-message allocation); one launch per
// (kind, word width, rank) group and device at flush time.
struct PendingList {
  std::vector<Op *> ops;
  std::vector<tempi_hip_batch_item> items;
  std::vector<int> itemDev;
  std::vector<tempi_hip_copy_item> copies; // direct: strided -> strided (unpack list only)
  std::vector<int> copyDev;
  struct Stage { // STAGED: D2H copy after the packs
    void *dst;
    const void *src;
    size_t n;
    int dev;
  };
  std::vector<Stage> stages;
  bool afterPack = false; // (unpack list) holds a scatter of a gather still on lane 0
  bool empty() const { return ops.empty(); }
  size_t size() const { return ops.size(); }
  void clear() {
    ops.clear();
    items.clear();
    itemDev.clear();
    copies.clear();
    copyDev.clear();
    stages.clear();
    afterPack = false;
  }
  void add_items(const Op *op, const Packer &pk, void *packed, const void *origin, int64_t count) {
    pk.items(packed, origin, count, items);
    itemDev.resize(items.size(), op->device);
  }
  void add_copy(const Op *op, const tempi_hip_copy_item &c) {
    copies.push_back(c);
    copyDev.push_back(op->device);
  }
  void queue(Op *op) {
    op->queued = true;
    ops.push_back(op);
  }
};
PendingList pendingPack, pendingUnpack;
constexpr size_t kMaxPending = 512;
size_t earlyFlush = 32; // TEMPI_EARLY_FLUSH
size_t firstFlush = 16;  // TEMPI_FIRST_FLUSH: the same while no scatter batch is in flight
int scattersInFlight = 0; // scatter / copy batches launched and not yet seen complete
bool eagerFlush = false;  // TEMPI_EAGER_FLUSH (A/B): waits launch queued scatters even while every lane is busy

template <typename T> const T *select(const std::vector<T> &v, const std::vector<int> &dev, int d, bool all,
                                      std::vector<T> &tmp) {
  if (all) return v.data();
  tmp.clear();
  for (size_t i = 0; i < v.size(); ++i)
    if (dev[i] == d) tmp.push_back(v[i]);
  return tmp.data();
}

int nextLane = 0; // round robin over the scatter lanes

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
    if (nitems)
      gpu::check(pack ? tempi_hip_pack_batch(items, int(nitems), s) : tempi_hip_unpack_batch(items, int(nitems), s),
                 pack ? "batched pack" : "batched unpack");
    if (ncopies) gpu::check(tempi_hip_copy_batch(copies, int(ncopies), s), "batched direct copy");
    for (const PendingList::Stage &st : list.stages)
      if (st.dev == dev) gpu::check(tempi_hip_memcpy_async(st.dst, st.src, st.n, s), "staged D2H");
    auto b = std::make_shared<GpuBatch>();
    b->device = dev;
    b->lane = lane;
    b->scatter = !pack;
    if (!pack) ++scattersInFlight;
    b->event = get_event();
    gpu::check(tempi_hip_event_record(b->event, s), "event record");
    if (cur != dev) tempi_hip_set_device(cur);
    for (Op *op : list.ops)
      if (op->device == dev) {
        op->queued = false;
        b->ops.push_back(op);
      }
    batches.push_back(b);
  }
  list.clear();
}

void flush() {
  flush_list(pendingPack, true);
  flush_list(pendingUnpack, false);
}

// Peer allocations stay mapped for reuse (keyed by buffer id). A peer that
// keeps allocating new buffers would make that grow without bound and hold
// its freed memory alive, so past kMaxAllocMaps every mapping is closed --
// after the copies that may still read them have been launched and run.
constexpr size_t kMaxAllocMaps = 256;
void recycle_alloc_maps() {
  if (ipcAllocOpen.size() < kMaxAllocMaps) return;
  flush_list(pendingUnpack, false);
  gpu::check(tempi_hip_device_synchronize(), "ipc mapping recycle");
  for (auto &kv : ipcAllocOpen) tempi_hip_ipc_close_handle(kv.second.base);
  ipcAllocOpen.clear();
}

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

  IsendOp(const TypeRecord *r, const char *o, int c, MPI_Datatype d, int de, int t, MPI_Comm cm, int dev,
          Method m, int64_t b)
      : rec(r->ref()), origin(o), count(c), dest(de), tag(t), dt(d), comm(cm), method(m), bytes(b),
        key(gate_key(cm, de)) {
    device = dev;
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
  void post() override {
    switch (method) {
    case Method::ONESHOT:
    case Method::STAGED:
      next.MPI_Isend(hslab->host, int(bytes), MPI_PACKED, dest, tag, comm, &lib);
      watch(this);
      break;
    case Method::DEVICE:
      next.MPI_Isend(dslab->dev, int(bytes), MPI_PACKED, dest, tag, comm, &lib);
      watch(this);
      break;
    case Method::IPC: {
      desc.magic[0] = kMagic0;
      desc.magic[1] = kMagic1;
      desc.slabId = dslab->id;
      desc.offset = 0;
      desc.bytes = bytes;
      desc.senderWorld = state.worldRank;
      desc.senderPid = int32_t(getpid());
      desc.rawPtr = reinterpret_cast<uint64_t>(dslab->dev);
      desc.gpu = gpu::identity(device);
      std::memcpy(desc.handle, slab_ipc_handle(dslab), sizeof desc.handle);
      // the slab is reused once the receiver acknowledges: in a board slot,
      // or as a library message on the private communicator (those tags take
      // [board.slots, tagUb/2); IPC COPY's the upper half)
      const int peer = topology::world_rank(comm, dest);
      const int slot = board_take(peer);
      const uint32_t span = uint32_t(std::max(1, tagUb / 2 - board.slots));
      desc.ackTag = slot >= 0 ? slot : board.slots + int32_t(dslab->id % span);
      pendingAcks.push_back(
          std::unique_ptr<PendingAck>(new PendingAck{MPI_REQUEST_NULL, dslab, peer, desc.ackTag, bytes, -1, slot >= 0}));
      PendingAck &pa = *pendingAcks.back();
      if (slot < 0) next.MPI_Irecv(&pa.code, 1, MPI_INT, peer, desc.ackTag, ctrlComm, &pa.req);
      dslab = nullptr;
      next.MPI_Isend(&desc, int(sizeof desc), MPI_PACKED, dest, tag, comm, &lib);
      watch(this);
      break;
    }
    default:
      break;
    }
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
      s->MPI_ERROR = MPI_SUCCESS;
      MPI_Status_set_elements(s, MPI_BYTE, 0);
    }
  }
};

struct IsendDirectOp;
// the self channel (below) took this direct send: matched to a waiting
// receive, or kept for a later one -- no library message (false: post the
// descriptor through the library)
bool self_send(IsendDirectOp *op);

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
    desc.senderPid = int32_t(getpid());
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
    if (self_send(this)) {
      maybe_done();
      return;
    }
    directShared[sh->desc.token] = sh; // claimed by the receive that matches the descriptor
    // the library may hold a send to this same process open until its
    // receive is posted (MPICH does), so the send's completion cannot wait for
    // it: the request is released now and the descriptor outlives it in `sh`
    MPI_Request sreq;
    next.MPI_Isend(&sh->desc, int(sizeof sh->desc), MPI_PACKED, dest, tag, comm, &sreq);
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
    maybe_done();
  }
  void peer_done() override { maybe_done(); }
  void stalled() override {
    if (sh->state != DirectShared::PENDING) return;
    // waited on before its receive exists: gather into a slab the receiver
    // will unpack, so the send can complete on its own
    counters.direct_fallbacks++;
    sh->state = DirectShared::PACKED;
    sh->slab = device_pool().get(size_t(bytes), device);
    pendingPack.add_items(this, *rec->packer, sh->slab->dev, origin, count);
    pendingPack.queue(this);
  }
  void status(MPI_Status *s) const override {
    if (s != MPI_STATUS_IGNORE) {
      s->MPI_SOURCE = MPI_ANY_SOURCE;
      s->MPI_TAG = MPI_ANY_TAG;
      s->MPI_ERROR = MPI_SUCCESS;
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
      boardAck = true;
      boardOps.push_back(this);
      next.MPI_Isend(&desc, int(sizeof desc), MPI_PACKED, dest, tag, comm, &lib);
      watch(this);
      return;
    }
    next.MPI_Irecv(&ack, 1, MPI_INT, peer, desc.ackTag, ctrlComm, &lib);
    watch(this);
    MPI_Request r; // the descriptor lives in this op until the ack, which follows its delivery
    next.MPI_Isend(&desc, int(sizeof desc), MPI_PACKED, dest, tag, comm, &r);
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
      s->MPI_ERROR = MPI_SUCCESS;
      MPI_Status_set_elements(s, MPI_BYTE, 0);
    }
  }
};

// the receiver side is done with a direct send's bytes
void direct_finish(std::shared_ptr<DirectShared> &sh) {
  if (!sh) return;
  if (sh->slab) {
    device_pool().put(sh->slab);
    sh->slab = nullptr;
  }
  sh->state = DirectShared::DONE;
  if (sh->sender) sh->sender->peer_done();
  sh.reset();
}

// the matched descriptor's shared state (unmatched until now)
std::shared_ptr<DirectShared> claim_direct(const DirectDesc &d) {
  auto it = directShared.find(d.token);
  if (d.senderPid != int32_t(getpid()) || it == directShared.end())
    LOG_FATAL("direct-send descriptor from another process (rank " << d.senderWorld << ")");
  std::shared_ptr<DirectShared> sh = it->second;
  directShared.erase(it);
  return sh;
}

// a direct send's packed bytes into pinned host memory `dst`, synchronously
// (receivers that are not a same-device TEMPI receive), then finish it
void materialise_direct(std::shared_ptr<DirectShared> &sh, const DirectDesc &d, Slab *dst) {
  void *s = gpu::stream(sh->device);
  int cur = 0;
  tempi_hip_get_device(&cur);
  if (cur != sh->device) tempi_hip_set_device(sh->device);
  if (sh->state == DirectShared::PACKED) {
    gpu::check(tempi_hip_stream_synchronize(s), "direct fallback sync");
    gpu::check(tempi_hip_memcpy(dst->host, sh->slab->dev, size_t(d.bytes)), "direct fallback copy");
  } else {
    gpu::check(tempi_hip_pack(dst->dev, reinterpret_cast<const void *>(d.first), &d.desc, s), "direct gather");
    gpu::check(tempi_hip_stream_synchronize(s), "direct gather sync");
  }
  if (cur != sh->device) tempi_hip_set_device(cur);
  direct_finish(sh);
}

bool is_direct(const void *msg, int n) {
  if (size_t(n) != sizeof(DirectDesc)) return false;
  uint64_t m[2];
  std::memcpy(m, msg, sizeof m);
  return m[0] == kMagicDirect && m[1] == kMagic1;
}
bool is_ipc_copy(const void *msg, int n) {
  if (size_t(n) != sizeof(IpcCopyDesc)) return false;
  uint64_t m[2];
  std::memcpy(m, msg, sizeof m);
  return m[0] == kMagicCopy && m[1] == kMagic1;
}
bool is_ipc(const void *msg, int n) {
  if (size_t(n) != sizeof(IpcDesc)) return false;
  uint64_t m[2];
  std::memcpy(m, msg, sizeof m);
  return m[0] == kMagic0 && m[1] == kMagic1;
}

// A descriptor landed in a host buffer of a receive that cannot use it
// in place (library receives): fetch the bytes it names into `out` (the IPC
// pull or the direct gather, blocking) and release the sender.
void land_descriptor(const void *msg, int n, std::vector<char> &out) {
  if (is_direct(msg, n)) {
    DirectDesc d;
    std::memcpy(&d, msg, sizeof d);
    std::shared_ptr<DirectShared> sh = claim_direct(d);
    Slab *h = pinned_pool().get(size_t(std::max<int64_t>(d.bytes, 1)), sh->device);
    materialise_direct(sh, d, h);
    out.assign(static_cast<char *>(h->host), static_cast<char *>(h->host) + d.bytes);
    pinned_pool().put(h);
    return;
  }
  auto resend = [&](int world, int tag, int64_t bytes, int code) { // the sender gathers and sends the bytes
    MPI_Request r;
    next.MPI_Irecv(out.data(), int(bytes), MPI_PACKED, world, tag, ctrlComm, &r);
    send_ack(world, tag, code);
    for (;;) {
      int flag = 0;
      next.MPI_Test(&r, &flag, MPI_STATUS_IGNORE);
      if (flag) break;
      progress();
    }
  };
  if (is_ipc_copy(msg, n)) { // a host receive: the sender gathers for it
    IpcCopyDesc d;
    std::memcpy(&d, msg, sizeof d);
    out.resize(size_t(std::max<int64_t>(d.bytes, 1)));
    resend(d.senderWorld, d.ackTag, d.bytes, kCopyResend);
    out.resize(size_t(d.bytes));
    return;
  }
  IpcDesc d;
  std::memcpy(&d, msg, sizeof d);
  out.resize(size_t(std::max<int64_t>(d.bytes, 1)));
  if (void *base = peer_pointer(d)) {
    gpu::check(tempi_hip_memcpy(out.data(), static_cast<const char *>(base) + d.offset, size_t(d.bytes)), "ipc pull");
    send_ack(d);
  } else { // the sender re-sends through the host
    resend(d.senderWorld, d.ackTag, d.bytes, 1);
  }
  out.resize(size_t(d.bytes));
}

constexpr size_t kDescCap = std::max({sizeof(DirectDesc), sizeof(IpcDesc), sizeof(IpcCopyDesc)});

int64_t desc_bytes(const tempi_hip_desc &d) {
  int64_t b = d.block;
  for (int k = 0; k < d.ndims; ++k) b *= d.counts[k];
  return b;
}

// what tempi_hip_copy_supported() decides, from descriptors that are already
// simplified (Packer::flat): the kernel's own normalisation can only merge
// further, so <= 3 dimensions here is <= 3 there
bool copy_ok(const tempi_hip_desc &dst, const tempi_hip_desc &src) {
  const int64_t b = desc_bytes(src);
  return dst.ndims <= 3 && src.ndims <= 3 && b == desc_bytes(dst) && b < (int64_t(1) << 31);
}

// A message a probe had to receive to look at it (it has a descriptor's
// size): it stays matchable, in arrival order, until a receive or probe takes
// it, or an MPI_Mprobe handle claims it.
struct Probed {
  MPI_Comm comm = MPI_COMM_NULL;
  MPI_Status st{};         // source and tag as the library reported them
  std::vector<char> bytes; // the message as received (MPI_BYTE)
  int64_t payload = 0;     // what the application receives (a descriptor's payload size)
};
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

bool is_descriptor(const void *msg, int n) { return is_direct(msg, n) || is_ipc(msg, n) || is_ipc_copy(msg, n); }

int64_t descriptor_payload(const void *msg, int n) {
  int64_t b = n;
  if (is_direct(msg, n)) std::memcpy(&b, static_cast<const char *>(msg) + offsetof(DirectDesc, bytes), sizeof b);
  if (is_ipc(msg, n)) std::memcpy(&b, static_cast<const char *>(msg) + offsetof(IpcDesc, bytes), sizeof b);
  if (is_ipc_copy(msg, n)) std::memcpy(&b, static_cast<const char *>(msg) + offsetof(IpcCopyDesc, bytes), sizeof b);
  return b;
}

// A message that reached host memory (`msg`, n bytes: a descriptor or the
// packed bytes themselves) delivered into the application's host receive
// (buf, count, dt): the descriptor's bytes are fetched first, then unpacked.
// Returns MPI_SUCCESS or MPI_ERR_TRUNCATE (nothing written); *received =
// bytes delivered.
int land_host(const char *msg, int n, void *buf, int count, MPI_Datatype dt, MPI_Comm comm, int64_t *received) {
  std::vector<char> fetched;
  if (is_descriptor(msg, n)) {
    land_descriptor(msg, n, fetched); // releases the sender whatever happens next
    msg = fetched.data();
    n = int(fetched.size());
  }
  int size = 0;
  MPI_Type_size(dt, &size);
  *received = 0;
  if (int64_t(n) > int64_t(size) * count) return MPI_ERR_TRUNCATE;
  const int elems = size ? n / size : 0;
  int pos = 0;
  if (elems) next.MPI_Unpack(msg, n, &pos, buf, elems, dt, comm);
  *received = int64_t(elems) * size;
  return MPI_SUCCESS;
}

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
    if (msg)
      next.MPI_Imrecv(hslab->host, int(cap), MPI_PACKED, msg, &lib);
    else
      next.MPI_Irecv(hslab->host, int(cap), MPI_PACKED, source, tag, comm, &lib);
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
        pendingUnpack.add_items(this, packer, direct->slab->dev, origin, elems);
        pendingUnpack.afterPack = true;
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
      const bool local = xd.senderPid == int32_t(getpid());
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
        if (!local && ipcSystemLoads && xd.gpu != gpu::identity(device)) c.flags = TEMPI_HIP_ITEM_REMOTE;
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
      if (base && d.senderPid != int32_t(getpid()) && d.gpu != gpu::identity(device) &&
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
      if (ipcSystemLoads && d.gpu != gpu::identity(device)) // another GPU's slab, reused between messages
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
bool selfChannelEnabled = true;

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

bool tags_match(int want, int got) { return want == MPI_ANY_TAG || want == got; }

bool self_send(IsendDirectOp *op) {
  if (!selfChannelEnabled) return false;
  SelfChannel &ch = self_channel(op->comm);
  if (ch.spilled) return false;
  for (auto it = ch.recvs.begin(); it != ch.recvs.end(); ++it)
    if (tags_match((*it)->selfTag, op->tag)) {
      IrecvOp *r = *it;
      ch.recvs.erase(it);
      r->take_self(op->sh, op->tag, ch.myRank);
      return true;
    }
  ch.sends.push_back({op->sh, op->tag});
  return true;
}

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

// library-packed transfer of a device buffer whose type TEMPI cannot pack
// (the touched span is staged through host memory by tempi::pack / unpack)
struct LibIsendOp : Op {
  std::vector<char> buf;
  MPI_Datatype dt;
  int n = 0, dest, tag;
  MPI_Comm comm;
  LibIsendOp(const void *b, int c, MPI_Datatype d, int de, int t, MPI_Comm cm) : dt(d), dest(de), tag(t), comm(cm) {
    buf.resize(size_t(std::max<int64_t>(pack_size(c, d, comm), 1)));
    tempi::pack(b, c, d, buf.data(), int(buf.size()), &n, comm);
    post_or_queue(gate_key(comm, dest), this);
  }
  void post() override {
    next.MPI_Isend(buf.data(), n, MPI_PACKED, dest, tag, comm, &lib);
    watch(this);
  }
  void lib_done(const MPI_Status &) override { done = true; }
  void status(MPI_Status *s) const override {
    if (s != MPI_STATUS_IGNORE) {
      s->MPI_ERROR = MPI_SUCCESS;
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
    next.MPI_Isend(buf, count, dt, dest, tag, comm, &lib);
    watch(this);
  }
  void lib_done(const MPI_Status &) override { done = true; }
  void status(MPI_Status *s) const override {
    if (s != MPI_STATUS_IGNORE) {
      s->MPI_ERROR = MPI_SUCCESS;
      MPI_Status_set_elements(s, MPI_BYTE, 0);
    }
  }
};

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
    if (msg)
      next.MPI_Imrecv(buf.data(), int(buf.size()), MPI_PACKED, msg, &lib);
    else
      next.MPI_Irecv(buf.data(), int(buf.size()), MPI_PACKED, source, tag, comm, &lib);
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
  std::vector<char> stage;
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
      next.MPI_Irecv(b, c, d, source, tag, cm, &lib);
      watch(this);
      return;
    }
    dt = hold_type(d);
    if (pre) {
      libStatus = pre->st;
      deliver(pre->bytes.data(), int(pre->bytes.size()));
      return;
    }
    stage.resize(std::max({size_t(std::max<int64_t>(cap, 1)), size_t(pack_size(c, d, cm)), kDescCap}));
    next.MPI_Irecv(stage.data(), int(stage.size()), MPI_PACKED, source, tag, cm, &lib);
    watch(this);
  }
  ~HostIrecvOp() override { drop_type(dt); }
  void cancel() override {
    if (lib != MPI_REQUEST_NULL) next.MPI_Cancel(&lib);
  }
  void deliver(const char *msg, int n) {
    err = land_host(msg, n, user, count, dt, comm, &received);
    done = true;
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
    if (!inPlace) return deliver(stage.data(), n);
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
      s->MPI_ERROR = MPI_SUCCESS;
      set_received(s, bytes);
    }
  }
};

// ------------------------------------------------------------- request table

// TEMPI request handles live in [1, 2^26): the top bits of an MPICH handle
// always encode a non-zero kind, so the library never issues one of these
// (the reference uses a plain counter that can collide: SURVEY F9)
constexpr uint32_t kHandleSpace = 1u << 26;
uint32_t nextHandle = 1;
std::pmr::unordered_map<uint32_t, std::unique_ptr<Op>> active{&op_pool()};
std::vector<uint32_t> detachedOps; // freed by the application, still running

bool handlesWrapped = false; // once the counter has wrapped, skip handles still in use

MPI_Request add(std::unique_ptr<Op> op) {
  if (handlesWrapped)
    while (active.count(nextHandle) || nextHandle == 0) nextHandle = (nextHandle + 1) % kHandleSpace;
  const uint32_t h = nextHandle;
  nextHandle = (nextHandle + 1) % kHandleSpace;
  if (nextHandle == 0) {
    nextHandle = 1;
    handlesWrapped = true;
  }
  active.emplace(h, std::move(op));
  return MPI_Request(h);
}

// scratch for progress()
std::vector<MPI_Request> pollReqs;
std::vector<Op *> pollOps;   // nullptr: a pending ack
std::vector<PendingAck *> pollAck; // the pending ack of each request (nullptr: an op's)
int progressDepth = 0;             // progress() passes on the stack
std::vector<int> pollIdx;
std::vector<MPI_Status> pollSt;

} // namespace

int collectiveDepth = 0;

void init() {
  gpu::choose_lanes(topology::ranks_on_node());
  gpuAwareLibrary = std::getenv("TEMPI_MPI_GPU_AWARE") != nullptr;
  directEnabled = std::getenv("TEMPI_NO_DIRECT") == nullptr;
  ipcSystemLoads = std::getenv("TEMPI_IPC_PLAIN_LOADS") == nullptr;
  hostRecvAware = std::getenv("TEMPI_NO_HOST_RECV") == nullptr;
  selfChannelEnabled = directEnabled && std::getenv("TEMPI_NO_SELF_CHANNEL") == nullptr; // it carries direct sends
  selfChannels.clear();
  faultCanary = std::getenv("TEMPI_FAULT_CANARY") != nullptr;
  canaryVerdict.clear();
  ipcCopyEnabled = std::getenv("TEMPI_NO_IPC_COPY") == nullptr;
  collCopyEnabled = std::getenv("TEMPI_NO_COLL_COPY") == nullptr;
  if (const char *s = std::getenv("TEMPI_IPC_COPY_MIN_BYTES")) ipcCopyMinBytes = std::atoll(s);
  if (const char *s = std::getenv("TEMPI_IPC_COPY_MIN_BLOCK")) ipcCopyMinBlock = std::atoll(s);
  if (const char *s = std::getenv("TEMPI_EARLY_FLUSH")) earlyFlush = size_t(std::max(1, std::atoi(s)));
  firstFlush = std::min<size_t>(16, earlyFlush);
  if (const char *s = std::getenv("TEMPI_FIRST_FLUSH")) firstFlush = size_t(std::max(1, std::atoi(s)));
  scattersInFlight = 0;
  eagerFlush = std::getenv("TEMPI_EAGER_FLUSH") != nullptr;
  directShared.clear();
  directShared.reserve(512);
  active.reserve(2048);
  systemPerformanceLoaded = import_system_performance(&systemPerformance);
  modelCache.clear();
  if (const char *s = std::getenv("TEMPI_IPC_MIN_BYTES")) ipcMinBytes = std::atoll(s);
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
  modelCache.clear();
}

void finalize() {
  // complete everything the application left behind, then wait (bounded) for
  // the acks that let us release IPC slabs
  const auto t0 = std::chrono::steady_clock::now();
  auto all_done = [] {
    for (auto &kv : active)
      if (!kv.second->done) return false;
    return true;
  };
  while (!all_done()) {
    progress();
    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(30)) {
      LOG_WARN("request(s) left incomplete at MPI_Finalize");
      break;
    }
  }
  selfChannels.clear(); // (receives still waiting there die with `active`)
  active.clear();
  detachedOps.clear();
  gates.clear();
  gatedOps = 0;
  libWatch.clear();
  boardOps.clear(); // (their ops died with `active`)
  for (auto &b : batches)
    if (b->event) tempi_hip_event_destroy(b->event);
  batches.clear();
  scattersInFlight = 0;
  while (!pendingAcks.empty()) {
    progress();
    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(30)) {
      LOG_WARN(pendingAcks.size() << " IPC slab(s) never acknowledged; abandoning");
      for (auto &pa : pendingAcks)
        if (pa->req != MPI_REQUEST_NULL) MPI_Cancel(&pa->req);
      pendingAcks.clear();
    }
  }
  for (void *e : eventPool) tempi_hip_event_destroy(e);
  eventPool.clear();
  for (auto &kv : ipcOpen) tempi_hip_ipc_close_handle(kv.second);
  ipcOpen.clear();
  for (auto &kv : ipcAllocOpen) tempi_hip_ipc_close_handle(kv.second.base);
  ipcAllocOpen.clear();
  ipcExports.clear();
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

namespace {
// packed bytes of `count` elements: the type size for a strided record
// (homogeneous MPI_Pack_size adds no header), else the library's answer
int64_t packed_bytes(const TypeRecord *rec, int count, MPI_Datatype dt, MPI_Comm comm) {
  if (rec->desc.valid) return rec->desc.size * int64_t(count);
  return pack_size(count, dt, comm);
}
} // namespace

int isend(const void *buf, int count, MPI_Datatype dt, int dest, int tag, MPI_Comm comm, MPI_Request *req,
          const Route &route, int force, bool blocking) {
  const TypeRecord *rec = route.rec;
  ScopedNs timer(counters.ns_isend);
  if (pendingPack.size() >= kMaxPending) flush(); // (no progress(): consecutive Isends share a launch)
  counters.isends++;
  if (!rec->packer) {
    self_spill(comm, dest);
    *req = add(std::make_unique<LibIsendOp>(buf, count, dt, dest, tag, comm));
    return MPI_SUCCESS;
  }
  const gpu::Ptr &p = route.ptr;
  const int64_t bytes = packed_bytes(rec, count, dt, comm);
  const char *origin = static_cast<const char *>(p.dptr) - rec->desc.start;
  const int destWorld = topology::world_rank(comm, dest);
  // a non-blocking send to this same process: the receiver copies directly
  tempi_hip_desc flat;
  if (directEnabled && !blocking && force < 0 && destWorld == state.worldRank && rec->flat(count, &flat)) {
    counters.send_direct++;
    *req = add(std::make_unique<IsendDirectOp>(rec, origin, count, dt, dest, tag, comm, p.device, bytes, flat));
    return MPI_SUCCESS;
  }
  if (destWorld == state.worldRank) spill_channel(comm); // a message to this rank the self channel cannot carry
  const bool colocated = topology::colocated_world(destWorld);
  modelBlock = std::min<int64_t>(std::max<int64_t>(1, rec->desc.block), 512);
  Method m = choose(bytes, colocated);
  if (force >= 0) m = Method(force);
  if (m == Method::IPC && (!colocated || ipc_broken(destWorld))) m = Method::ONESHOT;
  if (m == Method::DEVICE && !gpuAwareLibrary) m = colocated ? Method::IPC : Method::STAGED;
  switch (m) {
  case Method::ONESHOT: counters.send_oneshot++; break;
  case Method::STAGED: counters.send_staged++; break;
  case Method::DEVICE: counters.send_device++; break;
  case Method::IPC: counters.send_ipc++; break;
  default: break;
  }
  // IPC COPY: a large message of wide rows is copied by the receiver straight
  // out of this process's object (no gather, no slab)
  const int64_t copyMin = (collectiveDepth > 0 && collCopyEnabled) ? 1 : ipcCopyMinBytes;
  if (m == Method::IPC && ipcCopyEnabled && bytes >= copyMin && rec->flat(count, &flat) &&
      flat.ndims <= 3 && flat.block >= ipcCopyMinBlock && bytes < (int64_t(1) << 31)) {
    IpcCopyDesc d{};
    d.magic[0] = kMagicCopy;
    d.magic[1] = kMagic1;
    d.bytes = bytes;
    d.senderWorld = state.worldRank;
    d.senderPid = int32_t(getpid());
    d.device = p.device;
    d.rawFirst = reinterpret_cast<uint64_t>(origin + rec->desc.start);
    d.desc = flat;
    d.gpu = gpu::identity(p.device);
    const int half = std::max(1, tagUb / 2);
    d.ackTag = half + int32_t(nextCopyTag++ % uint32_t(half)); // slab ids (the IPC acks) stay below
    if (export_object(origin + rec->desc.start, &d)) {
      counters.send_ipc_copy++;
      *req = add(std::make_unique<IsendCopyOp>(rec, origin, count, dt, dest, tag, comm, p.device, bytes, destWorld, d));
      return MPI_SUCCESS;
    }
  }
  int cur = 0;
  tempi_hip_get_device(&cur);
  if (cur != p.device) tempi_hip_set_device(p.device);
  *req = add(std::make_unique<IsendOp>(rec, origin, count, dt, dest, tag, comm, p.device, m, bytes));
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
    *req = add(std::make_unique<LibIrecvOp>(buf, count, dt, source, tag, comm, nullptr, std::move(pre)));
    return MPI_SUCCESS;
  }
  const gpu::Ptr &p = route.ptr;
  const int64_t bytes = packed_bytes(rec, count, dt, comm);
  char *origin = static_cast<char *>(p.dptr) - rec->desc.start;
  *req = add(std::make_unique<IrecvOp>(rec, origin, count, dt, source, tag, comm, p.device, bytes, nullptr,
                                       std::move(pre)));
  // keep the GPU busy while the caller is still posting: launch arrived
  // messages' copies / unpacks once a launch's worth has queued up
  // (sooner while the GPU has no scatter work: the first batch starts early)
  if (pendingUnpack.size() >= (scattersInFlight ? earlyFlush : firstFlush)) flush_list(pendingUnpack, false);
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
  return add(std::make_unique<LocalCopyOp>(plan));
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

void self_forget(MPI_Comm comm) {
  auto it = selfChannels.find(comm_key(comm));
  if (it == selfChannels.end()) return;
  spill_channel(comm);
  selfChannels.erase(it);
}

int isend_host(const void *buf, int count, MPI_Datatype dt, int dest, int tag, MPI_Comm comm, MPI_Request *req) {
  counters.lib_sends++;
  *req = add(std::make_unique<HostIsendOp>(buf, count, dt, dest, tag, comm));
  return MPI_SUCCESS;
}

void drain_sends(MPI_Comm comm, int dest) {
  const uint64_t key = gate_key(comm, dest);
  while (gate_busy(key)) progress();
}

bool is_tempi_request(MPI_Request r) {
  const uint32_t h = uint32_t(r);
  return h != 0 && h < kHandleSpace && active.count(h);
}

bool peek(MPI_Request r) {
  auto it = active.find(uint32_t(r));
  return it != active.end() && it->second->done;
}

void release(MPI_Request *req) {
  auto it = active.find(uint32_t(*req));
  if (it != active.end()) {
    if (it->second->done) {
      active.erase(it);
    } else {
      it->second->detached = true;
      detachedOps.push_back(uint32_t(*req));
    }
  }
  *req = MPI_REQUEST_NULL;
}

int get_status(MPI_Request r, int *flag, MPI_Status *status) {
  auto it = active.find(uint32_t(r));
  if (it == active.end()) return next.MPI_Request_get_status(r, flag, status);
  progress();
  *flag = it->second->done ? 1 : 0;
  if (*flag) it->second->status(status);
  return MPI_SUCCESS;
}

int cancel(MPI_Request r) {
  auto it = active.find(uint32_t(r));
  if (it != active.end()) it->second->cancel();
  return MPI_SUCCESS;
}

namespace {
// Queued scatters / copies are launched by a waiting pass only while a
// scatter lane is free, or once a launch's worth has queued: with every lane
// busy the GPU has work either way, and messages arriving one at a time then
// share a launch instead of each taking one (a cheap pass -- no library
// request to test -- would otherwise launch every arrival on its own).
bool scatter_flush_due() {
  return eagerFlush || scattersInFlight < std::max(1, gpu::lanes() - 1) || pendingUnpack.size() >= earlyFlush;
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
    const int q = tempi_hip_event_query(b->event);
    if (q == 1) {
      blocked |= bit;
      continue;
    }
    gpu::check(q, "event query");
    put_event(b->event);
    b->event = nullptr;
    b->complete = true;
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
      auto it = active.find(h);
      if (it == active.end()) continue;
      if (it->second->done)
        active.erase(it);
      else
        detachedOps[w++] = h;
    }
    detachedOps.resize(w);
  }
  return moved;
}

bool busy() { return !active.empty() || !pendingAcks.empty(); }

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
  auto it = active.find(h);
  if (it == active.end()) return next.MPI_Wait(req, status);
  ScopedNs timer(counters.ns_wait);
  Op *op = it->second.get();
  while (!op->done) {
    progress();
    if (!op->done) op->stalled();
  }
  it->second->status(status);
  const int err = op->err;
  const MPI_Comm ec = op->errComm;
  active.erase(it);
  *req = MPI_REQUEST_NULL;
  return finish_error(err, ec);
}

int test(MPI_Request *req, int *flag, MPI_Status *status) {
  const uint32_t h = uint32_t(*req);
  auto it = active.find(h);
  if (it == active.end()) return next.MPI_Test(req, flag, status);
  progress();
  if (!it->second->done) it->second->stalled();
  *flag = it->second->done ? 1 : 0;
  if (*flag) {
    it->second->status(status);
    const int err = it->second->err;
    const MPI_Comm ec = it->second->errComm;
    active.erase(it);
    *req = MPI_REQUEST_NULL;
    return finish_error(err, ec);
  }
  return MPI_SUCCESS;
}

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
  }
  int n = 0;
  MPI_Get_count(&st, MPI_BYTE, &n);
  if (size_t(n) != sizeof(IpcDesc) && size_t(n) != sizeof(DirectDesc) && size_t(n) != sizeof(IpcCopyDesc))
    return next.MPI_Mrecv(buf, count, dt, &msg, status);
  alignas(16) char raw[kDescCap];
  next.MPI_Mrecv(raw, n, MPI_BYTE, &msg, &st);
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
  if (!hostRecvAware) return false; // TEMPI_NO_HOST_RECV (A/B only): host receives straight to the library
  return source == MPI_ANY_SOURCE || topology::colocated(comm, source);
}

int irecv_host(void *buf, int count, MPI_Datatype dt, int source, int tag, MPI_Comm comm, MPI_Request *req) {
  counters.lib_recvs++;
  self_spill(comm, source);
  *req = add(std::make_unique<HostIrecvOp>(buf, count, dt, source, tag, comm, take_probed(source, tag, comm)));
  return MPI_SUCCESS;
}

namespace {
bool descriptor_sized(int n) {
  return size_t(n) == sizeof(IpcDesc) || size_t(n) == sizeof(DirectDesc) || size_t(n) == sizeof(IpcCopyDesc);
}

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
void hold_through(int src, int tag, MPI_Comm comm) {
  for (;;) {
    MPI_Message m = MPI_MESSAGE_NULL;
    MPI_Status st;
    int g = 0;
    next.MPI_Improbe(src, MPI_ANY_TAG, comm, &g, &m, &st); // the earliest message of src
    if (!g) LOG_FATAL("a probed message could not be matched");
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
    return flag ? next.MPI_Iprobe(source, tag, comm, flag, status) : next.MPI_Probe(source, tag, comm, status);
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
      rc = next.MPI_Probe(source, tag, comm, &st);
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
  }
}

int mprobe(int source, int tag, MPI_Comm comm, int *flag, MPI_Message *msg, MPI_Status *status) {
  if (source == MPI_PROC_NULL || !state.active || !gpu::available()) // no descriptors can arrive
    return flag ? next.MPI_Improbe(source, tag, comm, flag, msg, status) : next.MPI_Mprobe(source, tag, comm, msg, status);
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
      rc = next.MPI_Mprobe(source, tag, comm, &m, &st);
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
      *req = add(std::make_unique<LibIrecvOp>(buf, count, dt, MPI_ANY_SOURCE, MPI_ANY_TAG, mc, msg));
    } else {
      const int64_t bytes = packed_bytes(route.rec, count, dt, mc);
      char *origin = static_cast<char *>(route.ptr.dptr) - route.rec->desc.start;
      *req = add(std::make_unique<IrecvOp>(route.rec, origin, count, dt, MPI_ANY_SOURCE, MPI_ANY_TAG, mc,
                                           route.ptr.device, bytes, msg));
    }
    *msg = MPI_MESSAGE_NULL;
    return MPI_SUCCESS;
  }
  std::unique_ptr<Probed> p = std::move(it->second);
  probedMsgs.erase(it);
  *msg = MPI_MESSAGE_NULL;
  const MPI_Comm comm = p->comm;
  if (!handles(buf, count, dt, 0, &route)) {
    *req = add(std::make_unique<HostIrecvOp>(buf, count, dt, MPI_ANY_SOURCE, MPI_ANY_TAG, comm, std::move(p)));
    return MPI_SUCCESS;
  }
  counters.irecvs++;
  if (!route.rec->packer) {
    *req = add(std::make_unique<LibIrecvOp>(buf, count, dt, MPI_ANY_SOURCE, MPI_ANY_TAG, comm, nullptr, std::move(p)));
    return MPI_SUCCESS;
  }
  const int64_t bytes = packed_bytes(route.rec, count, dt, comm);
  char *origin = static_cast<char *>(route.ptr.dptr) - route.rec->desc.start;
  *req = add(std::make_unique<IrecvOp>(route.rec, origin, count, dt, MPI_ANY_SOURCE, MPI_ANY_TAG, comm,
                                       route.ptr.device, bytes, nullptr, std::move(p)));
  return MPI_SUCCESS;
}

int mrecv(void *buf, int count, MPI_Datatype dt, MPI_Message *msg, MPI_Status *status) {
  Route route;
  if (!probedMsgs.count(uint32_t(*msg)) && !handles(buf, count, dt, 0, &route)) {
    libMsgComm.erase(*msg);
    return next.MPI_Mrecv(buf, count, dt, msg, status); // the library's message into host memory
  }
  MPI_Request r = MPI_REQUEST_NULL;
  const int rc = imrecv(buf, count, dt, msg, &r);
  if (rc != MPI_SUCCESS) return rc;
  return is_tempi_request(r) ? wait(&r, status) : next.MPI_Wait(&r, status);
}

} // namespace p2p
} // namespace tempi
