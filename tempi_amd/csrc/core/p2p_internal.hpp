// tempi_amd/csrc/core/p2p_internal.hpp -- what the transport's translation
// units share (p2p.hpp is the interface the interposer sees).
//
//   p2p.cpp         request table, init / finalize, isend / irecv routing,
//                   progress(), wait / test
//   p2p_board.cpp   the shared-memory ack board and the slabs awaiting acks
//   p2p_routes.cpp  method choice, descriptors (IPC, IPC COPY, DIRECT), peer
//                   mappings, the first-contact canary, landing descriptors in
//                   host memory
//   p2p_ops.cpp     operation plumbing (events, batches, watch list, send
//                   gates, pending GPU work) and the send state machines
//   p2p_recv.cpp    the receive state machines and the self channel
//   p2p_probe.cpp   the probe family, held messages, host receives
//
// Reference counterpart of the whole: /root/reference/src/internal/
// async_operation.cpp:71-521 and sender.cpp:26-328 (see p2p.hpp).
#pragma once

#include "alloc.hpp"
#include "p2p.hpp"
#include "type_cache.hpp"

#include "tempi_hip.h"

#include <mpi.h>

#include <cstddef>
#include <cstdint>
#include <deque>
#include <map>
#include <memory>
#include <memory_resource>
#include <tuple>
#include <unordered_map>
#include <vector>

namespace tempi {
class Packer;
namespace p2p {

enum class Method { ONESHOT, STAGED, DEVICE, IPC, LIBPACK };

namespace detail {

// ------------------------------------------------------------- descriptors

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

constexpr size_t kDescCap = sizeof(IpcCopyDesc) > sizeof(DirectDesc)
                                ? (sizeof(IpcCopyDesc) > sizeof(IpcDesc) ? sizeof(IpcCopyDesc) : sizeof(IpcDesc))
                                : (sizeof(DirectDesc) > sizeof(IpcDesc) ? sizeof(DirectDesc) : sizeof(IpcDesc));

bool is_direct(const void *msg, int n);
bool is_ipc_copy(const void *msg, int n);
bool is_ipc(const void *msg, int n);
bool is_descriptor(const void *msg, int n);
// the payload a descriptor-sized message stands for (n for anything else)
int64_t descriptor_payload(const void *msg, int n);
bool descriptor_sized(int n);

// ------------------------------------------------------------ shared state

// Operation objects, the shared state of direct sends and the request table
// are carved from one unsynchronised pool (the transport runs on the MPI
// thread only), so a message's bookkeeping costs no malloc / free. The pool
// is never destroyed: objects that outlive MPI_Finalize (statics torn down at
// exit) still return their memory to it.
std::pmr::unsynchronized_pool_resource &op_pool();

struct Op;
struct DirectShared {
  DirectDesc desc{}; // the library's send buffer: alive until the receiver claims it
  enum State { PENDING, CLAIMED, PACKED, DONE } state = PENDING;
  Slab *slab = nullptr; // PACKED: the sender's gather (released by the receiver)
  bool gathered = false; // PACKED: that gather's batch has been seen complete
  int device = 0;
  Op *sender = nullptr; // while the send is incomplete
};
extern std::unordered_map<uint64_t, std::shared_ptr<DirectShared>> directShared; // sent, not yet matched
extern uint64_t nextDirectToken;
extern bool directEnabled;

extern MPI_Comm ctrlComm; // private duplicate of MPI_COMM_WORLD for acks
extern int tagUb;
extern bool gpuAwareLibrary;
extern int64_t ipcMinBytes;

// TEMPI request handles live in [1, 2^26): the top bits of an MPICH handle
// always encode a non-zero kind, so the library never issues one of these
// (the reference uses a plain counter that can collide: SURVEY F9). TEMPI
// message handles (MPI_Mprobe) use the same space.
constexpr uint32_t kHandleSpace = 1u << 26;

// --------------------------------------------------- ack board (p2p_board)

struct AckBoard {
  MPI_Comm node = MPI_COMM_NULL;
  MPI_Win win = MPI_WIN_NULL;
  std::vector<uint32_t *> of; // per world rank: its slots (nullptr: not on this board)
  std::vector<int> freeSlots;
  int slots = 0; // 0: off
};
extern AckBoard board;
// a free slot of this rank's board for a message to world rank `peer`, or -1
int board_take(int peer);
void board_give(int slot); // a slot taken for a message that was never sent
// the ack code in this rank's slot (and the slot freed), or -1 until it arrives
int board_poll(int slot);
void board_init();
void board_finalize();

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
extern std::vector<std::unique_ptr<PendingAck>> pendingAcks; // stable addresses: Irecv targets

// ack payload of an IPC slab: 0 = pulled, release the slab; 1 = could not map
// it, send the bytes through the host on (ctrlComm, ackTag)
void send_ack(int world, int tag, int code);
void send_ack(const IpcDesc &d, int code = 0);

// IPC COPY acks: 0 = copied; 1 = cannot copy this shape, send the packed
// bytes through the host on (ctrlComm, ackTag); 2 = the same, and the
// sender's memory could not be mapped (no more IPC with that rank)
enum { kCopyDone = 0, kCopyResend = 1, kCopyUnmapped = 2 };

// ------------------------------------------------------ routes (p2p_routes)

extern bool ipcCopyEnabled;     // TEMPI_NO_IPC_COPY
extern int64_t ipcCopyMinBytes; // TEMPI_IPC_COPY_MIN_BYTES
extern int64_t ipcCopyMinBlock; // TEMPI_IPC_COPY_MIN_BLOCK
extern uint32_t nextCopyTag;
extern bool faultCanary;        // TEMPI_FAULT_CANARY
extern int64_t modelBlock;      // block length of the type being sent (set per call)

// an application datatype kept valid while an operation needs it
MPI_Datatype hold_type(MPI_Datatype t);
void drop_type(MPI_Datatype t);
// the status of a completed receive: `bytes` received
void set_received(MPI_Status *s, int64_t bytes);
int64_t pack_size(int count, MPI_Datatype dt, MPI_Comm comm);
// packed bytes of `count` elements: the type size for a strided record
// (homogeneous MPI_Pack_size adds no header), else the library's answer
int64_t packed_bytes(const TypeRecord *rec, int count, MPI_Datatype dt, MPI_Comm comm);

// the method for a message (TEMPI_DATATYPE_* or AUTO; AUTO prices only
// blocking sends by the measured model, see p2p_routes.cpp)
Method choose(int64_t bytes, bool colocated, bool blocking);
void clear_model_cache();

bool ipc_broken(int world);
void mark_ipc_broken(int world);
void *peer_pointer(const IpcDesc &d);
bool canary(int world, const void *peerBytes, int64_t n, int device);
void clear_canary();
const char *peer_object(const IpcCopyDesc &d);
bool export_object(const void *first, IpcCopyDesc *d);
// Peer allocations stay mapped for reuse; past a bound every mapping is
// closed (after the copies that may still read them have run)
void recycle_alloc_maps();
// every peer mapping and export closed (MPI_Finalize)
void close_mappings();

void direct_finish(std::shared_ptr<DirectShared> &sh);
std::shared_ptr<DirectShared> claim_direct(const DirectDesc &d);
void materialise_direct(std::shared_ptr<DirectShared> &sh, const DirectDesc &d, Slab *dst);
void land_descriptor(const void *msg, int n, std::vector<char> &out);
int land_host(const char *msg, int n, void *buf, int count, MPI_Datatype dt, MPI_Comm comm, int64_t *received);

int64_t desc_bytes(const tempi_hip_desc &d);
bool copy_ok(const tempi_hip_desc &dst, const tempi_hip_desc &src);

// ---------------------------------------------------- operations (p2p_ops)

// one batched launch (+ its trailing copies) and how its completion is seen:
// the ticket its last launch stores (flag != nullptr), or an event behind it
struct GpuBatch {
  const uint32_t *flag = nullptr; // ticket flag (pinned host memory)
  uint32_t ticket = 0;
  uint32_t polls = 0;             // ticket polls so far (the stream is queried now and then)
  void *stream = nullptr;
  void *event = nullptr;
  int device = 0;
  int lane = 0;
  bool scatter = false;
  bool complete = false;
  std::vector<Op *> ops; // whose GPU work this batch carries (alive until gpu_done)
};
extern std::deque<std::shared_ptr<GpuBatch>> batches; // launch order

struct PersistentOp; // p2p_persistent.cpp

struct Op {
  virtual ~Op() { settle_buffered(); }
  virtual PersistentOp *persistent() { return nullptr; }
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
  // a buffered-mode send counts in bufferedUnposted (MPI_Buffer_detach waits
  // for it) from construction until its post() -- or its destruction, should
  // it never be posted, so that the detach cannot wait forever
  bool unpostedBuffered = false;
  void count_buffered();
  void settle_buffered();
};

// a library post of the application's message that the library refused
// (its arguments, under MPI_ERRORS_RETURN): the op completes with that error
// -- raised by its wait -- instead of waiting on a request that does not exist
void fail_post(Op *op, int rc, MPI_Comm comm);

void *get_event();
void put_event(void *e);
void destroy_events();

// ops waiting for an ack on this rank's board (polled by progress())
extern std::vector<Op *> boardOps;
// ops with a library request outstanding (tested together by progress()).
// Every post of Op::lib is followed by watch(op).
extern std::vector<Op *> libWatch;
void watch(Op *op);
void unwatch(Op *op);

// send order per (comm, dest): see p2p_ops.cpp
uint64_t gate_key(MPI_Comm comm, int dest);
bool gate_busy(uint64_t key);
void gate_enter(uint64_t key, Op *op);
void gate_advance(uint64_t key);
void post_or_queue(uint64_t key, Op *op);
void clear_gates();

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
  void add_items(const Op *op, const Packer &pk, void *packed, const void *origin, int64_t count);
  void add_copy(const Op *op, const tempi_hip_copy_item &c) {
    copies.push_back(c);
    copyDev.push_back(op->device);
  }
  void queue(Op *op) {
    op->queued = true;
    ops.push_back(op);
  }
};
extern PendingList pendingPack, pendingUnpack;
extern int64_t bufferedUnposted; // MPI_Ibsend-mode sends not yet handed to the library (MPI_Buffer_detach waits)
constexpr size_t kMaxPending = 512;
// queued scatters are launched by a light pass once this many have queued
// (kFirstFlush while no scatter batch is in flight: the GPU is idle then)
constexpr size_t kEarlyFlush = 32;
constexpr size_t kFirstFlush = 16;
extern int batchesInFlight;    // batches launched and not yet seen complete (any kind)
extern int scattersInFlight;   // scatter / copy batches launched and not yet seen complete
void flush_list(PendingList &list, bool pack);
// counters.ns_gpu_inflight bookkeeping: a batch launched / observed complete
void batch_launched();
void batch_observed_done();
void flush();

// the send state machines (p2p_ops.cpp)
std::unique_ptr<Op> new_isend(const TypeRecord *r, const char *origin, int count, MPI_Datatype dt, int dest, int tag,
                              MPI_Comm comm, int dev, Method m, int64_t bytes, SendMode mode);
std::unique_ptr<Op> new_isend_direct(const TypeRecord *r, const char *origin, int count, MPI_Datatype dt, int dest,
                                     int tag, MPI_Comm comm, int dev, int64_t bytes, const tempi_hip_desc &flat);
std::unique_ptr<Op> new_isend_copy(const TypeRecord *r, const char *origin, int count, MPI_Datatype dt, int dest,
                                   int tag, MPI_Comm comm, int dev, int64_t bytes, int peerWorld,
                                   const IpcCopyDesc &filled);
std::unique_ptr<Op> new_lib_isend(const void *buf, int count, MPI_Datatype dt, int dest, int tag, MPI_Comm comm,
                                  SendMode mode);
// the library send of a TEMPI message in the application's send mode
int lib_isend(SendMode mode, const void *buf, int count, MPI_Datatype dt, int dest, int tag, MPI_Comm comm,
              MPI_Request *req);
std::unique_ptr<Op> new_host_isend(const void *buf, int count, MPI_Datatype dt, int dest, int tag, MPI_Comm comm);
std::unique_ptr<Op> new_local_copies(const LocalCopies &plan);

// ------------------------------------------------- held messages (p2p_probe)

// A message a probe had to receive to look at it (it has a descriptor's
// size): it stays matchable, in arrival order, until a receive or probe takes
// it, or an MPI_Mprobe handle claims it.
struct Probed {
  MPI_Comm comm = MPI_COMM_NULL;
  MPI_Status st{};         // source and tag as the library reported them
  std::vector<char> bytes; // the message as received (MPI_BYTE)
  int64_t payload = 0;     // what the application receives (a descriptor's payload size)
};
// the earliest kept message a receive (source, tag, comm) matches, taken out
std::unique_ptr<Probed> take_probed(int source, int tag, MPI_Comm comm);

// ------------------------------------------------------ receives (p2p_recv)

// msg: receive this library message (MPI_Mrecv); pre: a message a probe
// already received (it is delivered at once)
std::unique_ptr<Op> new_irecv(const TypeRecord *r, char *origin, int count, MPI_Datatype dt, int source, int tag,
                              MPI_Comm comm, int dev, int64_t bytes, MPI_Message *msg = nullptr,
                              std::unique_ptr<Probed> pre = nullptr);
std::unique_ptr<Op> new_lib_irecv(void *buf, int count, MPI_Datatype dt, int source, int tag, MPI_Comm comm,
                                  MPI_Message *msg = nullptr, std::unique_ptr<Probed> pre = nullptr);
std::unique_ptr<Op> new_host_irecv(void *buf, int count, MPI_Datatype dt, int source, int tag, MPI_Comm comm,
                                   std::unique_ptr<Probed> pre);

// the self channel (p2p_recv.cpp): a direct send of this process to itself
// on `comm` matched to a waiting receive, or kept for a later one -- no
// library message (false: post the descriptor through the library)
extern bool selfChannelEnabled;
bool self_send(const std::shared_ptr<DirectShared> &sh, MPI_Comm comm, int tag);
void spill_channel(MPI_Comm comm);
bool forget_channel(MPI_Comm comm); // false when comm had no channel
void clear_channels();

// ---------------------------------------------------- request table (p2p.cpp)

MPI_Request add(std::unique_ptr<Op> op);

// the op behind a TEMPI request (nullptr: not one)
Op *find_op(MPI_Request r);
// persistent requests (p2p_persistent.cpp): the completion family's side
extern int persistent_count; // PersistentOps in the request table
int persistent_wait(PersistentOp *p, MPI_Status *status);
int persistent_test(PersistentOp *p, int *flag, MPI_Status *status);
bool persistent_peek(PersistentOp *p);
int persistent_get_status(PersistentOp *p, int *flag, MPI_Status *status);
int persistent_cancel(PersistentOp *p);
void persistent_free(PersistentOp *p); // before the request is dropped

} // namespace detail
} // namespace p2p
} // namespace tempi
