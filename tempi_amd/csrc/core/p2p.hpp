// tempi_amd/csrc/core/p2p.hpp -- strided point-to-point transfers of device
// buffers: method selection and the Isend / Irecv state machines.
//
// Reference counterparts: the blocking senders (/root/reference/src/internal/
// sender.cpp:26-328: DEVICE / ONE_SHOT / STAGED, AUTO by model) and the async
// operations (/root/reference/src/internal/async_operation.cpp:71-521:
// Isend = pack -> event -> MPI_Start of a persistent send; Irecv = MPI_Irecv ->
// MPI_Test -> unpack).
//
// Methods (TEMPI_DATATYPE_*; every method sends the same wire format, the
// packed bytes as MPI_PACKED, except IPC):
//   ONESHOT  the pack kernel writes straight into pinned, mapped host memory,
//            the library sends it; the receiver's unpack kernel reads the
//            received pinned buffer directly
//   STAGED   pack into device memory, copy to pinned host, library send
//   DEVICE   pack into device memory and hand the device buffer to the library
//            (needs a GPU-aware MPI: TEMPI_MPI_GPU_AWARE=1). Without one, the
//            DEVICE choice is carried out by IPC for co-located peers, STAGED
//            otherwise
//   IPC      (MI355X-native, intra-node) pack into a device slab, send a
//            128-byte descriptor (IPC handle + offset) through the library;
//            the receiver maps the sender's slab and its unpack kernel reads
//            the packed bytes over xGMI, then acknowledges so the sender can
//            reuse the slab
//   DIRECT   (sends to the same process, non-blocking only) the descriptor
//            names the sender's object; the receiver copies it strided ->
//            strided with one kernel (no packed intermediate); a send waited
//            on before its receive is posted falls back to a gathered slab.
//            TEMPI_NO_DIRECT disables it
//   AUTO     blocking sends: the cheapest method the perf model prices
//            (perf.json); otherwise IPC for co-located peers at >= 4 KiB,
//            ONESHOT otherwise (with no perf.json the reference would stop
//            here with LOG_FATAL: SURVEY F10)
// Receives are adaptive: a TEMPI device receive lands in pinned host memory
// and recognises an IPC descriptor by size + 16-byte magic, so it works with
// any sender method. Host receives (MPI_Recv, MPI_Irecv, MPI_Sendrecv, the
// collectives' host blocks) and the probe family recognise descriptors too,
// so an application never sees one.
#pragma once

#include "gpu.hpp"
#include "type_cache.hpp"

#include <mpi.h>

#include <vector>

namespace tempi {
struct TypeRecord;
namespace p2p {

void init();
void finalize();
// re-read the perf model (after measure_system wrote this node's perf.json)
void reload_perf_model();
// the route a strided message would take (tempi_choose_method): 1 ONESHOT,
// 2 DEVICE, 3 STAGED, 4 IPC; *fromModel set when the perf model decided
// the IPC / ONESHOT threshold non-blocking AUTO sends of `block`-byte blocks
// use; *fromModel when it was priced from this node's perf.json
int64_t query_ipc_threshold(int64_t block, bool *fromModel);
int query_method(int64_t bytes, int64_t block, bool colocated, bool blocking, bool *fromModel);

// what handles() found out, handed on to isend / irecv
struct Route {
  const TypeRecord *rec = nullptr;
  gpu::Ptr ptr; // the first byte the type touches
};

// true when TEMPI handles this send / receive (otherwise: library)
bool handles(const void *buf, int count, MPI_Datatype dt, int peer, Route *route);

// A collective that posts every receive before it waits on any send
// (MPI_Alltoallv) opens this scope; inside it IPC COPY (a rendezvous: the
// send completes when the receiver has copied) is used at every message size
extern int collectiveDepth;
struct CollectiveScope {
  CollectiveScope() { ++collectiveDepth; }
  ~CollectiveScope() { --collectiveDepth; }
  CollectiveScope(const CollectiveScope &) = delete;
  CollectiveScope &operator=(const CollectiveScope &) = delete;
};

// MPI's send modes. A TEMPI send hands the library one message (the packed
// bytes or a descriptor) with the matching library call: MPI_Issend for
// SYNC (the send completes once a receive has matched it), MPI_Ibsend for
// BUFFERED (local completion, from the application's attached buffer),
// MPI_Isend for STANDARD and READY (a standard send is a valid ready send).
// SYNC never takes the DIRECT route (a stalled direct send completes alone);
// BUFFERED takes neither DIRECT nor IPC COPY (rendezvous) nor a descriptor
// larger than its payload (the attached buffer is sized for the payload).
enum class SendMode { STANDARD, SYNC, BUFFERED, READY };

// force: -1 = choose by TEMPI_DATATYPE_* / AUTO; else a forced method
// (0 ONESHOT, 1 STAGED, 2 DEVICE, 3 IPC)
// blocking = true (MPI_Send) never takes the DIRECT route, whose completion
// needs the matching receive
int isend(const void *buf, int count, MPI_Datatype dt, int dest, int tag, MPI_Comm comm, MPI_Request *req,
          const Route &route, int force = -1, bool blocking = false, SendMode mode = SendMode::STANDARD);
int irecv(void *buf, int count, MPI_Datatype dt, int source, int tag, MPI_Comm comm, MPI_Request *req,
          const Route &route);

// Send order for sends TEMPI does not carry (host buffers): while an earlier
// TEMPI send to (comm, dest) is still gathering, a library send there would
// overtake it. send_gated() says so; isend_host() then queues the host send
// behind it (a TEMPI request) and drain_sends() waits until it has left.
// A message from this process to itself whose receive is known at the same
// time (a neighbourhood collective's self edge): one strided -> strided copy
// queued on the GPU, no library messages. False (nothing queued) when it
// cannot be one copy: host memory, unequal sizes, shapes the copy kernel does
// not take, different devices, TEMPI_NO_DIRECT. start_queued() launches what
// is queued.
bool local_copy(const void *sbuf, int scount, MPI_Datatype stype, void *rbuf, int rcount, MPI_Datatype rtype,
                MPI_Request *req);
void start_queued();
// The same copies planned once and started many times (a neighbourhood
// collective's self edges, cached per call signature): plan_local_copy
// appends one copy to `plan` (false, nothing appended, when local_copy would
// refuse it); start_local_copies queues all of them as ONE request.
struct LocalCopies {
  std::vector<tempi_hip_copy_item> items;
  std::vector<RecordRef> recs; // the copies' type records, held while planned
  int device = -1;
  int64_t bytes = 0;
};
bool plan_local_copy(const void *sbuf, int scount, MPI_Datatype stype, void *rbuf, int rcount, MPI_Datatype rtype,
                     LocalCopies *plan);
MPI_Request start_local_copies(const LocalCopies &plan);

// Messages of this process to itself are matched inside TEMPI while every
// such message of the communicator can be (p2p.cpp, "self channel"). An
// operation on a message to / from this rank that the channel cannot carry
// calls self_spill first: peer = the other end's rank in comm (a send's dest,
// a receive's or probe's source, MPI_ANY_SOURCE included); no-op for other
// ranks. self_forget drops the channel of a communicator being freed.
void self_spill(MPI_Comm comm, int peer);
void self_forget(MPI_Comm comm);

bool send_gated(MPI_Comm comm, int dest);
int isend_host(const void *buf, int count, MPI_Datatype dt, int dest, int tag, MPI_Comm comm, MPI_Request *req);
void drain_sends(MPI_Comm comm, int dest);
// progress until every buffered-mode send TEMPI holds has reached the library
void drain_buffered();

// Persistent requests (p2p_persistent.cpp): a TEMPI request remembering its
// arguments; start() posts the operation through the interposed MPI_Isend /
// MPI_Issend / MPI_Ibsend / MPI_Irsend / MPI_Irecv. wait / test / peek /
// get_status / cancel / release understand them; a completed one stays,
// inactive (inactive(): skipped like MPI_REQUEST_NULL by MPI_Testany,
// MPI_Waitany, MPI_Testsome, MPI_Waitsome).
int persistent_init(bool send, const void *buf, int count, MPI_Datatype dt, int peer, int tag, MPI_Comm comm,
                    SendMode mode, MPI_Request *req);
int start(MPI_Request *req);
bool inactive(MPI_Request r);

bool is_tempi_request(MPI_Request r);
// complete? (no progress, no release: MPI_Testall's all-or-nothing rule)
bool peek(MPI_Request r);
// MPI_Request_free: the operation finishes in the background; *req = NULL
void release(MPI_Request *req);
// MPI_Request_get_status: complete? (status filled when it is; the request
// stays until a wait / test / free)
int get_status(MPI_Request r, int *flag, MPI_Status *status);
// MPI_Cancel: a receive that nothing has matched yet is cancelled (its wait
// then returns a status for which MPI_Test_cancelled is true); any other
// operation completes normally, which MPI permits
int cancel(MPI_Request r);
// drive every TEMPI operation one step; returns true if anything moved.
// full = false (from MPI_Isend / MPI_Irecv) leaves arrived messages' unpacks
// queued so that a burst shares one launch; waits use full = true
bool progress(bool full = true);
bool busy(); // active operations or unacknowledged IPC slabs exist
int progress_depth(); // progress() passes on this call stack (mt.cpp: no lock hand-off inside one)

// complete a TEMPI request (blocking); fills status, sets *req to NULL
int wait(MPI_Request *req, MPI_Status *status);
// non-blocking: *flag = completion
int test(MPI_Request *req, int *flag, MPI_Status *status);

// blocking MPI_Recv into a host buffer that may receive an IPC descriptor
int recv_host_ipc_aware(void *buf, int count, MPI_Datatype dt, int source, int tag, MPI_Comm comm,
                        MPI_Status *status, bool *handled);

// ----------------------------------------------------- descriptor-aware receives
// A TEMPI device send to a co-located rank may travel as a descriptor (IPC
// slab, IPC COPY, DIRECT) instead of its bytes. Every receive an application
// can post must therefore see the payload, as it would with the reference's
// senders, which always send MPI_PACKED bytes (/root/reference/src/internal/
// sender.cpp:109,161, async_operation.cpp:127,261).
//
// true when a host-buffer receive from `source` could meet a descriptor
// (TEMPI active with a GPU, and the source is this node or MPI_ANY_SOURCE),
// or a message a probe is holding
bool host_recv_aware(int source, int tag, MPI_Comm comm);
// a probe holds a message a receive (source, tag, comm) would match
bool holds(int source, int tag, MPI_Comm comm);
// MPI_Irecv into host memory that recognises a descriptor and lands its bytes
int irecv_host(void *buf, int count, MPI_Datatype dt, int source, int tag, MPI_Comm comm, MPI_Request *req);
// MPI_Probe (flag == nullptr) / MPI_Iprobe: a descriptor is reported with its
// payload size (MPI_Get_count works on the status). To look at a message of a
// descriptor's size the probe must receive it; it is then kept, still
// matchable, and the next receive or probe that matches takes it from there.
int probe(int source, int tag, MPI_Comm comm, int *flag, MPI_Status *status);
// MPI_Mprobe (flag == nullptr) / MPI_Improbe: a descriptor becomes a TEMPI
// message handle (outside the library's handle space), the rest stay the
// library's
int mprobe(int source, int tag, MPI_Comm comm, int *flag, MPI_Message *msg, MPI_Status *status);
// MPI_Mrecv / MPI_Imrecv of either kind of message into host or device memory
int mrecv(void *buf, int count, MPI_Datatype dt, MPI_Message *msg, MPI_Status *status);
int imrecv(void *buf, int count, MPI_Datatype dt, MPI_Message *msg, MPI_Request *req);

} // namespace p2p
} // namespace tempi
