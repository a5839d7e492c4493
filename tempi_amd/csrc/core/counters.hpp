// tempi_amd/csrc/core/counters.hpp -- per-process operation counters, the
// equivalent of the reference's always-on counters
// (/root/reference/include/counters.hpp:8-115, dumped at MPI_Finalize by
// /root/reference/src/internal/counters.cpp:30-121). Read them through
// tempi_get_counters() (include/tempi_ext.h) or TEMPI_LOG_LEVEL=DEBUG.
#pragma once

#include <cstdint>

namespace tempi {

struct Counters {
  uint64_t packs = 0, unpacks = 0;
  uint64_t pack_bytes = 0, unpack_bytes = 0;
  uint64_t launches = 0;
  uint64_t lib_packs = 0, lib_unpacks = 0; // handed to the library
  // GPU packs into / unpacks from pageable host memory through a pinned slab
  uint64_t staged_packs = 0, staged_unpacks = 0;
  // synchronous MPI_Pack / MPI_Unpack completed by a ticket (device memory or
  // TEMPI's coherent slab written) or by hipStreamSynchronize (the
  // application's pinned host memory written)
  uint64_t ticket_waits = 0, sync_waits = 0;
  uint64_t ticket_batches = 0; // transport batches completed by a ticket their last launch stored
  uint64_t persistent_starts = 0; // MPI_Start of a TEMPI persistent request
  uint64_t sends = 0, recvs = 0, isends = 0, irecvs = 0;
  uint64_t send_device = 0, send_oneshot = 0, send_staged = 0, send_ipc = 0;
  uint64_t lib_sends = 0, lib_recvs = 0;
  // sends to this same process: strided->strided copies, and those that
  // had to be packed because their wait came before the matching receive
  uint64_t send_direct = 0, direct_fallbacks = 0;
  uint64_t neighbor_colls = 0; // neighbourhood collectives on device buffers
  uint64_t send_ipc_copy = 0, copy_resends = 0; // IPC COPY sends; those answered through the host
  uint64_t ipc_maps_replaced = 0; // peer allocation mappings closed because the peer replaced them
  // first contact with a peer on another GPU: its memory read back through
  // the remote-load kernel agreed with a DMA read (ok) or did not (fail)
  uint64_t canary_ok = 0, canary_fail = 0;
  uint64_t self_matched = 0; // messages to this process matched in TEMPI's self channel
  // payload bytes of device-object sends by route: IPC
  // (IPC COPY included, and counted again on its own), ONESHOT, STAGED,
  // DEVICE (a GPU-aware library) and DIRECT (this same process)
  uint64_t bytes_ipc = 0, bytes_ipc_copy = 0, bytes_oneshot = 0, bytes_staged = 0, bytes_device = 0,
           bytes_direct = 0;
  // kernel time of synchronous MPI_Pack / MPI_Unpack while profiling is on
  double pack_kernel_ms = 0, unpack_kernel_ms = 0;
  uint64_t pack_timed = 0, unpack_timed = 0;
  // host time (ns) inside the transport, for TEMPI_PRINT_COUNTERS
  uint64_t ns_isend = 0, ns_irecv = 0, ns_flush = 0, ns_events = 0, ns_testsome = 0, ns_wait = 0;
  // neighbourhood collectives: plan lookup + posting the per-edge operations,
  // and the MPI_Waitall that completes them (the call is blocking)
  uint64_t ns_nbr_post = 0, ns_nbr_wait = 0;
  uint64_t progress_passes = 0, batches = 0, batched_items = 0;
  // time (ns) with at least one transport batch in flight by the host's own
  // account: from a batched launch's return to that batch observed complete
  // (always on: two clock reads per batch)
  uint64_t ns_gpu_inflight = 0;
};

extern Counters counters;
extern bool kernelProfiling;
// settle the kernel-profiling events still pending (interpose_core.cpp)
void settle_kernel_times();
void *timing_event(int device);
void timed(int device, bool pack, void *ev0, void *ev1, bool ok);
void destroy_timing_events();
// the ns_* host timers run only when asked for (TEMPI_PRINT_COUNTERS): a
// clock read is ~20 ns, several per message
extern bool hostTiming;

uint64_t now_ns();
inline uint64_t tick() { return hostTiming ? now_ns() : 0; }
inline void tock(uint64_t &acc, uint64_t t0) {
  if (hostTiming) acc += now_ns() - t0;
}
struct ScopedNs {
  uint64_t &acc;
  uint64_t t0;
  explicit ScopedNs(uint64_t &a) : acc(a), t0(tick()) {}
  ~ScopedNs() { tock(acc, t0); }
};

} // namespace tempi
