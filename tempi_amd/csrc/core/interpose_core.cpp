// tempi_amd/csrc/core/interpose_core.cpp -- interposed MPI_Init /
// MPI_Init_thread / MPI_Finalize / MPI_Type_commit / MPI_Type_free /
// MPI_Pack / MPI_Unpack (declared in include/tempi_mpi.h).
//
// Reference behaviour kept: env kill switches first, then dispatch to TEMPI
// only for committed strided types whose buffers the GPU can reach, else the
// library (/root/reference/src/pack.cpp:28-68, unpack.cpp:20-59,
// type_commit.cpp:16-114, type_free.cpp:14-27, init.cpp:22-65).
// Changed: the pointer test is done on the FIRST BYTE the type touches (the
// origin itself may lie outside the allocation for offset types), outsize /
// insize are checked (MPI_ERR_TRUNCATE instead of an overrun), a type with no
// strided form goes to the library instead of a null packer, and
// MPI_Init_thread is interposed too (F8).
#include "trace.hpp"
#include "alloc.hpp"
#include "counters.hpp"
#include "env.hpp"
#include "gpu.hpp"
#include "log.hpp"
#include "mt.hpp"
#include "next_mpi.hpp"
#include "state.hpp"
#include "p2p.hpp"
#include "topology.hpp"
#include "type_cache.hpp"

#include "tempi_mpi.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <unistd.h>
#include <cstring>
#include <vector>

#define TEMPI_EXPORT extern "C" __attribute__((visibility("default")))

namespace tempi {

void coll_init();
void coll_finalize();

State state;
Counters counters;
bool kernelProfiling = false;
bool hostTiming = false;

int raise_error(MPI_Comm comm, int code) {
  MPI_Comm_call_errhandler(comm, code);
  return code;
}


// Kernel profiling (tempi_set_kernel_profiling): each synchronous call's
// launches are bracketed by a pair of HIP timing events, and a pair is
// settled -- synchronised, its elapsed time added to the counters -- only when
// the times are read (tempi_get_kernel_times) or once kMaxTimed pairs are
// pending. Settling inside the call would add HIP's own completion latency
// (hipEventSynchronize, ~5 us) to every call, the latency the ticket wait
// exists to avoid, and bench.py times its headline with profiling on.
namespace {
struct Timed {
  void *ev0, *ev1;
  int device;
  bool pack;
};
std::vector<Timed> timedPending;
std::vector<std::vector<void *>> timedFree; // per device
constexpr size_t kMaxTimed = 512;
} // namespace

void *timing_event(int device) {
  if (device < 0) return nullptr;
  if (timedFree.size() <= size_t(device)) timedFree.resize(size_t(device) + 1);
  std::vector<void *> &f = timedFree[size_t(device)];
  if (!f.empty()) {
    void *e = f.back();
    f.pop_back();
    return e;
  }
  void *e = nullptr;
  return tempi_hip_event_create(&e, 1) == 0 ? e : nullptr;
}

void settle_kernel_times() {
  for (const Timed &t : timedPending) {
    float ms = 0;
    if (tempi_hip_event_synchronize(t.ev1) == 0 && tempi_hip_event_elapsed_ms(&ms, t.ev0, t.ev1) == 0) {
      if (t.pack) {
        counters.pack_kernel_ms += ms;
        counters.pack_timed++;
      } else {
        counters.unpack_kernel_ms += ms;
        counters.unpack_timed++;
      }
    }
    timedFree[size_t(t.device)].push_back(t.ev0);
    timedFree[size_t(t.device)].push_back(t.ev1);
  }
  timedPending.clear();
}

void timed(int device, bool pack, void *ev0, void *ev1, bool ok) {
  if (!ok) { // nothing to time: the events go back (re-recorded before any later read)
    timedFree[size_t(device)].push_back(ev0);
    timedFree[size_t(device)].push_back(ev1);
    return;
  }
  timedPending.push_back({ev0, ev1, device, pack});
  if (timedPending.size() >= kMaxTimed) settle_kernel_times();
}

void destroy_timing_events() {
  settle_kernel_times();
  for (auto &f : timedFree)
    for (void *e : f) tempi_hip_event_destroy(e);
  timedFree.clear();
}

void init_after_mpi() {
  if (env.noTempi) return;
  MPI_Comm_rank(MPI_COMM_WORLD, &state.worldRank);
  MPI_Comm_size(MPI_COMM_WORLD, &state.worldSize);
  state.pid = int32_t(getpid());
  logRank = state.worldRank;
  trace::init();
  hostTiming = std::getenv("TEMPI_PRINT_COUNTERS") != nullptr;
  gpu::init();
  types_init();
  state.active = true;
  topology::init();
  p2p::init();
  coll_init();
  LOG_DEBUG("TEMPI active: rank " << state.worldRank << "/" << state.worldSize
                                  << ", GPU " << (gpu::available() ? "yes" : "no"));
}

uint64_t now_ns() {
  return uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(
                      std::chrono::steady_clock::now().time_since_epoch())
                      .count());
}

void finalize_before_mpi() {
  if (!state.active) return;
  if (hostTiming) { // (TEMPI_PRINT_COUNTERS)
    const Counters &c = counters;
    std::fprintf(stderr,
                 "[tempi r%d] packs=%lu unpacks=%lu isends=%lu irecvs=%lu ipc=%lu (copy %lu/%lu) oneshot=%lu staged=%lu "
                 "direct=%lu/%lu "
                 "batches=%lu items=%lu passes=%lu | host ms: isend=%.2f irecv=%.2f flush=%.2f events=%.2f "
                 "testsome=%.2f wait=%.2f | nbr=%lu post=%.2f wait=%.2f | slabs MB: device=%.1f pinned=%.1f\n",
                 state.worldRank, (unsigned long)c.packs, (unsigned long)c.unpacks, (unsigned long)c.isends,
                 (unsigned long)c.irecvs, (unsigned long)c.send_ipc, (unsigned long)c.send_ipc_copy,
                 (unsigned long)c.copy_resends, (unsigned long)c.send_oneshot,
                 (unsigned long)c.send_staged, (unsigned long)c.send_direct, (unsigned long)c.direct_fallbacks,
                 (unsigned long)c.batches, (unsigned long)c.batched_items,
                 (unsigned long)c.progress_passes, c.ns_isend * 1e-6, c.ns_irecv * 1e-6, c.ns_flush * 1e-6,
                 c.ns_events * 1e-6, c.ns_testsome * 1e-6, c.ns_wait * 1e-6, (unsigned long)c.neighbor_colls,
                 c.ns_nbr_post * 1e-6, c.ns_nbr_wait * 1e-6, device_pool().bytes_held() / 1e6,
                 pinned_pool().bytes_held() / 1e6);
  }
  coll_finalize();
  p2p::finalize();
  destroy_timing_events();
  topology::finalize();
  LOG_DEBUG("counters: packs=" << counters.packs << " unpacks=" << counters.unpacks
                               << " launches=" << counters.launches << " lib_packs="
                               << counters.lib_packs << " sends=" << counters.sends);
  types_finalize();
  gpu::finalize();
  trace::finalize(state.worldRank);
  state.active = false;
}

namespace {

// run fn on the stream of `device`, with that device current, and wait for
// it (MPI_Pack / MPI_Unpack are synchronous: /root/reference/src/internal/
// packer_2d.cu:101-118). fn(stream, done) launches; `done` is non-null when
// the call may complete by ticket (Packer::Completion), i.e. when everything
// the work writes is device memory or a TEMPI coherent slab: kernel stores
// to the application's pinned host memory (possibly coarse-grained) are made
// host-visible by hipStreamSynchronize's system-scope release, not by a
// ticket. With kernel profiling on, HIP events bracket the
// launches on that stream and their elapsed time is accumulated.
template <typename F> int on_device(int device, bool pack, bool ticketOk, F &&fn) {
  int cur = 0;
  tempi_hip_get_device(&cur);
  if (cur != device) tempi_hip_set_device(device);
  void *s = gpu::stream(device);
  void *ev0 = nullptr, *ev1 = nullptr;
  if (kernelProfiling) {
    ev0 = timing_event(device);
    ev1 = timing_event(device);
  }
  if (ev0) tempi_hip_event_record(ev0, s);
  const bool byTicket = ticketOk;
  Packer::Completion done;
  int e = fn(s, byTicket ? &done : nullptr);
  if (ev1) tempi_hip_event_record(ev1, s);
  if (e == 0) {
    if (!byTicket) {
      counters.sync_waits++;
      e = tempi_hip_stream_synchronize(s);
    } else if (done.flag) {
      counters.ticket_waits++;
      e = tempi_hip_ticket_wait(s, done.flag, done.ticket);
    }
  }
  if (ev0 && ev1) timed(device, pack, ev0, ev1, e == 0);
  if (cur != device) tempi_hip_set_device(cur);
  return e;
}

// A staged MPI_Pack / MPI_Unpack's pinned slab is as large as the payload.
// Kept in the pool it would hold up to GiB of pinned memory until MPI_Finalize
// (ADVICE r02): slabs above this go back to the system after the call. After
// a failed GPU call the slab is only returned once its stream has drained
// (and leaked if that fails: a kernel may still be using it).
constexpr size_t kKeepStagedMax = size_t(64) << 20;
void stage_done(Slab *s, int device, bool failed) {
  if (!s) return;
  if (failed && tempi_hip_stream_synchronize(gpu::stream(device)) != 0) {
    pinned_pool().discard(s, false);
    return;
  }
  if (s->size > kKeepStagedMax)
    pinned_pool().discard(s);
  else
    pinned_pool().put(s);
}

// byte span [lo, hi) relative to the origin touched by `n` elements
void touched_span(MPI_Datatype t, int n, int64_t *lo, int64_t *hi) {
  MPI_Aint tlb, text, lb, ext;
  MPI_Type_get_true_extent(t, &tlb, &text);
  MPI_Type_get_extent(t, &lb, &ext);
  const int64_t d = int64_t(n - 1) * int64_t(ext);
  *lo = int64_t(tlb) + (d < 0 ? d : 0);
  *hi = int64_t(tlb) + int64_t(text) + (d > 0 ? d : 0);
}

// The library handles datatypes TEMPI cannot pack (irregular indexed,
// struct, darray). When one side lives in device-only memory and the library
// is not GPU-aware (MPICH here), the touched bytes travel through host memory
// around the library call; host-reachable sides are used in place.
int library_pack(const void *inbuf, int incount, MPI_Datatype t, void *outbuf, int outsize,
                 int *position, MPI_Comm comm) {
  counters.lib_packs++;
  int64_t lo, hi;
  touched_span(t, incount, &lo, &hi);
  const gpu::Ptr in = gpu::classify(static_cast<const char *>(inbuf) + lo);
  const gpu::Ptr out = gpu::classify(static_cast<char *>(outbuf) + *position);
  if ((!in.device_accessible || in.host_accessible) && (!out.device_accessible || out.host_accessible))
    return next.MPI_Pack(inbuf, incount, t, outbuf, outsize, position, comm);
  std::vector<char> hin, hout;
  const char *src = static_cast<const char *>(inbuf);
  if (in.device_accessible && !in.host_accessible) {
    hin.resize(size_t(hi - lo));
    gpu::check(tempi_hip_memcpy(hin.data(), src + lo, size_t(hi - lo)), "library pack D2H");
    src = hin.data() - lo;
  }
  int size = 0;
  MPI_Pack_size(incount, t, comm, &size);
  if (!(out.device_accessible && !out.host_accessible))
    return next.MPI_Pack(src, incount, t, outbuf, outsize, position, comm);
  hout.resize(size_t(size > 0 ? size : 1));
  int pos = 0;
  const int rc = next.MPI_Pack(src, incount, t, hout.data(), size, &pos, comm);
  if (rc != MPI_SUCCESS) return rc;
  if (int64_t(*position) + pos > outsize) return raise_error(comm, MPI_ERR_TRUNCATE);
  gpu::check(tempi_hip_memcpy(static_cast<char *>(outbuf) + *position, hout.data(), size_t(pos)),
             "library pack H2D");
  *position += pos;
  return MPI_SUCCESS;
}

int library_unpack(const void *inbuf, int insize, int *position, void *outbuf, int outcount,
                   MPI_Datatype t, MPI_Comm comm) {
  counters.lib_unpacks++;
  int64_t lo, hi;
  touched_span(t, outcount, &lo, &hi);
  const gpu::Ptr in = gpu::classify(static_cast<const char *>(inbuf) + *position);
  const gpu::Ptr out = gpu::classify(static_cast<char *>(outbuf) + lo);
  if ((!in.device_accessible || in.host_accessible) && (!out.device_accessible || out.host_accessible))
    return next.MPI_Unpack(inbuf, insize, position, outbuf, outcount, t, comm);
  int size = 0;
  MPI_Pack_size(outcount, t, comm, &size);
  std::vector<char> hin, hout;
  const char *src = static_cast<const char *>(inbuf);
  int srcsize = insize, pos = *position;
  if (in.device_accessible && !in.host_accessible) {
    const int64_t n = std::min<int64_t>(size, int64_t(insize) - *position);
    if (n < 0) return raise_error(comm, MPI_ERR_TRUNCATE);
    hin.resize(size_t(n > 0 ? n : 1));
    gpu::check(tempi_hip_memcpy(hin.data(), src + *position, size_t(n)), "library unpack D2H");
    src = hin.data();
    srcsize = int(n);
    pos = 0;
  }
  char *dst = static_cast<char *>(outbuf);
  const bool stageOut = out.device_accessible && !out.host_accessible;
  if (stageOut) { // read-modify-write: bytes between blocks keep their values
    hout.resize(size_t(hi - lo));
    gpu::check(tempi_hip_memcpy(hout.data(), dst + lo, size_t(hi - lo)), "library unpack D2H");
    dst = hout.data() - lo;
  }
  const int before = pos;
  const int rc = next.MPI_Unpack(src, srcsize, &pos, dst, outcount, t, comm);
  if (rc != MPI_SUCCESS) return rc;
  if (stageOut)
    gpu::check(tempi_hip_memcpy(static_cast<char *>(outbuf) + lo, hout.data(), size_t(hi - lo)),
               "library unpack H2D");
  *position += pos - before;
  return MPI_SUCCESS;
}

} // namespace
} // namespace tempi

using namespace tempi;

TEMPI_EXPORT int MPI_Init(int *argc, char ***argv) {
  resolve_next();
  read_environment();
  const int rc = next.MPI_Init(argc, argv);
  if (rc == MPI_SUCCESS) init_after_mpi();
  return rc;
}

// Thread support. TEMPI's transport keeps unsynchronised process-wide state
// (p2p_internal.hpp). An application that asks for MPI_THREAD_MULTIPLE, and
// gets it from the library, gets it from TEMPI too: every interposed call then
// runs under TEMPI's lock, which wait loops and blocking library calls give
// up (mt.hpp). Any other request is answered with at most
// MPI_THREAD_SERIALIZED -- the level the unlocked state is safe at -- so that
// applications that never asked for MULTIPLE pay nothing for the lock. (The
// reference only logs the level, /root/reference/src/init.cpp:36-46, and
// hands back whatever the library granted.) With TEMPI disabled the library's
// level stands.
namespace tempi {
constexpr int kMaxUnlockedLevel = MPI_THREAD_SERIALIZED;
int cap_thread_level(int level) {
  if (!state.active) return level;
  if (mt::on) return MPI_THREAD_MULTIPLE;
  return level > kMaxUnlockedLevel ? kMaxUnlockedLevel : level;
}
} // namespace tempi

TEMPI_EXPORT int MPI_Init_thread(int *argc, char ***argv, int required, int *provided) {
  resolve_next();
  read_environment();
  const int rc = next.MPI_Init_thread(argc, argv, required, provided);
  if (rc == MPI_SUCCESS) {
    init_after_mpi();
    if (provided && state.active) {
      mt::on = required == MPI_THREAD_MULTIPLE && *provided == MPI_THREAD_MULTIPLE;
      // TEMPI_FAULT_NO_MT_LOCK (tools/cpu_tsan.sh's negative control): report
      // MULTIPLE but leave the lock off, so that TSan shows what it guards
      const bool unguarded = mt::on && std::getenv("TEMPI_FAULT_NO_MT_LOCK") != nullptr;
      if (mt::on && state.worldRank == 0)
        LOG_DEBUG("MPI_THREAD_MULTIPLE: TEMPI's calls run under one process-wide lock");
      *provided = cap_thread_level(*provided);
      if (unguarded) { // never silent: a stray variable would make a threaded application unsafe
        LOG_WARN("TEMPI_FAULT_NO_MT_LOCK is set: MPI_THREAD_MULTIPLE is reported but TEMPI runs WITHOUT its lock "
                 "(a sanitizer negative control; unsafe for threaded applications)");
        mt::on = false;
      }
    }
  }
  return rc;
}

TEMPI_EXPORT int MPI_Query_thread(int *provided) {
  resolve_next();
  const int rc = next.MPI_Query_thread(provided);
  if (rc == MPI_SUCCESS && provided) *provided = cap_thread_level(*provided);
  return rc;
}

TEMPI_EXPORT int MPI_Finalize(void) {
  TEMPI_MT_ENTRY;
  resolve_next();
  finalize_before_mpi();
  mt::on = false; // (this call's own Entry still unlocks: it captured `on`)
  return next.MPI_Finalize();
}

TEMPI_EXPORT int MPI_Type_commit(MPI_Datatype *datatype) {
  TEMPI_MT_ENTRY;
  resolve_next();
  const int rc = next.MPI_Type_commit(datatype);
  if (rc != MPI_SUCCESS || !state.active || env.noTypeCommit) return rc;
  type_commit(*datatype);
  return rc;
}

TEMPI_EXPORT int MPI_Type_free(MPI_Datatype *datatype) {
  TEMPI_MT_ENTRY;
  resolve_next();
  // the library may hand the handle out again: forget it first
  if (state.active && !env.noTypeCommit) type_release(*datatype);
  return next.MPI_Type_free(datatype);
}

namespace tempi {
int pack(const void *inbuf, int incount, MPI_Datatype datatype, void *outbuf, int outsize, int *position,
         MPI_Comm comm) {
  if (!state.active || env.noPack || incount <= 0 || !position)
    return next.MPI_Pack(inbuf, incount, datatype, outbuf, outsize, position, comm);
  const TypeRecord *rec = type_lookup(datatype);
  if (!rec || !rec->packer || rec->desc.size == 0)
    return library_pack(inbuf, incount, datatype, outbuf, outsize, position, comm);
  const char *first = static_cast<const char *>(inbuf) + rec->desc.start;
  const gpu::Ptr src = gpu::classify(first);
  if (!src.device_accessible)
    return library_pack(inbuf, incount, datatype, outbuf, outsize, position, comm);
  const gpu::Ptr dst = gpu::classify(static_cast<char *>(outbuf) + *position);
  const int64_t bytes = rec->packer->packed_bytes(incount);
  if (*position < 0 || int64_t(*position) + bytes > int64_t(outsize))
    return raise_error(comm, MPI_ERR_TRUNCATE);
  const char *origin = static_cast<const char *>(src.dptr) - rec->desc.start;
  // a GPU object packed into pageable host memory: the kernel gathers into a
  // pinned, mapped slab (as the ONESHOT sender does) and the packed bytes are
  // copied out on the host -- only the payload crosses the host link, where
  // the library route would copy the object's whole span and pack on the CPU
  Slab *stage = dst.device_accessible ? nullptr : pinned_pool().get(size_t(std::max<int64_t>(bytes, 1)), src.device);
  if (!dst.device_accessible && !stage)
    return library_pack(inbuf, incount, datatype, outbuf, outsize, position, comm);
  // the kernel writes device memory or TEMPI's coherent slab: the ticket may
  // complete the call; into the application's pinned host memory it may not
  const bool ticketOk = stage != nullptr || !dst.host_accessible;
  const int e = env.faultPack ? 1 : on_device(src.device, true, ticketOk, [&](void *s, Packer::Completion *done) {
    void *out = stage ? stage->dev : dst.dptr;
    return done ? rec->packer->pack_ticket(out, origin, incount, s, done)
                : rec->packer->pack_async(out, origin, incount, s);
  });
  if (e != 0) { // (a GPU error falls back to the library instead of exiting)
    LOG_WARN("MPI_Pack: the GPU pack failed (" << tempi_hip_error_string(e) << "); the library packs it");
    stage_done(stage, src.device, true);
    return library_pack(inbuf, incount, datatype, outbuf, outsize, position, comm);
  }
  if (stage) {
    counters.staged_packs++;
    std::memcpy(static_cast<char *>(outbuf) + *position, stage->host, size_t(bytes));
    stage_done(stage, src.device, false);
  }
  *position += int(bytes);
  return MPI_SUCCESS;
}

int unpack(const void *inbuf, int insize, int *position, void *outbuf, int outcount, MPI_Datatype datatype,
           MPI_Comm comm) {
  if (!state.active || env.noPack || outcount <= 0 || !position)
    return next.MPI_Unpack(inbuf, insize, position, outbuf, outcount, datatype, comm);
  const TypeRecord *rec = type_lookup(datatype);
  if (!rec || !rec->packer || rec->desc.size == 0)
    return library_unpack(inbuf, insize, position, outbuf, outcount, datatype, comm);
  char *first = static_cast<char *>(outbuf) + rec->desc.start;
  const gpu::Ptr dst = gpu::classify(first);
  if (!dst.device_accessible)
    return library_unpack(inbuf, insize, position, outbuf, outcount, datatype, comm);
  const gpu::Ptr src = gpu::classify(static_cast<const char *>(inbuf) + *position);
  const int64_t bytes = rec->packer->packed_bytes(outcount);
  if (*position < 0 || int64_t(*position) + bytes > int64_t(insize))
    return raise_error(comm, MPI_ERR_TRUNCATE);
  char *origin = static_cast<char *>(dst.dptr) - rec->desc.start;
  // packed bytes in pageable host memory: copied into a pinned, mapped slab
  // on the host, scattered from there by the kernel (the ONESHOT receive)
  Slab *stage = src.device_accessible ? nullptr : pinned_pool().get(size_t(std::max<int64_t>(bytes, 1)), dst.device);
  if (!src.device_accessible && !stage)
    return library_unpack(inbuf, insize, position, outbuf, outcount, datatype, comm);
  if (stage) {
    counters.staged_unpacks++;
    std::memcpy(stage->host, static_cast<const char *>(inbuf) + *position, size_t(bytes));
  }
  // the kernel writes the strided object: by ticket only when it is device memory
  const int e = env.faultPack ? 1 : on_device(dst.device, false, !dst.host_accessible,
                                              [&](void *s, Packer::Completion *done) {
    const void *in = stage ? stage->dev : src.dptr;
    return done ? rec->packer->unpack_ticket(origin, in, outcount, s, done)
                : rec->packer->unpack_async(origin, in, outcount, s);
  });
  stage_done(stage, dst.device, e != 0);
  if (e != 0) {
    LOG_WARN("MPI_Unpack: the GPU unpack failed (" << tempi_hip_error_string(e) << "); the library unpacks it");
    return library_unpack(inbuf, insize, position, outbuf, outcount, datatype, comm);
  }
  *position += int(bytes);
  return MPI_SUCCESS;
}
} // namespace tempi

TEMPI_EXPORT int MPI_Pack(const void *inbuf, int incount, MPI_Datatype datatype, void *outbuf,
                          int outsize, int *position, MPI_Comm comm) {
  TEMPI_MT_ENTRY;
  resolve_next();
  TEMPI_RANGE("MPI_Pack");
  return tempi::pack(inbuf, incount, datatype, outbuf, outsize, position, comm);
}

TEMPI_EXPORT int MPI_Unpack(const void *inbuf, int insize, int *position, void *outbuf, int outcount,
                            MPI_Datatype datatype, MPI_Comm comm) {
  TEMPI_MT_ENTRY;
  resolve_next();
  TEMPI_RANGE("MPI_Unpack");
  return tempi::unpack(inbuf, insize, position, outbuf, outcount, datatype, comm);
}
