// tempi_amd/csrc/core/ext.cpp -- TEMPI's non-MPI entry points
// (include/tempi_ext.h): type introspection, counters, stream access, and the
// MPI ABI constants of the library TEMPI was compiled against.
#include "counters.hpp"
#include "env.hpp"
#include "gpu.hpp"
#include "mt.hpp"
#include "p2p.hpp"
#include "perf_model.hpp"
#include "placement.hpp"
#include "state.hpp"
#include "type_cache.hpp"

#include "tempi_ext.h"

#include <cstdio>
#include <cstring>

#define TEMPI_EXPORT extern "C" __attribute__((visibility("default")))

using namespace tempi;

// Every entry point that reads TEMPI state a concurrent interposed call may
// change (the type table, counters, the perf model, placement) takes TEMPI's
// lock at MPI_THREAD_MULTIPLE, as the interposed calls do.
TEMPI_EXPORT int tempi_type_describe(int64_t datatype, tempi_type_info *out) {
  TEMPI_MT_ENTRY;
  std::memset(out, 0, sizeof *out);
  const TypeRecord *rec = type_lookup(MPI_Datatype(datatype));
  if (!rec) return 0;
  out->known = 1;
  const StridedBlock &sb = rec->desc;
  out->valid = sb.valid ? 1 : 0;
  out->start = sb.start;
  out->block = sb.block;
  out->size = sb.size;
  out->lb = sb.lb;
  out->extent = sb.extent;
  out->ndims = int32_t(sb.dims.size());
  if (out->ndims > TEMPI_EXT_MAX_DIMS) {
    out->ndims = -1;
    return 0;
  }
  for (size_t k = 0; k < sb.dims.size(); ++k) {
    out->counts[k] = sb.dims[k].count;
    out->strides[k] = sb.dims[k].stride;
  }
  return 1;
}

TEMPI_EXPORT void tempi_get_counters(tempi_counters_t *o) {
  TEMPI_MT_ENTRY;
  const Counters &c = counters;
  o->packs = c.packs;
  o->unpacks = c.unpacks;
  o->pack_bytes = c.pack_bytes;
  o->unpack_bytes = c.unpack_bytes;
  o->launches = c.launches;
  o->lib_packs = c.lib_packs;
  o->lib_unpacks = c.lib_unpacks;
  o->sends = c.sends;
  o->recvs = c.recvs;
  o->isends = c.isends;
  o->irecvs = c.irecvs;
  o->send_device = c.send_device;
  o->send_oneshot = c.send_oneshot;
  o->send_staged = c.send_staged;
  o->send_ipc = c.send_ipc;
  o->lib_sends = c.lib_sends;
  o->lib_recvs = c.lib_recvs;
  o->send_direct = c.send_direct;
  o->direct_fallbacks = c.direct_fallbacks;
  o->neighbor_colls = c.neighbor_colls;
  o->send_ipc_copy = c.send_ipc_copy;
  o->copy_resends = c.copy_resends;
  o->ipc_maps_replaced = c.ipc_maps_replaced;
  o->canary_ok = c.canary_ok;
  o->canary_fail = c.canary_fail;
  o->self_matched = c.self_matched;
  o->staged_packs = c.staged_packs;
  o->staged_unpacks = c.staged_unpacks;
  o->ticket_waits = c.ticket_waits;
  o->sync_waits = c.sync_waits;
  o->ticket_batches = c.ticket_batches;
  o->persistent_starts = c.persistent_starts;
  o->batches = c.batches;
  o->gpu_inflight_ns = c.ns_gpu_inflight;
  o->bytes_ipc = c.bytes_ipc;
  o->bytes_ipc_copy = c.bytes_ipc_copy;
  o->bytes_oneshot = c.bytes_oneshot;
  o->bytes_staged = c.bytes_staged;
  o->bytes_device = c.bytes_device;
  o->bytes_direct = c.bytes_direct;
}

TEMPI_EXPORT void tempi_reset_counters(void) {
  TEMPI_MT_ENTRY;
  settle_kernel_times(); // (pending pairs belong to the counters being reset)
  counters = Counters();
}

TEMPI_EXPORT void tempi_set_kernel_profiling(int on) {
  kernelProfiling = on != 0;
}

TEMPI_EXPORT void tempi_get_kernel_times(tempi_kernel_times *o) {
  TEMPI_MT_ENTRY;
  settle_kernel_times();
  o->pack_ms = counters.pack_kernel_ms;
  o->unpack_ms = counters.unpack_kernel_ms;
  o->packs = counters.pack_timed;
  o->unpacks = counters.unpack_timed;
}

TEMPI_EXPORT void *tempi_get_stream(int device) { return gpu::available() ? gpu::stream(device) : nullptr; }

TEMPI_EXPORT int tempi_gpu_available(void) { return gpu::available() ? 1 : 0; }

TEMPI_EXPORT int tempi_hip_runtimes(char *paths, int cap) {
  const std::vector<std::string> rt = gpu::hip_runtimes();
  std::string all;
  for (const std::string &r : rt) all += (all.empty() ? "" : ";") + r;
  if (paths && cap > 0) std::snprintf(paths, size_t(cap), "%s", all.c_str());
  return int(rt.size());
}

TEMPI_EXPORT const char *tempi_version(void) { return "tempi-mi355x 0.1 (gfx950)"; }

TEMPI_EXPORT int64_t tempi_mpi_constant(const char *name, int *found) {
  struct C {
    const char *n;
    int64_t v;
  };
#define H(x) {#x, int64_t(x)}
#define P(x) {#x, int64_t(reinterpret_cast<intptr_t>(x))}
  static const C table[] = {
      H(MPI_SUCCESS), H(MPI_ERR_TRUNCATE), H(MPI_ERR_OTHER), H(MPI_ERR_TYPE),
      H(MPI_BYTE), H(MPI_CHAR), H(MPI_SHORT), H(MPI_INT), H(MPI_LONG), H(MPI_LONG_LONG),
      H(MPI_UNSIGNED), H(MPI_FLOAT), H(MPI_DOUBLE), H(MPI_PACKED), H(MPI_INT8_T), H(MPI_INT16_T),
      H(MPI_INT32_T), H(MPI_INT64_T), H(MPI_UINT8_T), H(MPI_UINT16_T), H(MPI_UINT32_T),
      H(MPI_UINT64_T), H(MPI_DATATYPE_NULL), H(MPI_COMM_WORLD), H(MPI_COMM_SELF), H(MPI_COMM_NULL),
      H(MPI_REQUEST_NULL), H(MPI_ORDER_C), H(MPI_ORDER_FORTRAN), H(MPI_ANY_SOURCE), H(MPI_ANY_TAG),
      H(MPI_PROC_NULL), H(MPI_SUM), H(MPI_MAX), H(MPI_MIN), H(MPI_THREAD_SINGLE),
      H(MPI_THREAD_FUNNELED), H(MPI_THREAD_SERIALIZED), H(MPI_THREAD_MULTIPLE),
      H(MPI_MAX_PROCESSOR_NAME), H(MPI_UNDEFINED), H(MPI_BSEND_OVERHEAD), H(MPI_ERR_REQUEST), H(MPI_ERR_IN_STATUS),
      P(MPI_STATUS_IGNORE), P(MPI_STATUSES_IGNORE), P(MPI_IN_PLACE), P(MPI_UNWEIGHTED), P(MPI_WEIGHTS_EMPTY), H(MPI_INFO_NULL),
      H(MPI_ERRORS_RETURN), H(MPI_ERRORS_ARE_FATAL), H(MPI_MESSAGE_NULL), H(MPI_MESSAGE_NO_PROC),
      {"sizeof(MPI_Message)", int64_t(sizeof(MPI_Message))},
      {"sizeof(MPI_Status)", int64_t(sizeof(MPI_Status))},
      {"sizeof(MPI_Aint)", int64_t(sizeof(MPI_Aint))},
      {"sizeof(MPI_Datatype)", int64_t(sizeof(MPI_Datatype))},
      {"sizeof(MPI_Comm)", int64_t(sizeof(MPI_Comm))},
      {"sizeof(MPI_Request)", int64_t(sizeof(MPI_Request))},
      {"sizeof(MPI_Op)", int64_t(sizeof(MPI_Op))},
      {"offsetof(MPI_Status,MPI_SOURCE)", int64_t(offsetof(MPI_Status, MPI_SOURCE))},
      {"offsetof(MPI_Status,MPI_TAG)", int64_t(offsetof(MPI_Status, MPI_TAG))},
      {"offsetof(MPI_Status,MPI_ERROR)", int64_t(offsetof(MPI_Status, MPI_ERROR))},
  };
#undef H
#undef P
  for (const C &c : table)
    if (!std::strcmp(c.n, name)) {
      if (found) *found = 1;
      return c.v;
    }
  if (found) *found = 0;
  return 0;
}

// ---- perf model (reference interpolation rules; tests replay its KATs)

static std::vector<IidTime> curve_of(const double *t, int n) {
  std::vector<IidTime> v(size_t(n > 0 ? n : 0));
  for (int i = 0; i < n; ++i) v[size_t(i)].time = t[i];
  return v;
}

TEMPI_EXPORT double tempi_interp_time(const double *times, int n, int64_t bytes) {
  return interp_time(curve_of(times, n), bytes);
}

TEMPI_EXPORT double tempi_interp_2d(const double *table, int rows, int cols, int64_t bytes, int64_t block) {
  std::vector<std::vector<IidTime>> a;
  for (int r = 0; r < rows; ++r) a.push_back(curve_of(table + size_t(r) * size_t(cols), cols));
  return interp_2d(a, bytes, block);
}

TEMPI_EXPORT int tempi_perf_loaded(void) { return systemPerformanceLoaded ? 1 : 0; }

TEMPI_EXPORT int tempi_perf_source(char *path, int cap) {
  TEMPI_MT_ENTRY;
  if (!path || cap <= 0) return -1;
  std::snprintf(path, size_t(cap), "%s", systemPerformanceSource.c_str());
  return systemPerformanceLoaded ? 1 : 0;
}

TEMPI_EXPORT void tempi_perf_reload(void) {
  TEMPI_MT_ENTRY;
  if (state.active) p2p::reload_perf_model();
}

TEMPI_EXPORT int tempi_perf_roundtrip(const char *json_in, char *json_out, int cap) {
  SystemPerformance sp;
  std::string err;
  if (!from_json(json_in, &sp, &err)) return -1;
  const std::string s = to_json(sp);
  if (int(s.size()) + 1 > cap) return int(s.size()) + 1;
  std::memcpy(json_out, s.c_str(), s.size() + 1);
  return 0;
}

TEMPI_EXPORT void tempi_set_datatype_method(int m) {
  TEMPI_MT_ENTRY;
  // 0 AUTO, 1 ONESHOT, 2 DEVICE, 3 STAGED, 4 IPC (as TEMPI_DATATYPE_*)
  static const DatatypeMethod map[] = {DatatypeMethod::AUTO, DatatypeMethod::ONESHOT, DatatypeMethod::DEVICE,
                                       DatatypeMethod::STAGED, DatatypeMethod::IPC};
  if (m >= 0 && m < 5) env.datatype = map[m];
}

TEMPI_EXPORT int tempi_choose_method(int64_t bytes, int64_t block, int colocated, int blocking, int *from_model) {
  TEMPI_MT_ENTRY; // (TEMPI state: under the lock at MPI_THREAD_MULTIPLE)
  bool fm = false;
  const int m = state.active ? p2p::query_method(bytes, block, colocated != 0, blocking != 0, &fm) : 0;
  if (from_model) *from_model = fm ? 1 : 0;
  return m;
}

TEMPI_EXPORT int64_t tempi_ipc_threshold(int64_t block, int *from_model) {
  TEMPI_MT_ENTRY;
  bool fm = false;
  const int64_t t = state.active ? p2p::query_ipc_threshold(block, &fm) : -1;
  if (from_model) *from_model = fm ? 1 : 0;
  return t;
}

TEMPI_EXPORT int64_t tempi_batch_ipc_threshold(const char *perf_json, int64_t block) {
  SystemPerformance sp;
  std::string err;
  if (!perf_json || !from_json(perf_json, &sp, &err)) return -2;
  return batch_ipc_threshold(sp, block);
}

// ---- rank placement (core/placement.hpp)

TEMPI_EXPORT int64_t tempi_partition(int n, const int *xadj, const int *adjncy, const int *adjwgt, int nparts,
                                     const int *sizes, int method, int *part) {
  if (n < 0 || nparts < 1 || !part || (n > 0 && (!xadj || !adjncy))) return -1;
  std::vector<int> sz(size_t(nparts), n / nparts);
  if (sizes) {
    sz.assign(sizes, sizes + nparts);
  } else if (n % nparts) {
    return -1;
  }
  int64_t total = 0;
  for (int s : sz) total += s;
  if (total != n) return -1;
  std::vector<placement::Edge> edges;
  for (int u = 0; u < n; ++u)
    for (int e = xadj[u]; e < xadj[u + 1]; ++e) edges.push_back({u, adjncy[e], adjwgt ? int64_t(adjwgt[e]) : 1});
  const placement::Graph g = placement::make_graph(n, edges);
  const std::vector<int> p = method == 1 ? placement::random_parts(sz) : placement::partition(g, sz);
  std::copy(p.begin(), p.end(), part);
  return placement::edge_cut(g, p);
}

TEMPI_EXPORT int tempi_placement_info(int64_t out[6]) {
  TEMPI_MT_ENTRY;
  const placement::Info i = placement::last();
  out[0] = i.placed;
  out[1] = i.nodes;
  out[2] = i.method;
  out[3] = i.appRank;
  out[4] = i.cutIdentity;
  out[5] = i.cutPlaced;
  return i.placed;
}
