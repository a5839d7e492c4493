/*
 * include/tempi_ext.h -- TEMPI's own (non-MPI) C entry points in libtempi.so:
 * introspection for tests and benchmarks, counters, and the MPI ABI constants
 * of the library TEMPI was built against (so ctypes front ends need no
 * compiler). Plain integers and pointers only. MPI handles are passed as
 * int64_t (MPICH's MPI_Datatype / MPI_Comm are int).
 */
#ifndef TEMPI_EXT_H
#define TEMPI_EXT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TEMPI_EXT_MAX_DIMS 16

/* the canonical form TEMPI derived for a committed datatype
   (the reference's StridedBlock: /root/reference/include/strided_block.hpp) */
typedef struct tempi_type_info {
  int32_t known;    /* 1 when the handle is in TEMPI's type cache */
  int32_t valid;    /* 1 when it is a strided block TEMPI packs on the GPU */
  int32_t ndims;    /* dims above the contiguous block, outermost first */
  int32_t pad_;
  int64_t start;    /* byte offset of the first byte from the buffer origin */
  int64_t block;    /* contiguous bytes */
  int64_t size, lb, extent;
  int64_t counts[TEMPI_EXT_MAX_DIMS];
  int64_t strides[TEMPI_EXT_MAX_DIMS];
} tempi_type_info;

int tempi_type_describe(int64_t datatype, tempi_type_info *out);

typedef struct tempi_counters_t {
  uint64_t packs, unpacks, pack_bytes, unpack_bytes, launches;
  uint64_t lib_packs, lib_unpacks;
  uint64_t sends, recvs, isends, irecvs;
  uint64_t send_device, send_oneshot, send_staged, send_ipc;
  uint64_t lib_sends, lib_recvs;
  uint64_t send_direct, direct_fallbacks; /* sends to the same process */
  uint64_t neighbor_colls; /* MPI_Neighbor_alltoall{v,w} taken by TEMPI */
  uint64_t send_ipc_copy;  /* IPC sends the receiver copied out of the sender's object */
  uint64_t copy_resends;   /* IPC COPY sends answered through the host instead */
  uint64_t ipc_maps_replaced; /* peer mappings closed because the peer freed and replaced that allocation */
  uint64_t canary_ok;   /* peers on another GPU whose mapped memory read back right at first contact */
  uint64_t canary_fail; /* ... and those that did not (IPC with them off: host-staged transfers) */
  uint64_t self_matched; /* messages to this same process matched inside TEMPI (no library message) */
  uint64_t staged_packs;   /* MPI_Pack of a GPU object into pageable host memory (through a pinned slab) */
  uint64_t staged_unpacks; /* MPI_Unpack into a GPU object from pageable host memory */
  uint64_t ticket_waits;   /* synchronous MPI_Pack / MPI_Unpack completed by a ticket the GPU stored */
  uint64_t sync_waits;     /* ... completed by hipStreamSynchronize (kernel wrote application host memory) */
  uint64_t ticket_batches; /* transport batches whose last launch stored a completion ticket (no event) */
  uint64_t persistent_starts; /* MPI_Start / MPI_Startall of persistent requests TEMPI holds */
  uint64_t batches;        /* transport batches launched (gathers, scatters, copies) */
  uint64_t gpu_inflight_ns; /* time with a transport batch in flight: from its launch's return to its
                               completion observed by the host (the GPU's busy time, by TEMPI's account) */
  /* payload bytes of device-object sends by route: IPC (IPC COPY included,
     and counted again on its own), ONESHOT, STAGED, DEVICE, DIRECT (this process) */
  uint64_t bytes_ipc, bytes_ipc_copy, bytes_oneshot, bytes_staged, bytes_device, bytes_direct;
} tempi_counters_t;
void tempi_get_counters(tempi_counters_t *out);
void tempi_reset_counters(void);

/* Kernel timing of synchronous MPI_Pack / MPI_Unpack: when on, TEMPI
   brackets each operation's launches with HIP events on its stream and
   accumulates the elapsed GPU time (read back with tempi_get_kernel_times;
   tempi_reset_counters clears it). */
typedef struct tempi_kernel_times {
  double pack_ms, unpack_ms;
  uint64_t packs, unpacks;
} tempi_kernel_times;
void tempi_set_kernel_profiling(int on);
void tempi_get_kernel_times(tempi_kernel_times *out);

/* the HIP stream (hipStream_t) TEMPI uses on `device`; NULL if none */
void *tempi_get_stream(int device);
/* 1 when TEMPI found a GPU at MPI_Init */
int tempi_gpu_available(void);

/* value of an MPI constant by name (e.g. "MPI_BYTE", "MPI_COMM_WORLD",
   "MPI_ORDER_C", "sizeof(MPI_Status)"); *found = 0 if unknown */
int64_t tempi_mpi_constant(const char *name, int *found);

const char *tempi_version(void);

/* the HIP runtimes (distinct libamdhip64 objects) mapped into this process,
   as ';'-separated paths into paths[cap]; returns their number. More than
   one (e.g. a PyTorch wheel's bundled runtime beside ROCm's) is reported
   once at MPI_Init: streams of different runtimes are not ordered with each
   other. */
int tempi_hip_runtimes(char *paths, int cap);

/* perf model (include the reference's interpolation rules,
   /root/reference/src/internal/measure_system.cpp:184-293):
   times[i] = seconds for 2^i bytes; table[r*cols+c] = seconds for 2^(2r+6)
   bytes in 2^c-byte blocks. +inf when unknown. */
double tempi_interp_time(const double *times, int n, int64_t bytes);
double tempi_interp_2d(const double *table, int rows, int cols, int64_t bytes, int64_t block);
/* 1 when TEMPI_CACHE_DIR/perf.json was loaded at MPI_Init */
int tempi_perf_loaded(void);
/* the file AUTO's model was read from (this node's TEMPI_CACHE_DIR/perf.json,
   or the shipped MI355X model) into path[cap]; "" and 0 for the built-in
   policy, 1 when a model is loaded */
int tempi_perf_source(char *path, int cap);
/* re-read the model, e.g. after apps/measure_system wrote this node's
   perf.json (call on every rank) */
void tempi_perf_reload(void);
/* the message size from which a NON-blocking AUTO send of `block`-byte
   blocks to a co-located peer takes IPC instead of ONESHOT: priced per batch
   from this node's own TEMPI_CACHE_DIR/perf.json when one was measured here
   (*from_model = 1; the model may lower the built-in 4096, never raise it),
   else the built-in 4096 (*from_model = 0); -1 before MPI_Init. */
int64_t tempi_ipc_threshold(int64_t block, int *from_model);
/* the same pricing over a perf.json document (no MPI needed): the threshold,
   INT64_MAX for never, -1 when a curve it needs is missing, -2 when the
   document does not parse */
int64_t tempi_batch_ipc_threshold(const char *perf_json, int64_t block);
/* parse + re-emit a perf.json document (schema check); 0 on success */
int tempi_perf_roundtrip(const char *json_in, char *json_out, int cap);
/* override TEMPI_DATATYPE_* at run time: 0 AUTO, 1 ONESHOT, 2 DEVICE,
   3 STAGED, 4 IPC (used by tools/measure_system) */
void tempi_set_datatype_method(int method);

/* the route TEMPI takes for a strided message of `bytes` packed bytes in
   `block`-byte blocks to a co-located (1) or off-node (0) peer, blocking (1)
   or non-blocking (0), under the current TEMPI_DATATYPE_* choice: 1 ONESHOT,
   2 DEVICE, 3 STAGED, 4 IPC (0 before MPI_Init); *from_model = 1 when AUTO
   priced it with the loaded perf.json (/root/reference/src/internal/
   sender.cpp:251-290), 0 when the built-in policy decided */
int tempi_choose_method(int64_t bytes, int64_t block, int colocated, int blocking, int *from_model);

/* NIST SP 800-90B sec. 5.1 permutation test: 1 when `samples` look IID
   (tools/measure_system repeats a measurement until they do) */
int tempi_sp800_90b_iid(const double *samples, int n, int perms, uint64_t seed);

/* rank placement (MPI_Dist_graph_create_adjacent with reorder = 1 and
   TEMPI_PLACEMENT_KAHIP / _METIS / _RANDOM; /root/reference/src/
   dist_graph_create_adjacent.cpp:55-470). tempi_partition splits the graph
   given as CSR (xadj[n + 1], adjncy; adjwgt NULL = unit weights; each entry
   u -> v adds its weight to the undirected edge {u, v}, self loops ignored)
   into nparts parts of sizes[k] vertices (NULL: n / nparts each). method 0:
   TEMPI's partitioner, 1: the reference's random rule (partition.cpp:27-34,
   one generator seeded 0 per process). Writes part[n] and returns the edge
   cut, or -1 for bad input. */
int64_t tempi_partition(int n, const int *xadj, const int *adjncy, const int *adjwgt, int nparts,
                        const int *sizes, int method, int *part);
/* the last placement this process took part in: out[0] 1 if any, [1] nodes,
   [2] method (1 random, 2 partitioner), [3] this process's new rank, [4] the
   edge cut of the library's rank order, [5] the placed edge cut (rank 0's
   graph; 0 for random). Returns out[0]. */
int tempi_placement_info(int64_t out[6]);

#ifdef __cplusplus
}
#endif
#endif
