/*
 * include/tempi_hip.h -- the thin C ABI between TEMPI's C++ host layer
 * (libtempi.so, the MPI interposer) and the GPU (libtempi_hip.so, hipcc-built
 * for gfx950). Plain pointers, sizes and integer status codes only: the
 * interposer never includes a HIP header, and nothing here is CUDA-shaped.
 *
 * Status: every function returns 0 on success, otherwise the hipError_t value
 * (tempi_hip_error_string() names it).
 *
 * What each group replaces in the reference:
 *   pack / unpack kernels   Packer2D/3D launch_pack/launch_unpack
 *                           (/root/reference/src/internal/packer_2d.cu:21-74,
 *                            packer_3d.cu:80-116) and the CUDA kernels
 *                           (/root/reference/include/pack_kernels.cuh:19-120,
 *                            :350-433), and Packer1D's cudaMemcpyAsync
 *                           (/root/reference/src/internal/packer_1d.cu:16-49)
 *   streams / events        /root/reference/src/internal/streams.cpp:19-42,
 *                           events.cpp:17-83
 *   memory                  device_allocator / host_allocator
 *                           (/root/reference/include/allocator_device.hpp:35-53,
 *                            allocator_host.hpp:31-60)
 *   pointer attributes      cudaPointerGetAttributes in
 *                           /root/reference/src/pack.cpp:42-49
 */
#ifndef TEMPI_HIP_H
#define TEMPI_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* maximum number of strided dimensions above the contiguous block (the
   element count of a Pack call counts as one) */
#define TEMPI_HIP_MAX_DIMS 5

/* A canonical strided object: `block` contiguous bytes, repeated over `ndims`
   dimensions listed OUTERMOST FIRST, dimension k having counts[k] elements
   strides[k] bytes apart (strides may be negative). The packed form is the
   blocks in row-major (odometer) order, back to back. */
typedef struct tempi_hip_desc {
  int64_t block;
  int32_t ndims;
  int32_t pad_;
  int64_t counts[TEMPI_HIP_MAX_DIMS];
  int64_t strides[TEMPI_HIP_MAX_DIMS];
} tempi_hip_desc;

/* gather: packed[0 .. bytes) <- strided object whose first byte is `first` */
int tempi_hip_pack(void *packed, const void *first, const tempi_hip_desc *d,
                   void *stream);
/* scatter: strided object whose first byte is `first` <- packed[0 .. bytes) */
int tempi_hip_unpack(void *first, const void *packed, const tempi_hip_desc *d,
                     void *stream);
/* Many objects in as few launches as possible (one per word width x rank
   group, up to a few dozen objects per launch): item i gathers (pack) or
   scatters (unpack) between items[i].packed and the strided object whose
   first byte is items[i].first. Used for bursts of MPI_Isend / MPI_Irecv. */
typedef struct tempi_hip_batch_item {
  void *packed;
  void *first;
  tempi_hip_desc desc;
  uint32_t flags; /* TEMPI_HIP_ITEM_*; 0 for ordinary items */
  uint32_t reserved_;
} tempi_hip_batch_item;
/* unpack: `packed` is another process's memory mapped through an IPC handle
   (possibly another GPU's), reused by its owner for later messages; the
   kernel reads it with system-scope loads so that no line this GPU cached
   from an earlier message in the same buffer is returned */
#define TEMPI_HIP_ITEM_REMOTE 1u
int tempi_hip_pack_batch(const tempi_hip_batch_item *items, int n, void *stream);
int tempi_hip_unpack_batch(const tempi_hip_batch_item *items, int n, void *stream);

/* Strided -> strided copy with no packed intermediate: the object at
   dst_first (shape dst) <- the object at src_first (shape src), in type-map
   order; both shapes must describe the same number of bytes. This is what a
   message between two buffers of one process (a send to self) reduces to.
   tempi_hip_copy_supported() says whether one item can run as a copy kernel
   (at most 3 strided dimensions a side after normalisation, < 2 GiB);
   tempi_hip_copy_batch() fails with hipErrorInvalidValue on an item that
   cannot, so callers route those through pack + unpack. */
typedef struct tempi_hip_copy_item {
  void *dst_first;
  const void *src_first;
  tempi_hip_desc dst;
  tempi_hip_desc src;
  uint32_t flags; /* TEMPI_HIP_ITEM_REMOTE: src is another process's IPC-mapped memory */
  uint32_t reserved_;
} tempi_hip_copy_item;
int tempi_hip_copy_supported(void *dst_first, const void *src_first,
                             const tempi_hip_desc *dst, const tempi_hip_desc *src);
int tempi_hip_copy_batch(const tempi_hip_copy_item *items, int n, void *stream);

/* synchronous forms (MPI_Pack / MPI_Unpack, /root/reference/src/internal/
   packer_2d.cu:101-118): the same work plus a completion ticket. Once `*flag`
   (pinned, coherent host memory) reaches `*ticket` (wrapping uint32 compare,
   tempi_hip_ticket_wait), the work is complete and its writes to device
   memory are visible device-wide. A launch of at most TEMPI_FOLD_MAX_BLOCKS
   workgroups stores the ticket from its own last workgroup; larger work gets
   the ticket kernel queued behind it. */
int tempi_hip_pack_ticket(void *packed, const void *first, const tempi_hip_desc *d, void *stream,
                          const uint32_t **flag, uint32_t *ticket);
int tempi_hip_unpack_ticket(void *first, const void *packed, const tempi_hip_desc *d, void *stream,
                            const uint32_t **flag, uint32_t *ticket);
/* the batched forms with a ticket folded into the batch's last launch: when
   that launch is small enough to fold (as above), *flag and *ticket are set
   as there; otherwise *flag is NULL and the caller waits for the work as it
   would without a ticket (an event). No ticket kernel is ever queued. Used by
   the transport: a batch whose ticket is seen is complete without HIP's own
   completion path. */
int tempi_hip_pack_batch_ticket(const tempi_hip_batch_item *items, int n, void *stream, const uint32_t **flag,
                                uint32_t *ticket);
int tempi_hip_unpack_batch_ticket(const tempi_hip_batch_item *items, int n, void *stream, const uint32_t **flag,
                                  uint32_t *ticket);
int tempi_hip_copy_batch_ticket(const tempi_hip_copy_item *items, int n, void *stream, const uint32_t **flag,
                                uint32_t *ticket);
/* synchronous forms served by the RESIDENT packer (pack_kernels.hip,
   "resident packer"): a kernel kept running between the calls of a burst
   takes the request from pinned host memory -- no launch per call. On return
   0 with *served = 1 the work is complete and visible device-wide; *served = 0
   means it was not taken (narrow words, > 3 dims, larger than
   TEMPI_RESIDENT_MAX_BYTES, TEMPI_RESIDENT=0) and the caller launches on
   `stream` as before. Replaces the launch + cudaStreamSynchronize of
   /root/reference/src/internal/packer_2d.cu:101-118 for small objects. */
int tempi_hip_pack_resident(void *packed, const void *first, const tempi_hip_desc *d, void *stream, int *served);
int tempi_hip_unpack_resident(void *first, const void *packed, const tempi_hip_desc *d, void *stream, int *served);
/* requests served, server launches, requests posted again after crossing a
   server's idle exit */
void tempi_hip_resident_stats(uint64_t *served, uint64_t *launches, uint64_t *reposts);
/* requests whose server ended with them neither served nor refused (its
   counters were then reset and the request posted again; 0 in every test) */
uint64_t tempi_hip_resident_lost(void);
/* an EXIT request to every running server; returns once they have left
   (MPI_Finalize) */
void tempi_hip_resident_stop(void);
/* turn the resident packer on (1) or off (0) for later calls; returns the
   previous setting (initially TEMPI_RESIDENT, default on) */
int tempi_hip_resident_enable(int on);
/* diagnostic (TEMPI_RESIDENT_STAMPS=1): the GPU clock (wall_clock64, 100 MHz)
   at five points of the last request -- the leader saw it; worker 0 saw the
   hand-off, finished its acquire, finished its share; the completion stored */
int tempi_hip_resident_stamps(uint64_t *out);

/* number of packed bytes a descriptor describes */
int64_t tempi_hip_desc_bytes(const tempi_hip_desc *d);
/* the word width (1,2,4,8,16) the strided -> strided copy kernel will use for
   this item; 0 = 16-byte chunks with 8-byte halves at row seams (both sides
   8 bytes past a 16-byte boundary, blocks and strides multiples of 16);
   -1 when the copy is unsupported (tempi_hip_copy_supported) */
int tempi_hip_copy_word_width(void *dst_first, const void *src_first, const tempi_hip_desc *dst,
                              const tempi_hip_desc *src);
/* the word width (1,2,4,8,16) the kernels will use for these pointers */
int tempi_hip_word_width(const void *packed, const void *first,
                         const tempi_hip_desc *d);

/* devices */
int tempi_hip_device_count(int *n);
/* a 16-byte identity of the physical GPU (the same in every process that
   sees it, whatever its ordinal there) */
int tempi_hip_device_uuid(int device, unsigned char uuid[16]);
int tempi_hip_get_device(int *dev);
int tempi_hip_set_device(int dev);
/* 1 when kernels on `device` can load from memory of `peer` (always 1 for
   device == peer), 0 otherwise */
int tempi_hip_can_access_peer(int device, int peer);
int tempi_hip_device_synchronize(void);

/* pointer classification (reference semantics: "device-accessible" means
   the GPU can dereference it: device, managed, or mapped pinned host) */
enum tempi_hip_mem_kind {
  TEMPI_HIP_MEM_HOST = 0,   /* pageable / unknown host memory */
  TEMPI_HIP_MEM_DEVICE = 1, /* hipMalloc */
  TEMPI_HIP_MEM_PINNED = 2, /* registered / hipHostMalloc, mapped */
  TEMPI_HIP_MEM_MANAGED = 3 /* hipMallocManaged */
};
typedef struct tempi_hip_ptrinfo {
  int kind;           /* tempi_hip_mem_kind */
  int device;         /* owning device, -1 for host */
  void *device_ptr;   /* GPU-visible address (NULL when not accessible) */
} tempi_hip_ptrinfo;
int tempi_hip_pointer_info(const void *p, tempi_hip_ptrinfo *out);

/* streams and events (opaque handles) */
int tempi_hip_stream_create(void **stream); /* non-blocking stream */
/* non-blocking stream at the device's highest priority (high != 0) or the
   default one */
int tempi_hip_stream_create_priority(void **stream, int high);
int tempi_hip_stream_destroy(void *stream);
int tempi_hip_stream_synchronize(void *stream);
/* 0 when everything queued on `stream` has completed, 1 when not yet,
   otherwise the stream's error */
int tempi_hip_stream_query(void *stream);
/* wait for `stream` by a ticket a kernel queued behind its work stores to
   pinned memory (faster than tempi_hip_stream_synchronize for small work) */
int tempi_hip_stream_signal_wait(void *stream);
/* queue a ticket behind the work on `stream`: once `*flag` (pinned host
   memory) reaches `*ticket` (as a wrapping uint32 compare), that work is done */
int tempi_hip_stream_ticket(void *stream, const uint32_t **flag, uint32_t *ticket);
/* spin until *flag reaches ticket; the stream is queried every ~20 us, so a
   faulted stream returns its error */
int tempi_hip_ticket_wait(void *stream, const uint32_t *flag, uint32_t ticket);
/* tickets issued so far: stored by the work kernel itself / by a ticket kernel */
void tempi_hip_ticket_stats(uint64_t *folded, uint64_t *queued);
int tempi_hip_stream_wait_event(void *stream, void *event);
/* flags: bit 0 = timing enabled, bit 1 = blocking sync, bit 2 = interprocess */
int tempi_hip_event_create(void **event, int flags);
int tempi_hip_event_destroy(void *event);
int tempi_hip_event_record(void *event, void *stream);
/* returns 0 when complete, 1 when not ready, otherwise an error */
int tempi_hip_event_query(void *event);
int tempi_hip_event_synchronize(void *event);
int tempi_hip_event_elapsed_ms(float *ms, void *start, void *stop);

/* memory */
int tempi_hip_malloc(void **p, size_t n);
int tempi_hip_free(void *p);
/* pinned, mapped host memory: *host for the CPU, *dev for kernels */
int tempi_hip_host_alloc(void **host, void **dev, size_t n);
int tempi_hip_host_free(void *host);
int tempi_hip_host_register(void *host, size_t n, void **dev);
int tempi_hip_host_unregister(void *host);
int tempi_hip_memcpy(void *dst, const void *src, size_t n);
int tempi_hip_memcpy_async(void *dst, const void *src, size_t n, void *stream);
int tempi_hip_memset_async(void *dst, int value, size_t n, void *stream);

/* inter-process (same node) device memory: 64-byte opaque handles */
#define TEMPI_HIP_IPC_HANDLE_BYTES 64
int tempi_hip_ipc_get_handle(void *handle_out, void *devptr);
int tempi_hip_ipc_open_handle(void **devptr, const void *handle);
int tempi_hip_ipc_close_handle(void *devptr);
/* the device allocation holding p: its base, size and process-unique buffer
   id (an allocation freed and replaced at the same address gets a new id) */
int tempi_hip_mem_info(const void *p, void **base, size_t *size, uint64_t *buffer_id);

const char *tempi_hip_error_string(int status);

#ifdef __cplusplus
}
#endif
#endif
