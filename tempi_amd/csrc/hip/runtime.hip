// tempi_amd/csrc/hip/runtime.hip -- HIP runtime half of the C ABI in
// include/tempi_hip.h: devices, pointer classification, streams, events,
// device / pinned-mapped host memory and IPC handles. The C++ interposer
// (libtempi.so) reaches the GPU only through these.
//
// Reference counterparts: streams_init (/root/reference/src/internal/
// streams.cpp:19-28, two non-blocking streams), the event pool flags
// (/root/reference/src/internal/events.cpp:64-65), the allocators'
// cudaMalloc / cudaHostRegister(Mapped) (/root/reference/include/
// allocator_device.hpp:35-43, allocator_host.hpp:31-49), and the pointer test
// of MPI_Pack (/root/reference/src/pack.cpp:42-49).
#include <hip/hip_runtime.h>

#include "tempi_hip.h"
#include "ticket.hpp"

#include <atomic>
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <unordered_map>

#define RET(expr) return int(expr)

extern "C" {

int tempi_hip_device_count(int *n) {
  hipError_t e = hipGetDeviceCount(n);
  if (e != hipSuccess) {
    *n = 0;
    (void)hipGetLastError();
  }
  return int(e);
}
int tempi_hip_get_device(int *dev) { RET(hipGetDevice(dev)); }
int tempi_hip_device_uuid(int device, unsigned char uuid[16]) {
  hipUUID u;
  std::memset(&u, 0, sizeof u);
  hipError_t e = hipDeviceGetUuid(&u, device);
  if (e != hipSuccess || std::all_of(u.bytes, u.bytes + 16, [](char c) { return c == 0; })) {
    (void)hipGetLastError();
    char bus[64] = {0}; // no UUID: the PCI bus id, zero padded
    e = hipDeviceGetPCIBusId(bus, int(sizeof bus), device);
    if (e != hipSuccess) RET(e);
    std::memset(uuid, 0, 16);
    for (int i = 0; bus[i] && i < 64; ++i) uuid[i % 16] ^= static_cast<unsigned char>(bus[i]);
    return 0;
  }
  std::memcpy(uuid, u.bytes, 16);
  return 0;
}
int tempi_hip_set_device(int dev) { RET(hipSetDevice(dev)); }
int tempi_hip_can_access_peer(int device, int peer) {
  if (device == peer) return 1;
  int can = 0;
  if (hipDeviceCanAccessPeer(&can, device, peer) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return can ? 1 : 0;
}
int tempi_hip_device_synchronize(void) { RET(hipDeviceSynchronize()); }

int tempi_hip_pointer_info(const void *p, tempi_hip_ptrinfo *out) {
  out->kind = TEMPI_HIP_MEM_HOST;
  out->device = -1;
  out->device_ptr = nullptr;
  if (!p) return 0;
  hipPointerAttribute_t a;
  std::memset(&a, 0, sizeof a);
  hipError_t e = hipPointerGetAttributes(&a, p);
  if (e != hipSuccess) {
    (void)hipGetLastError(); // unregistered host memory: not an error for us
    return 0;
  }
  switch (a.type) {
  case hipMemoryTypeDevice:
    out->kind = TEMPI_HIP_MEM_DEVICE;
    break;
  case hipMemoryTypeHost:
    out->kind = TEMPI_HIP_MEM_PINNED;
    break;
  case hipMemoryTypeManaged:
  case hipMemoryTypeUnified:
    out->kind = TEMPI_HIP_MEM_MANAGED;
    break;
  default:
    return 0; // unregistered
  }
  out->device = a.device;
  out->device_ptr = a.devicePointer;
  if (!out->device_ptr) out->kind = TEMPI_HIP_MEM_HOST;
  return 0;
}

int tempi_hip_stream_create(void **stream) {
  hipStream_t s = nullptr;
  hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  *stream = s;
  RET(e);
}
int tempi_hip_stream_create_priority(void **stream, int high) {
  int least = 0, greatest = 0;
  hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest);
  if (e != hipSuccess) return int(e);
  hipStream_t s = nullptr;
  e = hipStreamCreateWithPriority(&s, hipStreamNonBlocking, high ? greatest : least);
  *stream = s;
  RET(e);
}
int tempi_hip_stream_destroy(void *stream) { RET(hipStreamDestroy(static_cast<hipStream_t>(stream))); }
int tempi_hip_stream_synchronize(void *stream) {
  RET(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
}
int tempi_hip_stream_query(void *stream) {
  const hipError_t e = hipStreamQuery(static_cast<hipStream_t>(stream));
  if (e == hipSuccess) return 0;
  if (e == hipErrorNotReady) {
    (void)hipGetLastError();
    return 1;
  }
  RET(e);
}

} // extern "C"

namespace {
// one-lane kernel queued behind a synchronous call's work: its system-scope
// release store of `ticket` to pinned host memory is what the host waits for
__global__ void signal_ticket(uint32_t *flag, uint32_t ticket) {
  if (threadIdx.x == 0) __hip_atomic_store(flag, ticket, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
// one flag per stream: tickets reach a stream in increasing order (issued
// under the mutex), so a flag >= mine means the work before my ticket is done
std::unordered_map<void *, tempi_ticket::Ticket> tickets;
} // namespace

namespace tempi_ticket {

std::mutex &mutex() {
  static std::mutex m;
  return m;
}

Stats &stats() {
  static Stats s;
  return s;
}

Ticket *of(hipStream_t s) {
  Ticket &t = tickets[s];
  if (!t.host) {
    void *h = nullptr, *d = nullptr;
    hipError_t e = hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable);
    if (e == hipSuccess) e = hipHostGetDevicePointer(&d, h, 0);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      return nullptr;
    }
    t.host = static_cast<uint32_t *>(h);
    t.dev = static_cast<uint32_t *>(d);
    __atomic_store_n(t.host, 0u, __ATOMIC_RELEASE);
  }
  if (!t.counter || t.broken) { // (re)start the workgroup count at 0 once the stream is idle
    if (!t.counter && hipMalloc(reinterpret_cast<void **>(&t.counter), kCounterWords * sizeof(uint32_t)) != hipSuccess) {
      (void)hipGetLastError();
      t.counter = nullptr;
      return &t; // tickets work; folds are refused (no counter)
    }
    if (hipStreamSynchronize(s) != hipSuccess ||
        hipMemsetAsync(t.counter, 0, kCounterWords * sizeof(uint32_t), s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
      (void)hipGetLastError();
      t.broken = true;
      return &t;
    }
    for (uint32_t &c : t.counted) c = 0;
    t.broken = false;
  }
  return &t;
}

hipError_t queue_kernel(Ticket &t, hipStream_t s, uint32_t ticket) {
  stats().queued++;
  hipLaunchKernelGGL(signal_ticket, dim3(1), dim3(64), 0, s, t.dev, ticket);
  return hipGetLastError();
}

int wait(hipStream_t s, const uint32_t *flag, uint32_t ticket) {
  for (uint32_t spins = 1;; ++spins) {
    if (int32_t(__atomic_load_n(flag, __ATOMIC_ACQUIRE) - ticket) >= 0) return 0;
    if ((spins & 1023) == 0) { // ~20 µs of pause loops
      const hipError_t e = hipStreamQuery(s);
      if (e == hipSuccess) return 0;
      if (e != hipSuccess && e != hipErrorNotReady) return int(e);
    }
    __builtin_ia32_pause();
  }
}

uint32_t fold_max_blocks() {
  static const uint32_t v = [] {
    const char *e = std::getenv("TEMPI_FOLD_MAX_BLOCKS");
    return e ? uint32_t(std::strtoul(e, nullptr, 10)) : uint32_t(TEMPI_FOLD_MAX_BLOCKS);
  }();
  return v;
}

uint32_t fold_max_blocks_wt() {
  static const uint32_t v = [] {
    const char *e = std::getenv("TEMPI_FOLD_MAX_BLOCKS_WT");
    return e ? uint32_t(std::strtoul(e, nullptr, 10)) : uint32_t(TEMPI_FOLD_MAX_BLOCKS_WT);
  }();
  return v;
}

} // namespace tempi_ticket

extern "C" {

// Wait for everything queued on `stream` the quick way: a kernel enqueued
// behind it stores a ticket to a pinned flag, and the host spins on the flag.
// Same-stream kernels run in order and each one's writes are visible
// device-wide before the next starts (HIP's stream semantics), so the ticket
// becomes visible only after the work before it is complete and written back
// from L2. On MI355X the host sees it 5 µs sooner than hipStreamSynchronize's
// completion (7.6-8.9 vs 12.9-14.3 µs for a small kernel: tools/flagbench.hip,
// profiles/r02/completion_flag_bench_s13.jsonl). Callers use it only when the
// work wrote device memory or TEMPI's own coherent slabs (host memory of the
// application may be coarse-grained: hipStreamSynchronize's system-scope
// release is what makes it host-visible).
int tempi_hip_stream_ticket(void *stream, const uint32_t **flag, uint32_t *ticket) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  std::lock_guard<std::mutex> lock(tempi_ticket::mutex());
  tempi_ticket::Ticket *t = tempi_ticket::of(s);
  if (!t) return int(hipErrorOutOfMemory);
  *ticket = ++t->next;
  *flag = t->host;
  RET(tempi_ticket::queue_kernel(*t, s, *ticket));
}

void tempi_hip_ticket_stats(uint64_t *folded, uint64_t *queued) {
  std::lock_guard<std::mutex> lock(tempi_ticket::mutex());
  *folded = tempi_ticket::stats().folded;
  *queued = tempi_ticket::stats().queued;
}

int tempi_hip_ticket_wait(void *stream, const uint32_t *flag, uint32_t ticket) {
  return tempi_ticket::wait(static_cast<hipStream_t>(stream), flag, ticket);
}

int tempi_hip_stream_signal_wait(void *stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  const uint32_t *flag = nullptr;
  uint32_t ticket = 0;
  if (tempi_hip_stream_ticket(stream, &flag, &ticket) != 0) RET(hipStreamSynchronize(s));
  return tempi_ticket::wait(s, flag, ticket);
}

int tempi_hip_stream_wait_event(void *stream, void *event) {
  RET(hipStreamWaitEvent(static_cast<hipStream_t>(stream), static_cast<hipEvent_t>(event), 0));
}

int tempi_hip_event_create(void **event, int flags) {
  unsigned f = 0;
  if (!(flags & 1)) f |= hipEventDisableTiming;
  if (flags & 2) f |= hipEventBlockingSync;
  if (flags & 4) f |= hipEventInterprocess | hipEventDisableTiming;
  hipEvent_t ev = nullptr;
  hipError_t e = hipEventCreateWithFlags(&ev, f);
  *event = ev;
  RET(e);
}
int tempi_hip_event_destroy(void *event) { RET(hipEventDestroy(static_cast<hipEvent_t>(event))); }
int tempi_hip_event_record(void *event, void *stream) {
  RET(hipEventRecord(static_cast<hipEvent_t>(event), static_cast<hipStream_t>(stream)));
}
int tempi_hip_event_query(void *event) {
  hipError_t e = hipEventQuery(static_cast<hipEvent_t>(event));
  if (e == hipSuccess) return 0;
  if (e == hipErrorNotReady) {
    (void)hipGetLastError();
    return 1;
  }
  return int(e);
}
int tempi_hip_event_synchronize(void *event) { RET(hipEventSynchronize(static_cast<hipEvent_t>(event))); }
int tempi_hip_event_elapsed_ms(float *ms, void *start, void *stop) {
  RET(hipEventElapsedTime(ms, static_cast<hipEvent_t>(start), static_cast<hipEvent_t>(stop)));
}

int tempi_hip_malloc(void **p, size_t n) { RET(hipMalloc(p, n ? n : 1)); }
int tempi_hip_free(void *p) { RET(hipFree(p)); }

// Pinned slabs are written by kernels and read by the host MPI, or written by
// the host and read by kernels, and then reused for the next message. They are
// allocated coherent (fine-grained): without hipHostMallocCoherent, HIP's
// default (HIP_HOST_COHERENT=0) is coarse-grained host memory, whose lines a
// kernel may find in L2 from the slab's previous message.
int tempi_hip_host_alloc(void **host, void **dev, size_t n) {
  hipError_t e =
      hipHostMalloc(host, n ? n : 1, hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent);
  if (e != hipSuccess) RET(e);
  RET(hipHostGetDevicePointer(dev, *host, 0));
}
int tempi_hip_host_free(void *host) { RET(hipHostFree(host)); }
int tempi_hip_host_register(void *host, size_t n, void **dev) {
  hipError_t e = hipHostRegister(host, n, hipHostRegisterMapped | hipHostRegisterPortable);
  if (e != hipSuccess) RET(e);
  RET(hipHostGetDevicePointer(dev, host, 0));
}
int tempi_hip_host_unregister(void *host) { RET(hipHostUnregister(host)); }

int tempi_hip_memcpy(void *dst, const void *src, size_t n) {
  RET(hipMemcpy(dst, src, n, hipMemcpyDefault));
}
int tempi_hip_memcpy_async(void *dst, const void *src, size_t n, void *stream) {
  RET(hipMemcpyAsync(dst, src, n, hipMemcpyDefault, static_cast<hipStream_t>(stream)));
}
int tempi_hip_memset_async(void *dst, int value, size_t n, void *stream) {
  RET(hipMemsetAsync(dst, value, n, static_cast<hipStream_t>(stream)));
}

int tempi_hip_ipc_get_handle(void *handle_out, void *devptr) {
  static_assert(sizeof(hipIpcMemHandle_t) <= TEMPI_HIP_IPC_HANDLE_BYTES, "ipc handle size");
  hipIpcMemHandle_t h;
  std::memset(&h, 0, sizeof h);
  hipError_t e = hipIpcGetMemHandle(&h, devptr);
  std::memset(handle_out, 0, TEMPI_HIP_IPC_HANDLE_BYTES);
  std::memcpy(handle_out, &h, sizeof h);
  RET(e);
}
int tempi_hip_ipc_open_handle(void **devptr, const void *handle) {
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle, sizeof h);
  RET(hipIpcOpenMemHandle(devptr, h, hipIpcMemLazyEnablePeerAccess));
}
int tempi_hip_ipc_close_handle(void *devptr) { RET(hipIpcCloseMemHandle(devptr)); }

int tempi_hip_mem_info(const void *p, void **base, size_t *size, uint64_t *buffer_id) {
  hipDeviceptr_t b = nullptr;
  size_t n = 0;
  hipError_t e = hipMemGetAddressRange(&b, &n, const_cast<void *>(p));
  if (e != hipSuccess) {
    (void)hipGetLastError();
    RET(e);
  }
  unsigned long long id = 0;
  e = hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, const_cast<void *>(p));
  if (e != hipSuccess) {
    (void)hipGetLastError();
    RET(e);
  }
  *base = b;
  *size = n;
  *buffer_id = uint64_t(id);
  return 0;
}

const char *tempi_hip_error_string(int status) {
  return hipGetErrorString(static_cast<hipError_t>(status));
}

} // extern "C"
