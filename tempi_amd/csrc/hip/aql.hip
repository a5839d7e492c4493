// tempi_amd/csrc/hip/aql.hip -- see aql.hpp.
#include "aql.hpp"

#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <hsa/hsa_ven_amd_loader.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

namespace tempi_aql {

namespace {

struct Kernel {
  uint64_t object = 0;
  uint32_t group = 0, priv = 0, kargSize = 0;
  int misses = 0; // lookups that found nothing (HIP may not have loaded it yet)
  bool ok = false;
};

// kernarg slot per queue packet: explicit arguments (<= 512 B here) + the
// 256 bytes of implicit ones
constexpr size_t kSlot = 1024;
constexpr uint32_t kQueueSize = 64;
// code object v5 implicit arguments, from their start (8-byte aligned after
// the explicit ones): block counts x/y/z (u32), group sizes x/y/z (u16),
// remainders x/y/z (u16), global offsets x/y/z (u64) at 40, grid dims (u16) at 64
constexpr size_t kImplicitBytes = 256;
constexpr size_t kGroupSizeAt = 12, kGridDimsAt = 64;

std::mutex mu;
bool hsaTried = false, hsaReady = false;
hsa_ven_amd_loader_1_03_pfn_t loader{};
std::atomic<bool> queueFailed{false};
Stats counts;

bool enabled() {
  static const bool on = [] {
    const char *e = std::getenv("TEMPI_AQL");
    return e && *e && std::strcmp(e, "0") != 0;
  }();
  return on;
}

void on_queue_error(hsa_status_t status, hsa_queue_t *, void *) {
  const char *msg = nullptr;
  hsa_status_string(status, &msg);
  std::fprintf(stderr, "[tempi] AQL queue error: %s\n", msg ? msg : "unknown");
  queueFailed = true;
}

bool init_hsa() {
  if (hsaTried) return hsaReady;
  hsaTried = true;
  if (hsa_init() != HSA_STATUS_SUCCESS) return false; // (reference counted: HIP's ROCr is the same)
  if (hsa_system_get_major_extension_table(HSA_EXTENSION_AMD_LOADER, 1, sizeof loader, &loader) !=
      HSA_STATUS_SUCCESS)
    return false;
  hsaReady = true;
  return true;
}

struct AgentFind {
  uint32_t bdf = 0, domain = 0;
  hsa_agent_t agent{};
  bool found = false;
  hsa_region_t kernarg{};
  bool haveKernarg = false;
};

hsa_status_t find_agent(hsa_agent_t a, void *d) {
  auto *f = static_cast<AgentFind *>(d);
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS || t != HSA_DEVICE_TYPE_GPU)
    return HSA_STATUS_SUCCESS;
  uint32_t bdf = 0, domain = 0;
  hsa_agent_get_info(a, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_BDFID), &bdf);
  hsa_agent_get_info(a, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_DOMAIN), &domain);
  if ((bdf & ~7u) == (f->bdf & ~7u) && domain == f->domain) { // (bus, device); any function
    f->agent = a;
    f->found = true;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

hsa_status_t find_kernarg(hsa_region_t r, void *d) {
  auto *f = static_cast<AgentFind *>(d);
  hsa_region_segment_t seg;
  if (hsa_region_get_info(r, HSA_REGION_INFO_SEGMENT, &seg) != HSA_STATUS_SUCCESS || seg != HSA_REGION_SEGMENT_GLOBAL)
    return HSA_STATUS_SUCCESS;
  uint32_t flags = 0;
  hsa_region_get_info(r, HSA_REGION_INFO_GLOBAL_FLAGS, &flags);
  if (flags & HSA_REGION_GLOBAL_FLAG_KERNARG) {
    f->kernarg = r;
    f->haveKernarg = true;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

// a device-memory pool the CPU may be given access to (kernel arguments the
// host writes through the BAR, read by the GPU from its own memory)
struct PoolFind {
  hsa_amd_memory_pool_t pool{};
  bool found = false;
};

hsa_status_t find_device_pool(hsa_amd_memory_pool_t p, void *d) {
  auto *f = static_cast<PoolFind *>(d);
  hsa_amd_segment_t seg;
  if (hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg) != HSA_STATUS_SUCCESS ||
      seg != HSA_AMD_SEGMENT_GLOBAL)
    return HSA_STATUS_SUCCESS;
  uint32_t flags = 0;
  bool alloc = false;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &alloc);
  if (alloc && (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_FINE_GRAINED)) {
    f->pool = p;
    f->found = true;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

hsa_status_t find_cpu(hsa_agent_t a, void *d) {
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_CPU) {
    *static_cast<hsa_agent_t *>(d) = a;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

struct SymFind {
  const char *name;
  hsa_agent_t agent;
  hsa_executable_symbol_t sym{};
  bool found = false;
};

hsa_status_t find_symbol(hsa_executable_t exe, void *d) {
  auto *f = static_cast<SymFind *>(d);
  hsa_executable_symbol_t s;
  if (hsa_executable_get_symbol_by_name(exe, f->name, &f->agent, &s) == HSA_STATUS_SUCCESS) {
    f->sym = s;
    f->found = true;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

} // namespace

struct Queue {
  int device = -1;
  hsa_agent_t agent{};
  hsa_queue_t *q = nullptr;
  char *kargs = nullptr; // kQueueSize slots of kSlot bytes, kernarg memory
  bool deviceKargs = false; // kargs in device memory (TEMPI_AQL_DEVICE_KERNARG=1)
  std::unordered_map<const void *, Kernel> kernels;
};

namespace {

std::vector<Queue *> queues;
std::vector<char> tried;

Queue *make_queue(int dev) {
  int bus = 0, slot = 0, domain = 0;
  if (hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, dev) != hipSuccess ||
      hipDeviceGetAttribute(&slot, hipDeviceAttributePciDeviceId, dev) != hipSuccess ||
      hipDeviceGetAttribute(&domain, hipDeviceAttributePciDomainId, dev) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  AgentFind f;
  f.bdf = uint32_t(bus) << 8 | uint32_t(slot) << 3;
  f.domain = uint32_t(domain);
  hsa_iterate_agents(find_agent, &f);
  if (!f.found) return nullptr;
  hsa_agent_iterate_regions(f.agent, find_kernarg, &f);
  if (!f.haveKernarg) return nullptr;
  hsa_queue_t *q = nullptr;
  if (hsa_queue_create(f.agent, kQueueSize, HSA_QUEUE_TYPE_SINGLE, on_queue_error, nullptr, UINT32_MAX, UINT32_MAX,
                       &q) != HSA_STATUS_SUCCESS)
    return nullptr;
  void *k = nullptr;
  bool deviceKargs = false;
  if (std::getenv("TEMPI_AQL_DEVICE_KERNARG")) {
    PoolFind pf;
    hsa_agent_t cpu{};
    hsa_amd_agent_iterate_memory_pools(f.agent, find_device_pool, &pf);
    hsa_iterate_agents(find_cpu, &cpu);
    if (pf.found && cpu.handle &&
        hsa_amd_memory_pool_allocate(pf.pool, size_t(q->size) * kSlot, 0, &k) == HSA_STATUS_SUCCESS) {
      if (hsa_amd_agents_allow_access(1, &cpu, nullptr, k) == HSA_STATUS_SUCCESS) {
        deviceKargs = true;
      } else {
        hsa_amd_memory_pool_free(k);
        k = nullptr;
      }
    }
  }
  if (!k && hsa_memory_allocate(f.kernarg, size_t(q->size) * kSlot, &k) != HSA_STATUS_SUCCESS) {
    hsa_queue_destroy(q);
    return nullptr;
  }
  std::memset(k, 0, size_t(q->size) * kSlot);
  auto *Q = new Queue;
  Q->device = dev;
  Q->agent = f.agent;
  Q->q = q;
  Q->kargs = static_cast<char *>(k);
  Q->deviceKargs = deviceKargs;
  return Q;
}

Kernel *lookup(Queue &Q, const void *kernel, hipStream_t s) {
  Kernel &k = Q.kernels[kernel];
  if (k.ok) return &k;
  if (k.misses >= 3) return nullptr;
  const char *name = hipKernelNameRefByPtr(kernel, s);
  if (!name) {
    (void)hipGetLastError();
    ++k.misses;
    return nullptr;
  }
  const std::string kd = std::string(name) + ".kd";
  SymFind f{kd.c_str(), Q.agent};
  loader.hsa_ven_amd_loader_iterate_executables(find_symbol, &f);
  if (!f.found) {
    ++k.misses;
    return nullptr;
  }
  if (hsa_executable_symbol_get_info(f.sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &k.object) !=
          HSA_STATUS_SUCCESS ||
      hsa_executable_symbol_get_info(f.sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &k.kargSize) !=
          HSA_STATUS_SUCCESS ||
      hsa_executable_symbol_get_info(f.sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &k.group) !=
          HSA_STATUS_SUCCESS ||
      hsa_executable_symbol_get_info(f.sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &k.priv) !=
          HSA_STATUS_SUCCESS) {
    k.misses = 3;
    return nullptr;
  }
  k.ok = true;
  return &k;
}

} // namespace

Queue *for_stream(hipStream_t s) {
  if (!enabled() || queueFailed) return nullptr;
  int dev = -1;
  if (hipStreamGetDevice(s, &dev) != hipSuccess || dev < 0) {
    (void)hipGetLastError();
    return nullptr;
  }
  std::lock_guard<std::mutex> lock(mu);
  if (!init_hsa()) return nullptr;
  if (size_t(dev) >= queues.size()) {
    queues.resize(size_t(dev) + 1, nullptr);
    tried.resize(size_t(dev) + 1, 0);
  }
  if (!tried[size_t(dev)]) {
    tried[size_t(dev)] = 1;
    queues[size_t(dev)] = make_queue(dev);
    if (!queues[size_t(dev)]) std::fprintf(stderr, "[tempi] TEMPI_AQL: no HSA queue for device %d; HIP launches\n", dev);
  }
  return queues[size_t(dev)];
}

bool dispatch(Queue *Q, const void *kernel, hipStream_t s, uint32_t blocks, uint32_t wg, const void *args,
              size_t bytes) {
  if (!Q || queueFailed || blocks == 0 || wg == 0 || wg > 1024) return false;
  Kernel *k = lookup(*Q, kernel, s);
  const size_t implicitAt = (bytes + 7) & ~size_t(7);
  // the layout written below: explicit arguments only, or followed by code
  // object v5's implicit block
  if (!k || k->kargSize > kSlot || k->kargSize < bytes ||
      (k->kargSize > implicitAt && k->kargSize != implicitAt + kImplicitBytes)) {
    counts.refused++;
    return false;
  }
  hsa_queue_t *q = Q->q;
  const uint64_t idx = hsa_queue_add_write_index_scacq_screl(q, 1);
  while (idx - hsa_queue_load_read_index_scacquire(q) >= q->size) // (a full queue: synchronous callers never fill it)
    __builtin_ia32_pause();
  char *ka = Q->kargs + (idx % q->size) * kSlot;
  std::memcpy(ka, args, bytes);
  if (k->kargSize > bytes) std::memset(ka + bytes, 0, k->kargSize - bytes);
  if (k->kargSize == implicitAt + kImplicitBytes) {
    char *h = ka + implicitAt;
    const uint32_t count[3] = {blocks, 1, 1};
    const uint16_t size[3] = {uint16_t(wg), 1, 1};
    const uint16_t dims = 1;
    std::memcpy(h, count, sizeof count);
    std::memcpy(h + kGroupSizeAt, size, sizeof size);
    std::memcpy(h + kGridDimsAt, &dims, sizeof dims); // (remainders and global offsets stay 0)
  }
  if (Q->deviceKargs) { // the writes through the BAR land before the packet becomes valid
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    (void)*reinterpret_cast<volatile char *>(ka + k->kargSize - 1);
  }
  auto *pkt = static_cast<hsa_kernel_dispatch_packet_t *>(q->base_address) + (idx % q->size);
  pkt->workgroup_size_x = uint16_t(wg);
  pkt->workgroup_size_y = 1;
  pkt->workgroup_size_z = 1;
  pkt->reserved0 = 0;
  pkt->grid_size_x = blocks * wg;
  pkt->grid_size_y = 1;
  pkt->grid_size_z = 1;
  pkt->private_segment_size = k->priv;
  pkt->group_segment_size = k->group;
  pkt->kernel_object = k->object;
  pkt->kernarg_address = ka;
  pkt->reserved2 = 0;
  pkt->completion_signal.handle = 0; // (completion is the kernel's own ticket)
  const uint16_t header = uint16_t((HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                                   (1 << HSA_PACKET_HEADER_BARRIER) |
                                   (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                   (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
  const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
  __atomic_store_n(reinterpret_cast<uint32_t *>(pkt), uint32_t(header) | uint32_t(setup) << 16, __ATOMIC_RELEASE);
  hsa_signal_store_screlease(q->doorbell_signal, hsa_signal_value_t(idx));
  counts.dispatched++;
  return true;
}

bool failed() { return queueFailed; }

Stats stats() { return counts; }

} // namespace tempi_aql
