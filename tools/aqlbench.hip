// tools/aqlbench.hip -- what the HIP launch costs a synchronous small call,
// against an AQL dispatch packet written straight into an HSA queue of our
// own (no HIP runtime on the launch path). One kernel, one 64-lane
// workgroup: copies N 16-byte words and stores a ticket (system scope) that
// the host polls. Per call, median of REPS:
//   hip_launch_us   hipLaunchKernelGGL alone (host side)
//   hip_ticket_us   hipLaunchKernelGGL + spin on the ticket
//   aql_submit_us   packet write + doorbell alone (host side)
//   aql_ticket_us   packet + doorbell + spin on the ticket
// The kernel reads no implicit (hidden) kernel arguments, so the AQL path
// fills only the explicit ones.
// build: hipcc --offload-arch=gfx950 -O2 -std=c++17 -o tools/_variants/aqlbench tools/aqlbench.hip -lhsa-runtime64
//        hipcc --offload-arch=gfx950 -O3 --offload-device-only --no-gpu-bundle-output -c -o tools/_variants/aqlbench.hsaco tools/aqlbench.hip -DKERNEL_ONLY
// usage: aqlbench HSACO [REPS]
#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>

extern "C" __global__ void __launch_bounds__(64) ticket_copy(const uint4 *src, uint4 *dst, uint32_t n,
                                                            uint32_t *flag, uint32_t ticket) {
  for (uint32_t i = threadIdx.x; i < n; i += 64) dst[i] = src[i];
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(flag, ticket, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

#ifndef KERNEL_ONLY
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}
#define HK(x) do { hsa_status_t s_ = (x); if (s_ != HSA_STATUS_SUCCESS) { std::fprintf(stderr, "%s: %d\n", #x, int(s_)); return 3; } } while (0)
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::fprintf(stderr, "%s: %d\n", #x, int(e_)); return 3; } } while (0)

struct Found {
  hsa_agent_t gpu{};
  bool have = false;
  hsa_region_t kernarg{};
  bool haveKernarg = false;
};

static hsa_status_t find_gpu(hsa_agent_t a, void *d) {
  auto *f = static_cast<Found *>(d);
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_GPU && !f->have) {
    f->gpu = a;
    f->have = true;
  }
  return HSA_STATUS_SUCCESS;
}
static hsa_status_t find_kernarg(hsa_region_t r, void *d) {
  auto *f = static_cast<Found *>(d);
  hsa_region_segment_t seg;
  hsa_region_get_info(r, HSA_REGION_INFO_SEGMENT, &seg);
  if (seg != HSA_REGION_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
  uint32_t flags = 0;
  hsa_region_get_info(r, HSA_REGION_INFO_GLOBAL_FLAGS, &flags);
  if ((flags & HSA_REGION_GLOBAL_FLAG_KERNARG) && !f->haveKernarg) {
    f->kernarg = r;
    f->haveKernarg = true;
  }
  return HSA_STATUS_SUCCESS;
}

struct Pools {
  hsa_amd_memory_pool_t devFine{};
  bool have = false;
};
static hsa_status_t find_dev_fine(hsa_amd_memory_pool_t p, void *d) {
  auto *f = static_cast<Pools *>(d);
  hsa_amd_segment_t seg;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
  if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
  uint32_t flags = 0;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
  bool alloc = false;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &alloc);
  if (alloc && (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_FINE_GRAINED) && !f->have) {
    f->devFine = p;
    f->have = true;
  }
  return HSA_STATUS_SUCCESS;
}
static hsa_status_t find_cpu(hsa_agent_t a, void *d) {
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_CPU) *static_cast<hsa_agent_t *>(d) = a;
  return HSA_STATUS_SUCCESS;
}

struct Args {
  const void *src;
  void *dst;
  uint32_t n;
  uint32_t pad;
  uint32_t *flag;
  uint32_t ticket;
};

int main(int argc, char **argv) {
  if (argc < 2) return 1;
  const int reps = argc > 2 ? std::atoi(argv[2]) : 2000;
  CK(hipSetDevice(0));
  CK(hipFree(nullptr));
  HK(hsa_init());
  Found f;
  hsa_iterate_agents(find_gpu, &f);
  if (!f.have) return 4;
  hsa_agent_iterate_regions(f.gpu, find_kernarg, &f);
  if (!f.haveKernarg) return 5;
  // the code object
  FILE *fp = fopen(argv[1], "rb");
  if (!fp) return 6;
  std::vector<char> blob;
  {
    fseek(fp, 0, SEEK_END);
    blob.resize(size_t(ftell(fp)));
    fseek(fp, 0, SEEK_SET);
    if (fread(blob.data(), 1, blob.size(), fp) != blob.size()) return 6;
    fclose(fp);
  }
  hsa_code_object_reader_t reader;
  HK(hsa_code_object_reader_create_from_memory(blob.data(), blob.size(), &reader));
  hsa_executable_t exe;
  HK(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &exe));
  HK(hsa_executable_load_agent_code_object(exe, f.gpu, reader, nullptr, nullptr));
  HK(hsa_executable_freeze(exe, nullptr));
  hsa_executable_symbol_t sym;
  HK(hsa_executable_get_symbol_by_name(exe, "ticket_copy.kd", &f.gpu, &sym));
  uint64_t kobj = 0;
  uint32_t kargSize = 0, groupSize = 0, privSize = 0;
  HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &kobj));
  HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &kargSize));
  HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &groupSize));
  HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &privSize));
  std::fprintf(stderr, "kernel object %llx kernarg %u group %u private %u\n", (unsigned long long)kobj, kargSize,
               groupSize, privSize);
  if (kargSize < offsetof(Args, ticket) + sizeof(uint32_t)) return 7;
  hsa_queue_t *q = nullptr;
  HK(hsa_queue_create(f.gpu, 64, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q));
  // kernarg buffers: one per queue slot (a packet's arguments stay until it ran)
  void *kargs = nullptr;
  HK(hsa_memory_allocate(f.kernarg, size_t(q->size) * 512, &kargs));
  std::memset(kargs, 0, size_t(q->size) * 512);

  // kernel arguments in device memory the host writes through the BAR (what
  // HIP does for its own launches on MI300-class parts), when the GPU has a
  // fine-grained pool the CPU may be given access to
  void *devKargs = nullptr;
  {
    Pools pools;
    hsa_amd_agent_iterate_memory_pools(f.gpu, find_dev_fine, &pools);
    hsa_agent_t cpu{};
    hsa_iterate_agents(find_cpu, &cpu);
    if (pools.have && hsa_amd_memory_pool_allocate(pools.devFine, size_t(q->size) * 512, 0, &devKargs) ==
                          HSA_STATUS_SUCCESS) {
      if (hsa_amd_agents_allow_access(1, &cpu, nullptr, devKargs) != HSA_STATUS_SUCCESS) {
        hsa_amd_memory_pool_free(devKargs);
        devKargs = nullptr;
      }
    }
    std::fprintf(stderr, "device kernarg buffer: %s\n", devKargs ? "yes" : "no");
  }

  void *src = nullptr, *dst = nullptr;
  uint32_t *flag = nullptr;
  CK(hipMalloc(&src, 1 << 20));
  CK(hipMalloc(&dst, 1 << 20));
  CK(hipMemset(src, 7, 1 << 20));
  CK(hipHostMalloc(reinterpret_cast<void **>(&flag), 64, hipHostMallocCoherent));
  *flag = 0;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipDeviceSynchronize());

  for (uint32_t n : {64u, 1024u, 32768u}) { // 1 KiB, 16 KiB, 512 KiB (one workgroup: latency, not bandwidth)
    std::vector<double> hl, ht, as, at, dt;
    uint32_t ticket = 0;
    for (int r = 0; r < reps + 50; ++r) {
      const bool keep = r >= 50;
      // HIP
      ++ticket;
      double t0 = now_us();
      hipLaunchKernelGGL(ticket_copy, dim3(1), dim3(64), 0, s, static_cast<const uint4 *>(src),
                         static_cast<uint4 *>(dst), n, flag, ticket);
      double t1 = now_us();
      while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != ticket) {
      }
      double t2 = now_us();
      // AQL, kernel arguments in system memory, then in device memory
      for (int variant = 0; variant < (devKargs ? 2 : 1); ++variant) {
        char *kbase = static_cast<char *>(variant ? devKargs : kargs);
        ++ticket;
        double t3 = now_us();
        const uint64_t idx = hsa_queue_add_write_index_scacq_screl(q, 1);
        while (idx - hsa_queue_load_read_index_scacquire(q) >= q->size) {
        }
        Args *a = reinterpret_cast<Args *>(kbase + (idx % q->size) * 512);
        a->src = src;
        a->dst = dst;
        a->n = n;
        a->flag = flag;
        a->ticket = ticket;
        auto *pkt = static_cast<hsa_kernel_dispatch_packet_t *>(q->base_address) + (idx % q->size);
        pkt->workgroup_size_x = 64;
        pkt->workgroup_size_y = 1;
        pkt->workgroup_size_z = 1;
        pkt->reserved0 = 0;
        pkt->grid_size_x = 64;
        pkt->grid_size_y = 1;
        pkt->grid_size_z = 1;
        pkt->private_segment_size = privSize;
        pkt->group_segment_size = groupSize;
        pkt->kernel_object = kobj;
        pkt->kernarg_address = a;
        pkt->reserved2 = 0;
        pkt->completion_signal.handle = 0;
        const uint16_t header = uint16_t((HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                                         (1 << HSA_PACKET_HEADER_BARRIER) |
                                         (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                         (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
        const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
        if (variant) { // the BAR writes land before the packet is valid
          __atomic_thread_fence(__ATOMIC_SEQ_CST);
          (void)*reinterpret_cast<volatile uint32_t *>(&a->ticket);
        }
        __atomic_store_n(reinterpret_cast<uint32_t *>(pkt), uint32_t(header) | (uint32_t(setup) << 16),
                         __ATOMIC_RELEASE);
        hsa_signal_store_screlease(q->doorbell_signal, hsa_signal_value_t(idx));
        double t4 = now_us();
        const double limit = t4 + 2e6;
        while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != ticket) {
          if (now_us() > limit) {
            std::fprintf(stderr, "AQL dispatch never completed\n");
            return 8;
          }
        }
        double t5 = now_us();
        if (keep) {
          if (variant) {
            dt.push_back(t5 - t3);
          } else {
            as.push_back(t4 - t3);
            at.push_back(t5 - t3);
          }
        }
      }
      if (keep) {
        hl.push_back(t1 - t0);
        ht.push_back(t2 - t0);
      }
    }
    // the copy really ran: dst equals src
    CK(hipDeviceSynchronize());
    std::vector<unsigned char> h(size_t(n) * 16);
    CK(hipMemcpy(h.data(), dst, h.size(), hipMemcpyDeviceToHost));
    bool ok = true;
    for (unsigned char c : h) ok &= c == 7;
    std::printf("{\"bench\": \"aqlbench\", \"bytes\": %u, \"reps\": %d, \"hip_launch_us\": %.2f, \"hip_ticket_us\": %.2f, "
                "\"aql_submit_us\": %.2f, \"aql_ticket_us\": %.2f, \"aql_devkarg_ticket_us\": %.2f, \"copied_ok\": %s}\n",
                n * 16, reps, median(hl), median(ht), median(as), median(at), dt.empty() ? -1.0 : median(dt),
                ok ? "true" : "false");
    std::fflush(stdout);
  }
  hsa_queue_destroy(q);
  hsa_memory_free(kargs);
  if (devKargs) hsa_amd_memory_pool_free(devKargs);
  hsa_executable_destroy(exe);
  hsa_code_object_reader_destroy(reader);
  return 0;
}
#endif
