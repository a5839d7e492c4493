// tools/vram_probe.hip -- can the host write device memory directly (large
// BAR), and how soon does a polling kernel see it? Candidates for the
// resident packer's request mailbox: pinned host memory (the kernel polls
// across the host link) against fine-grained device memory the CPU maps
// (the host's store crosses the link once, the kernel polls locally).
// Echo round trips (host writes i, a one-lane kernel waits for i and writes i
// back to pinned host memory), medians of REPS, per mailbox kind.
// usage: vram_probe [REPS]
//   hipcc --offload-arch=gfx950 -O2 -o tools/bin/vram_probe tools/vram_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static double med(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v.empty() ? -1 : v[v.size() / 2];
}

// wait (bounded) for *in == i, then *out = i; scope: agent (device mailbox) or system
template <bool SYS> __global__ void echo(const uint32_t *in, uint32_t *out, uint32_t n) {
  if (threadIdx.x) return;
  for (uint32_t i = 1; i <= n; ++i) {
    const uint64_t t0 = wall_clock64();
    for (;;) {
      const uint32_t v = SYS ? __hip_atomic_load(in, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                             : __hip_atomic_load(in, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (v == i) break;
      if (wall_clock64() - t0 > 100000000ull) { // 1 s
        __hip_atomic_store(out, 0xffffffffu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
      }
    }
    __hip_atomic_store(out, i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

static int run(const char *name, uint32_t *inHost, const uint32_t *inDev, bool sys, uint32_t *outHost,
               uint32_t *outDev, int reps) {
  *outHost = 0;
  *inHost = 0;
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking)) return 3;
  if (sys)
    hipLaunchKernelGGL(echo<true>, dim3(1), dim3(64), 0, s, inDev, outDev, uint32_t(reps));
  else
    hipLaunchKernelGGL(echo<false>, dim3(1), dim3(64), 0, s, inDev, outDev, uint32_t(reps));
  std::vector<double> rt;
  bool ok = true;
  for (int i = 1; i <= reps && ok; ++i) {
    const double t0 = now_us();
    __atomic_store_n(inHost, uint32_t(i), __ATOMIC_RELEASE);
    for (;;) {
      const uint32_t v = __atomic_load_n(outHost, __ATOMIC_ACQUIRE);
      if (v == uint32_t(i)) break;
      if (v == 0xffffffffu || now_us() - t0 > 2e6) {
        ok = false;
        break;
      }
    }
    rt.push_back(now_us() - t0);
  }
  hipStreamSynchronize(s);
  hipStreamDestroy(s);
  std::printf("{\"probe\": \"vram_mailbox\", \"mailbox\": \"%s\", \"ok\": %s, \"echo_round_trip_us\": %.2f}\n", name,
              ok ? "true" : "false", med(rt));
  std::fflush(stdout);
  return ok ? 0 : 4;
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 2000;
  uint32_t *pin, *pinDev;
  if (hipHostMalloc(reinterpret_cast<void **>(&pin), 4096, hipHostMallocMapped | hipHostMallocCoherent)) return 3;
  if (hipHostGetDevicePointer(reinterpret_cast<void **>(&pinDev), pin, 0)) return 3;
  // 1. pinned host mailbox (what the resident packer uses)
  int rc = run("pinned_host", pin + 64, pinDev + 64, true, pin, pinDev, reps);
  // 2. fine-grained device memory, if the host can reach it
  void *vram = nullptr;
  hipError_t e = hipExtMallocWithFlags(&vram, 4096, hipDeviceMallocFinegrained);
  hipPointerAttribute_t at{};
  if (e == hipSuccess) e = hipPointerGetAttributes(&at, vram);
  std::printf("{\"probe\": \"vram_alloc\", \"finegrained\": %d, \"hostPointer\": \"%p\", \"devicePointer\": \"%p\", "
              "\"type\": %d}\n",
              int(e), at.hostPointer, at.devicePointer, int(at.type));
  std::fflush(stdout);
  if (e == hipSuccess && at.hostPointer) {
    uint32_t *h = static_cast<uint32_t *>(at.hostPointer);
    rc |= run("finegrained_vram_agent", h, static_cast<uint32_t *>(vram), false, pin, pinDev, reps);
    rc |= run("finegrained_vram_system", h, static_cast<uint32_t *>(vram), true, pin, pinDev, reps);
  }
  // 3. uncached device memory
  void *unc = nullptr;
  e = hipExtMallocWithFlags(&unc, 4096, hipDeviceMallocUncached);
  hipPointerAttribute_t au{};
  if (e == hipSuccess) e = hipPointerGetAttributes(&au, unc);
  std::printf("{\"probe\": \"vram_alloc_uncached\", \"rc\": %d, \"hostPointer\": \"%p\"}\n", int(e), au.hostPointer);
  if (e == hipSuccess && au.hostPointer)
    rc |= run("uncached_vram_system", static_cast<uint32_t *>(au.hostPointer), static_cast<uint32_t *>(unc), true,
              pin, pinDev, reps);
  return rc;
}
