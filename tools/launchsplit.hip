// tools/launchsplit.hip -- VERDICT r05 next 6: where the synchronous small
// call's wait goes. Config 1 (vector(1024, 512, 1024), 512 KiB) packs in
// ~2.4 us of kernel, yet MPI_Pack's ticket wait after the launch returns is
// ~5.5 us. This splits launch -> ticket into
//   dispatch    launch call returned -> the first workgroup runs
//   execution   first workgroup runs -> last workgroup done
//   visibility  a store to pinned host memory -> the host sees it
// with a kernel of the packer's grid (256 workgroups x 128 lanes, 16 B per
// lane, the config-1 rows) that stores a flag to pinned host memory from the
// first workgroup to start and from the last to finish (a device counter, as
// the ticket's), and with a one-lane echo kernel that measures the one-way
// visibility: the host writes i, the kernel waits for it and writes i back
// (round trip / 2). Host times around each step, medians of REPS.
//   host_seen_first - launch_returned = dispatch + visibility
//   host_seen_last  - host_seen_first = execution (both carry one visibility)
// It also times TEMPI's own call (tempi_hip_pack_ticket + ticket_wait) and a
// bare launch + hipStreamSynchronize for comparison.
// usage: launchsplit [REPS]
//   hipcc --offload-arch=gfx950 -O2 -Iinclude -o tools/_variants/launchsplit tools/launchsplit.hip
//         -Ltempi_amd/lib -ltempi_hip -Wl,-rpath,'$ORIGIN/../../tempi_amd/lib'
#include <hip/hip_runtime.h>

#include "tempi_hip.h"

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

constexpr int kRows = 1024, kBlock = 512, kStride = 1024;

// flags[0]: first workgroup started (seq); flags[32]: last workgroup done
// (seq); stamps[0 / 1]: wall_clock64 at the first start / last end
__global__ void __launch_bounds__(128) stamped_pack(const char *src, char *dst, uint32_t *flags, uint32_t *counter,
                                                    uint64_t *stamps, uint32_t seq) {
  __shared__ uint32_t first;
  if (threadIdx.x == 0) {
    const uint32_t old = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    first = old == (seq - 1) * 2 * gridDim.x;
    if (first) {
      stamps[0] = wall_clock64();
      __hip_atomic_store(flags, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  __syncthreads();
  // chunk c = 16 bytes of the packed side: row c / 32, column (c % 32) * 16
  const uint32_t c = blockIdx.x * 128 + threadIdx.x;
  const uint32_t row = c / (kBlock / 16), col = (c % (kBlock / 16)) * 16;
  const uint4 v = *reinterpret_cast<const uint4 *>(src + size_t(row) * kStride + col);
  *reinterpret_cast<uint4 *>(dst + size_t(c) * 16) = v;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const uint32_t old = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old + 1 == seq * 2 * gridDim.x) {
      stamps[1] = wall_clock64();
      __hip_atomic_store(flags + 32, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// one lane: for i in 1..n wait (bounded) for h2d == i, then d2h = i; a wait
// that runs out stores 0xffffffff and ends the kernel (every path exits)
__global__ void echo(const uint32_t *h2d, uint32_t *d2h, uint32_t n) {
  if (threadIdx.x != 0) return;
  for (uint32_t i = 1; i <= n; ++i) {
    uint32_t spins = 0;
    while (__hip_atomic_load(h2d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != i) {
      if (++spins > (1u << 24)) {
        __hip_atomic_store(d2h, 0xffffffffu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    __hip_atomic_store(d2h, i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

static bool spin_until(volatile uint32_t *p, uint32_t v, double *t) {
  const double t0 = now_us();
  for (;;) {
    const uint32_t x = __atomic_load_n(p, __ATOMIC_ACQUIRE);
    if (x == v) {
      *t = now_us();
      return true;
    }
    if (x == 0xffffffffu || now_us() - t0 > 1e6) return false;
  }
}

#define CK(x)                                                                                                      \
  do {                                                                                                             \
    if ((x) != hipSuccess) {                                                                                       \
      std::fprintf(stderr, "%s failed\n", #x);                                                                     \
      return 3;                                                                                                    \
    }                                                                                                              \
  } while (0)

int main(int argc, char **argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 1000;
  char *src, *dst;
  uint32_t *flags, *counter;
  uint64_t *stamps;
  CK(hipMalloc(&src, size_t(kRows) * kStride));
  CK(hipMalloc(&dst, size_t(kRows) * kBlock));
  CK(hipMalloc(&counter, 256));
  CK(hipMalloc(&stamps, 64));
  CK(hipMemset(counter, 0, 256));
  CK(hipHostMalloc(reinterpret_cast<void **>(&flags), 4096, hipHostMallocMapped | hipHostMallocCoherent));
  for (int i = 0; i < 1024; ++i) flags[i] = 0;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const uint32_t grid = kRows * kBlock / 16 / 128; // 256

  // 1. one-way visibility: echo round trips
  uint32_t *h2d = flags + 64, *d2h = flags + 96;
  const uint32_t nEcho = uint32_t(reps);
  hipLaunchKernelGGL(echo, dim3(1), dim3(64), 0, s, h2d, d2h, nEcho);
  CK(hipGetLastError());
  std::vector<double> rt;
  bool echoOk = true;
  for (uint32_t i = 1; i <= nEcho && echoOk; ++i) {
    const double t0 = now_us();
    __atomic_store_n(h2d, i, __ATOMIC_RELEASE);
    double t1;
    echoOk = spin_until(d2h, i, &t1);
    rt.push_back(t1 - t0);
  }
  CK(hipStreamSynchronize(s));
  const double oneway = med(rt) / 2;

  // 2. the stamped pack: launch, first workgroup seen, last seen
  std::vector<double> launch, first, exec, total, devExec;
  uint32_t seq = 0;
  for (int i = 0; i < reps + 50 && echoOk; ++i) {
    ++seq;
    const double t0 = now_us();
    hipLaunchKernelGGL(stamped_pack, dim3(grid), dim3(128), 0, s, src, dst, flags, counter, stamps, seq);
    const double t1 = now_us();
    double t2, t3;
    if (!spin_until(flags, seq, &t2) || !spin_until(flags + 32, seq, &t3)) {
      std::fprintf(stderr, "stamped_pack %u: flag never seen\n", seq);
      return 4;
    }
    CK(hipStreamSynchronize(s));
    if (i >= 50) {
      uint64_t st[2];
      CK(hipMemcpy(st, stamps, 16, hipMemcpyDeviceToHost));
      launch.push_back(t1 - t0);
      first.push_back(t2 - t1);
      exec.push_back(t3 - t2);
      total.push_back(t3 - t0);
      devExec.push_back(double(st[1] - st[0]) / 100.0); // wall_clock64: 100 MHz
    }
  }

  // 3. TEMPI's call and HIP's synchronise path on the same object
  tempi_hip_desc d{};
  d.block = kBlock;
  d.ndims = 1;
  d.counts[0] = kRows;
  d.strides[0] = kStride;
  std::vector<double> tl, tw, hs;
  for (int i = 0; i < reps + 50; ++i) {
    const uint32_t *flag = nullptr;
    uint32_t ticket = 0;
    const double t0 = now_us();
    if (tempi_hip_pack_ticket(dst, src, &d, s, &flag, &ticket)) return 5;
    const double t1 = now_us();
    if (tempi_hip_ticket_wait(s, flag, ticket)) return 6;
    const double t2 = now_us();
    if (tempi_hip_pack(dst, src, &d, s)) return 7;
    CK(hipStreamSynchronize(s));
    const double t3 = now_us();
    if (i >= 50) {
      tl.push_back(t1 - t0);
      tw.push_back(t2 - t1);
      hs.push_back(t3 - t2);
    }
  }
  std::printf("{\"bench\": \"launchsplit\", \"reps\": %d, \"echo_ok\": %s, \"oneway_visibility_us\": %.2f, "
              "\"launch_us\": %.2f, \"launch_to_first_seen_us\": %.2f, \"dispatch_us\": %.2f, "
              "\"first_to_last_seen_us\": %.2f, \"device_exec_us\": %.2f, \"launch_to_last_seen_us\": %.2f, "
              "\"tempi_launch_us\": %.2f, \"tempi_ticket_wait_us\": %.2f, \"tempi_launch_plus_stream_sync_us\": %.2f}\n",
              reps, echoOk ? "true" : "false", oneway, med(launch), med(first), med(first) - oneway, med(exec),
              med(devExec), med(total), med(tl), med(tw), med(hs));
  return echoOk ? 0 : 8;
}
