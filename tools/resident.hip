// tools/resident.hip -- prototype for VERDICT r05 next 6 ("attack the
// synchronous small-call floor with a design not yet tried"): a RESIDENT
// packer. Config 1's synchronous MPI_Pack (vector(1024, 512, 1024), 512 KiB)
// spends ~2.5 us in hipLaunchKernel and ~2.4 us in dispatch before a wave runs
// (DESIGN §6.3). Here a kernel stays resident between calls: the host writes
// the request into pinned host memory, one leader wave polls it over the host
// link, hands it to the worker workgroups through device memory, the workers
// gather, and the last one stores the completion flag to pinned host memory.
//
// Request / hand-off records are 64 tagged 8-byte granules ({data dword,
// sequence number}): one wave-wide load reads a whole record, and the record
// is complete when every lane's tag matches -- no separate flag, no ordering
// between the host's granule stores.
//
// Coherence: the gathered bytes were written by an earlier kernel (or copy)
// whose completion the host observed before posting. The per-XCD L2s are not
// coherent with each other, so a reader must invalidate after it sees the
// request: modes
//   xcd  (bit 0): workers are the workgroups on XCC 0 only (HW_REG_XCC_ID);
//                 the leader, on XCC 0 too, invalidates that L2 (an agent-scope
//                 acquire) before handing the request over; the workers load
//                 with sc1 (L1 bypassed), so no per-CU invalidate is needed
//   noinv(bit 1): skip the leader's invalidate (pricing only: NOT coherent)
//   wgacq(bit 2): every worker does its own agent-scope acquire after the
//                 hand-off (workers on any XCD)
// Each mode is validated: between calls a kernel over the whole chip rewrites
// the source with a new pattern (so stale L2 / L1 lines would show), and the
// packed bytes are compared with the expected ones.
//
// Every wave has an exit: the leader after `idle` us without a request (it
// then hands the workers an EXIT record) or `cap` us after the start; workers
// also give up 4 x idle after their last request or at cap + 1 ms.
//
// usage: resident [REPS]   -> one JSON line per variant
//   hipcc --offload-arch=gfx950 -O2 -Iinclude -o tools/bin/resident tools/resident.hip
//         -Ltempi_amd/lib -ltempi_hip -Wl,-rpath,'$ORIGIN/../../tempi_amd/lib'
#include <hip/hip_runtime.h>

#include "tempi_hip.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static double med(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v.empty() ? -1 : v[v.size() / 2];
}
static double pct(std::vector<double> v, double p) {
  std::sort(v.begin(), v.end());
  return v.empty() ? -1 : v[size_t(p * (v.size() - 1))];
}

constexpr int kRows = 1024, kBlk = 512, kStride = 1024;
constexpr int kT = 256; // threads per worker workgroup
constexpr uint32_t kOpPack = 1, kOpExit = 2;
constexpr uint32_t kModeXcd = 1, kModeNoInv = 2, kModeWgAcq = 4;

struct Mail { // pinned, coherent, mapped host memory
  uint64_t req[64];
  uint32_t done;
  uint32_t pad0[31];
  uint32_t exitw; // the first sequence number the exiting server did not serve
  uint32_t pad1[31];
};
struct Dev { // device memory, zeroed before each server launch
  uint32_t arrived;
  uint32_t pad0[31];
  uint32_t ranks;
  uint32_t pad1[31];
  uint64_t bcast[64];
  uint32_t fold;
  uint32_t pad2[31];
  uint32_t nworkers;
  uint32_t pad3[31];
};

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, 0x7fffffff, 0x00020000);
}

__device__ __forceinline__ uint64_t ticks() { return wall_clock64(); } // 100 MHz

__global__ void __launch_bounds__(kT) resident(Mail *m, Dev *dv, uint32_t P, uint32_t firstSeq, uint32_t mode,
                                               uint64_t idle, uint64_t cap) {
  __shared__ uint32_t sreq[64];
  __shared__ uint32_t srank;
  const uint64_t t0 = ticks();
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (threadIdx.x == 0) {
    uint32_t xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    const bool mine = !(mode & kModeXcd) || (xcc & 15) == 0;
    srank = mine ? __hip_atomic_fetch_add(&dv->ranks, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : ~0u;
    __hip_atomic_fetch_add(&dv->arrived, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  const uint32_t rank = srank;
  if (rank > P) return; // (rank 0 leads, 1..P work)

  if (rank == 0) { // ------------------------------------------------ leader
    if (wave != 0) return;
    // the worker count is final once every workgroup has checked in
    uint32_t nw = 0;
    for (;;) {
      if (__hip_atomic_load(&dv->arrived, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x) {
        const uint32_t r = __hip_atomic_load(&dv->ranks, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        nw = (r - 1 < P ? r - 1 : P);
        break;
      }
      if (ticks() - t0 > cap) break;
      __builtin_amdgcn_s_sleep(1);
    }
    if (lane == 0) __hip_atomic_store(&dv->nworkers, nw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t expect = firstSeq;
    uint64_t last = ticks();
    for (;;) {
      const uint64_t g = __hip_atomic_load(&m->req[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      const bool ok = uint32_t(g >> 32) == expect;
      if (__ballot(ok) == ~0ull && nw) {
        uint32_t d = uint32_t(g);
        const uint32_t op = __shfl(d, 0);
        if ((mode & kModeXcd) && !(mode & kModeNoInv)) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        if (lane == 8) d = nw;
        __hip_atomic_store(&dv->bcast[lane], (uint64_t(expect) << 32) | d, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        ++expect;
        last = ticks();
        if (op == kOpExit) break;
        continue;
      }
      const uint64_t now = ticks();
      if (now - last > idle || now - t0 > cap || !nw) {
        __hip_atomic_store(&dv->bcast[lane], (uint64_t(expect) << 32) | (lane == 0 ? kOpExit : 0u),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_store(&m->exitw, expect, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }

  // -------------------------------------------------------------- workers
  const uint32_t w = rank - 1;
  uint32_t expect = firstSeq;
  uint64_t last = ticks();
  for (;;) {
    if (wave == 0) {
      uint32_t d = 0;
      for (;;) {
        const uint64_t g = __hip_atomic_load(&dv->bcast[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__ballot(uint32_t(g >> 32) == expect) == ~0ull) {
          d = uint32_t(g);
          break;
        }
        const uint64_t now = ticks();
        if (now - last > 4 * idle + 100000 || now - t0 > cap + 100000) { // (a lost leader: give up)
          d = lane == 0 ? kOpExit : 0u;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      sreq[lane] = d;
    }
    __syncthreads();
    const uint32_t op = sreq[0];
    if (op != kOpPack) return;
    if (mode & kModeWgAcq) {
      if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    const char *src = reinterpret_cast<const char *>(uint64_t(sreq[1]) | (uint64_t(sreq[2]) << 32));
    char *dst = reinterpret_cast<char *>(uint64_t(sreq[3]) | (uint64_t(sreq[4]) << 32));
    const uint32_t rows = sreq[5], blk = sreq[6], stride = sreq[7], nw = sreq[8];
    const uint32_t cpr = blk / 16, chunks = rows * cpr;
    const __amdgpu_buffer_rsrc_t rs = rsrc(src), rd = rsrc(dst);
    for (uint32_t c = w * kT + threadIdx.x; c < chunks; c += nw * kT) {
      const uint32_t row = c / cpr, col = (c - row * cpr) * 16;
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, int(row * stride + col), 0, 16);   // sc1
      __builtin_amdgcn_raw_buffer_store_b128(v, rd, int(c * 16), 0, 1 | 16);                       // sc0 sc1
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint32_t old = __hip_atomic_fetch_add(&dv->fold, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old + 1 == (expect - firstSeq + 1) * nw)
        __hip_atomic_store(&m->done, expect, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    ++expect;
    last = ticks();
  }
}

// rewrite the source with pattern p over the whole chip (every XCD writes)
__global__ void fill(uint32_t *src, uint32_t n, uint32_t p) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    src[i] = i * 2654435761u + p * 40503u;
}

#define CK(x)                                                                                                      \
  do {                                                                                                             \
    if ((x) != hipSuccess) {                                                                                       \
      std::fprintf(stderr, "%s failed\n", #x);                                                                     \
      return 3;                                                                                                    \
    }                                                                                                              \
  } while (0)

struct Server {
  Mail *m;
  Dev *dv;
  hipStream_t s;
  uint32_t seq = 0;
};

static void post(Mail *m, uint32_t seq, const uint32_t *d) {
  for (int i = 63; i >= 0; --i)
    __atomic_store_n(&m->req[i], (uint64_t(seq) << 32) | d[i], __ATOMIC_RELAXED);
}

// spin for done == seq (true) or exitw == seq / 1 s (false)
static bool wait_done(Mail *m, uint32_t seq) {
  const double t0 = now_us();
  for (;;) {
    if (__atomic_load_n(&m->done, __ATOMIC_ACQUIRE) == seq) return true;
    if (__atomic_load_n(&m->exitw, __ATOMIC_ACQUIRE) == seq || now_us() - t0 > 1e6) return false;
  }
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 2000;
  const int nval = 300;
  uint32_t *src;
  char *dst;
  Dev *dv;
  Mail *m;
  const size_t srcBytes = size_t(kRows) * kStride, dstBytes = size_t(kRows) * kBlk;
  CK(hipMalloc(&src, srcBytes));
  CK(hipMalloc(&dst, dstBytes));
  CK(hipMalloc(&dv, sizeof(Dev)));
  CK(hipHostMalloc(reinterpret_cast<void **>(&m), sizeof(Mail), hipHostMallocMapped | hipHostMallocCoherent));
  std::memset(m, 0, sizeof(Mail));
  Mail *md;
  CK(hipHostGetDevicePointer(reinterpret_cast<void **>(&md), m, 0));
  hipStream_t s, sf;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sf, hipStreamNonBlocking));
  std::vector<uint32_t> host(srcBytes / 4);
  std::vector<char> got(dstBytes), want(dstBytes);

  // baseline: TEMPI's synchronous call (launch + folded ticket)
  {
    tempi_hip_desc d{};
    d.block = kBlk;
    d.ndims = 1;
    d.counts[0] = kRows;
    d.strides[0] = kStride;
    std::vector<double> t;
    for (int i = 0; i < reps + 50; ++i) {
      const uint32_t *flag = nullptr;
      uint32_t ticket = 0;
      const double t0 = now_us();
      if (tempi_hip_pack_ticket(dst, src, &d, s, &flag, &ticket)) return 5;
      if (tempi_hip_ticket_wait(s, flag, ticket)) return 6;
      if (i >= 50) t.push_back(now_us() - t0);
    }
    std::printf("{\"variant\": \"tempi_launch\", \"reps\": %d, \"call_us_p50\": %.2f, \"p10\": %.2f, \"p90\": %.2f}\n",
                reps, med(t), pct(t, 0.1), pct(t, 0.9));
    std::fflush(stdout);
  }

  struct V {
    const char *name;
    uint32_t mode, P, grid;
  };
  const V vs[] = {
      {"xcd_p32", kModeXcd, 32, 8 * 40},
      {"xcd_p64", kModeXcd, 64, 8 * 72},
      {"xcd_p32_noinv", kModeXcd | kModeNoInv, 32, 8 * 40},
      {"any_p64_wgacq", kModeWgAcq, 64, 65},
      {"any_p128_wgacq", kModeWgAcq, 128, 129},
      {"any_p64_noacq", 0, 64, 65},
  };
  const uint64_t idle = 100 * 50000, cap = 100 * 20000000ull; // 50 ms idle, 20 s cap (100 MHz ticks)
  for (const V &v : vs) {
    CK(hipMemset(dv, 0, sizeof(Dev)));
    CK(hipDeviceSynchronize());
    std::memset(m, 0, sizeof(Mail));
    uint32_t seq = 1;
    hipLaunchKernelGGL(resident, dim3(v.grid), dim3(kT), 0, s, md, dv, v.P, seq, v.mode, idle, cap);
    CK(hipGetLastError());
    uint32_t d[64] = {};
    d[0] = kOpPack;
    d[1] = uint32_t(uintptr_t(src));
    d[2] = uint32_t(uintptr_t(src) >> 32);
    d[3] = uint32_t(uintptr_t(dst));
    d[4] = uint32_t(uintptr_t(dst) >> 32);
    d[5] = kRows;
    d[6] = kBlk;
    d[7] = kStride;
    bool ok = true;
    std::vector<double> t;
    for (int i = 0; i < reps + 50 && ok; ++i, ++seq) {
      const double t0 = now_us();
      post(m, seq, d);
      ok = wait_done(m, seq);
      if (i >= 50) t.push_back(now_us() - t0);
    }
    // validation: rewrite the source over the whole chip, pack, compare
    int bad = 0;
    for (int i = 0; i < nval && ok; ++i, ++seq) {
      hipLaunchKernelGGL(fill, dim3(512), dim3(256), 0, sf, src, uint32_t(srcBytes / 4), uint32_t(i + 7));
      CK(hipStreamSynchronize(sf));
      post(m, seq, d);
      ok = wait_done(m, seq);
      CK(hipMemcpyAsync(got.data(), dst, dstBytes, hipMemcpyDeviceToHost, sf));
      CK(hipStreamSynchronize(sf));
      for (uint32_t k = 0; k < srcBytes / 4; ++k) host[k] = k * 2654435761u + uint32_t(i + 7) * 40503u;
      const char *h = reinterpret_cast<const char *>(host.data());
      for (int r = 0; r < kRows; ++r) std::memcpy(want.data() + size_t(r) * kBlk, h + size_t(r) * kStride, kBlk);
      bad += std::memcmp(got.data(), want.data(), dstBytes) != 0;
    }
    // stop: an EXIT request, then the stream drains
    d[0] = kOpExit;
    post(m, seq, d);
    const double te = now_us();
    CK(hipStreamSynchronize(s));
    const double stop = now_us() - te;
    uint32_t nw = 0;
    CK(hipMemcpy(&nw, &dv->nworkers, 4, hipMemcpyDeviceToHost));
    std::printf("{\"variant\": \"%s\", \"mode\": %u, \"P\": %u, \"workers\": %u, \"grid\": %u, \"reps\": %d, "
                "\"served\": %s, \"call_us_p50\": %.2f, \"p10\": %.2f, \"p90\": %.2f, \"validated\": %d, "
                "\"stale_or_wrong\": %d, \"stop_us\": %.1f, \"exitw\": %u}\n",
                v.name, v.mode, v.P, nw, v.grid, reps, ok ? "true" : "false", med(t), pct(t, 0.1), pct(t, 0.9), nval,
                bad, stop, m->exitw);
    std::fflush(stdout);
    if (!ok) return 7;
  }
  return 0;
}
