// tools/xface.hip -- the 512^3 halo's x faces as a bare access pattern, with
// no packer index math (is the x-face copy at the bound
// of its own pattern, and how much of that bound is the partly written
// sectors?). Geometry of one rank's buffers (apps/halo_lib.cpp): 8 quantities,
// 518 x 518 x 518 cells of 8 B, pitch 4608 B, 518 rows per plane; the +x face
// (interior x = 512..514, bytes 4096..4119 of a row) goes to the -x halo
// (x = 0..2, bytes 0..23) and the -x face (x = 3..5, bytes 24..47) to the +x
// halo (x = 515..517, bytes 4120..4143), for the 512 x 512 interior rows.
// One lane per row; every variant moves or reads the same rows:
//   paired       both faces in one lane: 3 + 3 8-B loads, then 3 + 3 stores
//                (the packer's paired copy, copy_batch_kernel<8>)
//   single       one face per lane (two items, as without pairing)
//   full_sector  paired, but every destination 32-B sector written whole
//                (the bytes around the halo bytes loaded and stored back:
//                NOT allowed for the packer -- they are the application's --
//                so this is what the partly written sectors cost)
//   reads        the paired loads only
//   *_nt / *_sc1 / *_sys  the same with nontemporal loads, agent-scope
//                (global_load sc1: L1 bypassed) or system-scope (sc0 sc1)
//                loads: does a load's cache policy change how much of each
//                isolated row's 128-B line is fetched from memory?
//   reads8       one 8-B load per face row (how much of the time is lines,
//                how much bytes)
// usage: xface [REPS] -> one JSON line per variant (µs per exchange of the 8
// quantities' x faces, algorithmic GB/s = 2 x payload / time)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                      \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) {                                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));              \
      std::exit(3);                                                                                \
    }                                                                                              \
  } while (0)

constexpr int kL = 512, kR = 3, kQ = 8;
constexpr int64_t kPitch = 4608, kYs = kL + 2 * kR, kPlane = kPitch * kYs;
constexpr int64_t kBuf = kPlane * (kL + 2 * kR);
constexpr uint32_t kRows = uint32_t(kL) * kL; // per face

struct Bufs {
  char *b[kQ];
};

// byte offset of interior row r (z = r / 512, y = r % 512) in a buffer
__device__ __forceinline__ int64_t row_off(uint32_t r) {
  return (int64_t(r / kL) + kR) * kPlane + (int64_t(r % kL) + kR) * kPitch;
}

// load policy: 0 plain, 1 nontemporal, 2 agent scope (sc1), 3 system scope (sc0 sc1)
template <int POL> __device__ __forceinline__ uint64_t ldp(const uint64_t *p) {
  if constexpr (POL == 1) return __builtin_nontemporal_load(p);
  if constexpr (POL == 2) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if constexpr (POL == 3) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return *p;
}

template <int MODE, int POL = 0> // MODE 0 paired, 2 full_sector, 3 reads, 4 reads8
__global__ __launch_bounds__(256) void xface_paired(Bufs bufs, uint64_t *sink) {
  const uint32_t q = blockIdx.y;
  const uint32_t r = blockIdx.x * 256u + threadIdx.x;
  if (r >= kRows) return;
  char *row = bufs.b[q] + row_off(r);
  const uint64_t *s1 = reinterpret_cast<const uint64_t *>(row + 4096); // +x face
  const uint64_t *s2 = reinterpret_cast<const uint64_t *>(row + 24);   // -x face
  if constexpr (MODE == 4) {
    sink[blockIdx.y * gridDim.x * 256u + r] = ldp<POL>(s1) ^ ldp<POL>(s2);
    return;
  }
  uint64_t a0 = ldp<POL>(s1), a1 = ldp<POL>(s1 + 1), a2 = ldp<POL>(s1 + 2);
  uint64_t b0 = ldp<POL>(s2), b1 = ldp<POL>(s2 + 1), b2 = ldp<POL>(s2 + 2);
  if constexpr (MODE == 3) {
    sink[blockIdx.y * gridDim.x * 256u + r] = a0 ^ a1 ^ a2 ^ b0 ^ b1 ^ b2;
    return;
  }
  uint64_t *d1 = reinterpret_cast<uint64_t *>(row);        // -x halo, bytes 0..23
  uint64_t *d2 = reinterpret_cast<uint64_t *>(row + 4120); // +x halo, bytes 4120..4143
  if constexpr (MODE == 0) {
    d1[0] = a0, d1[1] = a1, d1[2] = a2;
    d2[0] = b0, d2[1] = b1, d2[2] = b2;
  } else { // whole sectors: [0, 32) = halo + x = 3 (b0); [4096, 4128) + [4128, 4160)
    uint64_t *sa = reinterpret_cast<uint64_t *>(row + 4096);
    const uint64_t p0 = sa[6], p1 = sa[7]; // bytes 4144..4159 (padding)
    d1[0] = a0, d1[1] = a1, d1[2] = a2, d1[3] = b0;
    sa[0] = a0, sa[1] = a1, sa[2] = a2, sa[3] = b0, sa[4] = b1, sa[5] = b2, sa[6] = p0, sa[7] = p1;
  }
}

__global__ __launch_bounds__(256) void xface_single(Bufs bufs, int face) {
  const uint32_t q = blockIdx.y;
  const uint32_t r = blockIdx.x * 256u + threadIdx.x;
  if (r >= kRows) return;
  char *row = bufs.b[q] + row_off(r);
  const uint64_t *s = reinterpret_cast<const uint64_t *>(row + (face ? 24 : 4096));
  uint64_t *d = reinterpret_cast<uint64_t *>(row + (face ? 4120 : 0));
  const uint64_t v0 = s[0], v1 = s[1], v2 = s[2];
  d[0] = v0, d[1] = v1, d[2] = v2;
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 20;
  Bufs bufs;
  for (int q = 0; q < kQ; ++q) {
    CK(hipMalloc(&bufs.b[q], size_t(kBuf)));
    CK(hipMemset(bufs.b[q], q + 1, size_t(kBuf)));
  }
  uint64_t *sink;
  CK(hipMalloc(&sink, size_t(kQ) * kRows * 8));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const dim3 grid((kRows + 255) / 256, kQ);
  const double payload = 2.0 * kQ * kRows * 24; // both faces of every quantity
  const char *names[] = {"paired",    "single",   "full_sector", "reads",     "paired_nt", "reads_nt",
                         "paired_sc1", "reads_sc1", "paired_sys",  "reads_sys", "reads8",    "reads8_nt"};
  constexpr int kVariants = 12;
  for (int v = 0; v < kVariants; ++v) {
    auto run = [&] {
      switch (v) {
      case 0: hipLaunchKernelGGL(xface_paired<0>, grid, dim3(256), 0, s, bufs, sink); break;
      case 1:
        hipLaunchKernelGGL(xface_single, grid, dim3(256), 0, s, bufs, 0);
        hipLaunchKernelGGL(xface_single, grid, dim3(256), 0, s, bufs, 1);
        break;
      case 2: hipLaunchKernelGGL(xface_paired<2>, grid, dim3(256), 0, s, bufs, sink); break;
      case 3: hipLaunchKernelGGL(xface_paired<3>, grid, dim3(256), 0, s, bufs, sink); break;
      case 4: hipLaunchKernelGGL((xface_paired<0, 1>), grid, dim3(256), 0, s, bufs, sink); break;
      case 5: hipLaunchKernelGGL((xface_paired<3, 1>), grid, dim3(256), 0, s, bufs, sink); break;
      case 6: hipLaunchKernelGGL((xface_paired<0, 2>), grid, dim3(256), 0, s, bufs, sink); break;
      case 7: hipLaunchKernelGGL((xface_paired<3, 2>), grid, dim3(256), 0, s, bufs, sink); break;
      case 8: hipLaunchKernelGGL((xface_paired<0, 3>), grid, dim3(256), 0, s, bufs, sink); break;
      case 9: hipLaunchKernelGGL((xface_paired<3, 3>), grid, dim3(256), 0, s, bufs, sink); break;
      case 10: hipLaunchKernelGGL((xface_paired<4, 0>), grid, dim3(256), 0, s, bufs, sink); break;
      default: hipLaunchKernelGGL((xface_paired<4, 1>), grid, dim3(256), 0, s, bufs, sink); break;
      }
    };
    run();
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < reps; ++i) run();
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = double(ms) * 1e3 / reps;
    std::printf("{\"bench\": \"xface\", \"variant\": \"%s\", \"rows\": %u, \"quants\": %d, \"payload\": %.0f, "
                "\"us\": %.1f, \"alg_GBps\": %.1f}\n",
                names[v], kRows * 2, kQ, payload, us,
                (v == 3 || v == 5 || v == 7 || v == 9 ? 1.0 : v >= 10 ? 1.0 / 3 : 2.0) * payload / (us * 1e-6) / 1e9);
    std::fflush(stdout);
  }
  return 0;
}
