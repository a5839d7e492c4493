// tools/calib.hip -- memory-system calibration on MI355X (gfx950) for the
// access patterns the packers produce, so that touched-byte arguments rest on
// measurement: for each pattern the kernel moves a KNOWN
// number of bytes; the program prints time and GB/s, and rocprofv3 --pmc
// passes over the same binary give the memory-side counters per kernel
// (tools/calib_summary.py divides them by the known byte counts).
//
// Patterns (buffers of >= 1 GiB, past the 256 MiB Infinity Cache):
//   rd_lines<P>   read the first B bytes of every 128-B line, 16 B per lane
//                 (B = 128: a full streaming read; B = 64: the 64 B : 128 pack)
//   rd_rows<T>    read one T-word of every S bytes (24-B rows at 4608: halo x
//                 faces use 8-B words; 8 : 16, 2 : 4, 1 : 8)
//   wr_lines<P>   write the first B bytes of every 128-B line
//   wr_rows<T>    write one T-word of every S bytes (the narrow scatters)
// P = load / store flavour: 0 plain, 1 nontemporal, 2 sc0, 3 sc1, 4 sc0 sc1
// (buffer instructions with that cache policy), so that a flavour which
// fetches less than a whole line would show up.
//
// usage: calib [REPS] [--only NAME]   -> one JSON line per pattern
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#define CK(x)                                                                                      \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) {                                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));              \
      std::exit(3);                                                                                \
    }                                                                                              \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, 0x7fffffff, 0x00020000);
}

// one 16-byte load of flavour P at base + off (off < 2 GiB for buffer forms)
template <int P> __device__ __forceinline__ u32x4 ld16(const char *base, uint32_t off) {
  if constexpr (P == 0) return *reinterpret_cast<const u32x4 *>(base + off);
  if constexpr (P == 1) return __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(base + off));
  constexpr int pol = P == 2 ? 1 : P == 3 ? 16 : 17;
  return __builtin_amdgcn_raw_buffer_load_b128(rsrc(base), int(off), 0, pol);
}
template <int P> __device__ __forceinline__ void st16(char *base, uint32_t off, u32x4 v) {
  if constexpr (P == 0) *reinterpret_cast<u32x4 *>(base + off) = v;
  else if constexpr (P == 1) __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(base + off));
  else {
    constexpr int pol = P == 2 ? 1 : P == 3 ? 16 : 17;
    __builtin_amdgcn_raw_buffer_store_b128(v, rsrc(base), int(off), 0, pol);
  }
}

// first `bytes` (multiple of 16) of each 128-B line of [base, base + lines*128);
// one 16-B word per lane; the XOR of what was read goes to sink[thread]
template <int P>
__global__ __launch_bounds__(256) void rd_lines(const char *base, uint32_t lines, uint32_t wpl, u32x4 *sink) {
  const uint32_t nwords = lines * wpl; // < 2^32; wpl a power of two
  const uint32_t lg = __builtin_ctz(wpl);
  u32x4 acc = {0, 0, 0, 0};
  for (uint32_t k = blockIdx.x * 256u + threadIdx.x; k < nwords; k += gridDim.x * 256u) {
    const uint32_t line = k >> lg, w = k & (wpl - 1);
    const uint64_t off = uint64_t(line) * 128 + w * 16;
    if constexpr (P >= 2) // buffer forms: one wave-uniform base, 32-bit offsets (< 2 GiB)
      acc ^= ld16<P>(base, uint32_t(off));
    else
      acc ^= ld16<P>(base + off, 0);
  }
  sink[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int P>
__global__ __launch_bounds__(256) void wr_lines(char *base, uint32_t lines, uint32_t wpl) {
  const uint32_t nwords = lines * wpl; // < 2^32; wpl a power of two
  const uint32_t lg = __builtin_ctz(wpl);
  for (uint32_t k = blockIdx.x * 256u + threadIdx.x; k < nwords; k += gridDim.x * 256u) {
    const uint32_t line = k >> lg, w = k & (wpl - 1);
    const uint64_t off = uint64_t(line) * 128 + w * 16;
    const u32x4 v = {k, ~k, 0x5a5a5a5au, line};
    if constexpr (P >= 2)
      st16<P>(base, uint32_t(off), v);
    else
      st16<P>(base + off, 0, v);
  }
}

// one T of every `stride` bytes, `rows` rows
template <typename T>
__global__ __launch_bounds__(256) void rd_rows(const char *base, uint64_t rows, uint32_t stride, T *sink) {
  T acc{};
  for (uint64_t r = blockIdx.x * 256ull + threadIdx.x; r < rows; r += uint64_t(gridDim.x) * 256)
    acc ^= *reinterpret_cast<const T *>(base + r * stride);
  sink[blockIdx.x * 256 + threadIdx.x] = acc;
}
template <typename T>
__global__ __launch_bounds__(256) void wr_rows(char *base, uint64_t rows, uint32_t stride) {
  for (uint64_t r = blockIdx.x * 256ull + threadIdx.x; r < rows; r += uint64_t(gridDim.x) * 256)
    *reinterpret_cast<T *>(base + r * stride) = T(r * 0x9E3779B97F4A7C15ull);
}

// The unpack / pack pattern itself without a packer's index math: chunk k
// (16 B) of a contiguous side <-> row k >> lg (2^lg chunks of 16 B a row) at
// `stride` on the strided side, nontemporal both sides. U chunks per lane (a
// workgroup owns 256 * U consecutive chunks, chunk u * 256 + lane of it, so
// every instruction of a wave stays coalesced); XR: the XCD-range tile order of
// pack_kernels.hip (XCD slot b % 8 walks one contiguous eighth of the tiles).
// Separates what the strided side's DRAM pattern costs (VERDICT r02 next 4:
// the whole-sector gapped unpacks) from what the kernel adds.
__device__ __forceinline__ uint32_t xr_tile(uint32_t b, uint32_t n) {
  const uint32_t x = b & 7, q = n >> 3, r = n & 7;
  return x * q + (x < r ? x : r) + (b >> 3);
}
template <bool SCATTER, int U, bool XR>
__global__ __launch_bounds__(256) void sect_copy(u32x4 *lin, char *strided, uint32_t lg, uint32_t stride) {
  const uint32_t tile = XR ? xr_tile(blockIdx.x, gridDim.x) : blockIdx.x;
  const uint32_t mask = (1u << lg) - 1;
  u32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t k = tile * (256u * U) + u * 256u + threadIdx.x;
    u32x4 *sp = reinterpret_cast<u32x4 *>(strided + uint64_t(k >> lg) * stride + (k & mask) * 16u);
    v[u] = SCATTER ? __builtin_nontemporal_load(lin + k) : __builtin_nontemporal_load(sp);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t k = tile * (256u * U) + u * 256u + threadIdx.x;
    u32x4 *sp = reinterpret_cast<u32x4 *>(strided + uint64_t(k >> lg) * stride + (k & mask) * 16u);
    if (SCATTER)
      __builtin_nontemporal_store(v[u], sp);
    else
      __builtin_nontemporal_store(v[u], lin + k);
  }
}

struct Case {
  std::string name;
  double algBytes;   // bytes the kernel reads or writes
  double lineBytes;  // 128-B lines it touches x 128
  std::function<void(hipStream_t)> run;
};

int main(int argc, char **argv) {
  int reps = 10;
  std::string only;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--only") && i + 1 < argc)
      only = argv[++i];
    else
      reps = std::atoi(argv[i]);
  }
  const size_t bufBytes = size_t(4) << 30; // 4 GiB: 16x the Infinity Cache
  char *buf = nullptr;
  CK(hipMalloc(&buf, bufBytes));
  CK(hipMemset(buf, 0x11, bufBytes));
  const int grid = 256 * 8 * 8; // 2048 CU-slots x 8: grid-stride
  u32x4 *sink = nullptr;
  CK(hipMalloc(&sink, size_t(grid) * 256 * sizeof(u32x4)));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  std::vector<Case> cases;
  auto add_lines = [&](int P, bool rd, uint32_t bytes) {
    const uint32_t wpl = bytes / 16;
    // buffer-instruction flavours address < 2 GiB from one base
    const uint32_t lines = uint32_t((P >= 2 ? (size_t(2) << 30) - 128 : bufBytes) / 128);
    Case c;
    c.name = std::string(rd ? "rd_lines" : "wr_lines") + "_B" + std::to_string(bytes) + "_P" + std::to_string(P);
    c.algBytes = double(lines) * bytes;
    c.lineBytes = double(lines) * 128;
    c.run = [=](hipStream_t st) {
      switch (P * 2 + (rd ? 1 : 0)) {
      case 1: hipLaunchKernelGGL(rd_lines<0>, dim3(grid), dim3(256), 0, st, buf, lines, wpl, sink); break;
      case 3: hipLaunchKernelGGL(rd_lines<1>, dim3(grid), dim3(256), 0, st, buf, lines, wpl, sink); break;
      case 5: hipLaunchKernelGGL(rd_lines<2>, dim3(grid), dim3(256), 0, st, buf, lines, wpl, sink); break;
      case 7: hipLaunchKernelGGL(rd_lines<3>, dim3(grid), dim3(256), 0, st, buf, lines, wpl, sink); break;
      case 9: hipLaunchKernelGGL(rd_lines<4>, dim3(grid), dim3(256), 0, st, buf, lines, wpl, sink); break;
      case 0: hipLaunchKernelGGL(wr_lines<0>, dim3(grid), dim3(256), 0, st, buf, lines, wpl); break;
      case 2: hipLaunchKernelGGL(wr_lines<1>, dim3(grid), dim3(256), 0, st, buf, lines, wpl); break;
      case 4: hipLaunchKernelGGL(wr_lines<2>, dim3(grid), dim3(256), 0, st, buf, lines, wpl); break;
      case 6: hipLaunchKernelGGL(wr_lines<3>, dim3(grid), dim3(256), 0, st, buf, lines, wpl); break;
      case 8: hipLaunchKernelGGL(wr_lines<4>, dim3(grid), dim3(256), 0, st, buf, lines, wpl); break;
      }
    };
    cases.push_back(c);
  };
  for (int P = 0; P <= 4; ++P)
    for (uint32_t b : {128u, 64u, 32u, 16u}) add_lines(P, true, b);
  for (int P = 0; P <= 1; ++P)
    for (uint32_t b : {128u, 64u, 32u, 16u}) add_lines(P, false, b);
  auto add_rows = [&](int T, uint32_t stride, bool rd) {
    const uint64_t rows = bufBytes / stride;
    Case c;
    c.name = std::string(rd ? "rd_rows" : "wr_rows") + "_T" + std::to_string(T) + "_S" + std::to_string(stride);
    c.algBytes = double(rows) * T;
    const double perLine = stride >= 128 ? 1.0 : 128.0 / stride; // rows per line
    c.lineBytes = stride >= 128 ? double(rows) * 128 : double(bufBytes);
    (void)perLine;
    c.run = [=](hipStream_t st) {
      if (rd) {
        if (T == 1) hipLaunchKernelGGL(rd_rows<uint8_t>, dim3(grid), dim3(256), 0, st, buf, rows, stride, reinterpret_cast<uint8_t *>(sink));
        if (T == 2) hipLaunchKernelGGL(rd_rows<uint16_t>, dim3(grid), dim3(256), 0, st, buf, rows, stride, reinterpret_cast<uint16_t *>(sink));
        if (T == 4) hipLaunchKernelGGL(rd_rows<uint32_t>, dim3(grid), dim3(256), 0, st, buf, rows, stride, reinterpret_cast<uint32_t *>(sink));
        if (T == 8) hipLaunchKernelGGL(rd_rows<uint64_t>, dim3(grid), dim3(256), 0, st, buf, rows, stride, reinterpret_cast<uint64_t *>(sink));
      } else {
        if (T == 1) hipLaunchKernelGGL(wr_rows<uint8_t>, dim3(grid), dim3(256), 0, st, buf, rows, stride);
        if (T == 2) hipLaunchKernelGGL(wr_rows<uint16_t>, dim3(grid), dim3(256), 0, st, buf, rows, stride);
        if (T == 4) hipLaunchKernelGGL(wr_rows<uint32_t>, dim3(grid), dim3(256), 0, st, buf, rows, stride);
        if (T == 8) hipLaunchKernelGGL(wr_rows<uint64_t>, dim3(grid), dim3(256), 0, st, buf, rows, stride);
      }
    };
    cases.push_back(c);
  };
  for (bool rd : {true, false}) {
    add_rows(8, 16, rd);   // 8 B : 16 (pack / unpack 8 : 16)
    add_rows(8, 4608, rd); // a 24-B halo row's words at pitch 4608 (one word of each row)
    add_rows(2, 4, rd);    // 2 B : 4
    add_rows(1, 8, rd);    // 1 B : 8
    add_rows(8, 128, rd);  // one 8-B word per line
    add_rows(8, 64, rd);   // one 8-B word per 64-B sector
    add_rows(8, 32, rd);   // one per 32-B sector
  }
  // sect_copy: 512 MiB of payload, rows of B bytes every S bytes (strided side
  // up to 32 GiB, allocated per case); alg bytes = payload x 2, "line" bytes =
  // contiguous side + the strided side's touched 64-B sectors
  char *lin = nullptr, *big = nullptr;
  size_t bigBytes = 0;
  auto add_sect = [&](bool scatter, uint32_t B, uint32_t S, int U, bool xr) {
    const uint64_t payload = uint64_t(512) << 20;
    const uint32_t lg = uint32_t(__builtin_ctz(B / 16));
    const uint64_t rows = payload / B;
    const uint32_t blocks = uint32_t(payload / 16 / (256u * U));
    Case c;
    c.name = std::string(scatter ? "sc" : "ga") + "_B" + std::to_string(B) + "_S" + std::to_string(S) + "_U" +
             std::to_string(U) + (xr ? "_xr" : "");
    c.algBytes = double(payload) * 2;
    c.lineBytes = double(payload) * 2;
    c.run = [=, &lin, &big, &bigBytes](hipStream_t st) {
      const size_t need = size_t(rows) * S;
      if (!lin) CK(hipMalloc(&lin, payload));
      if (bigBytes < need) {
        if (big) CK(hipFree(big));
        CK(hipMalloc(&big, need));
        CK(hipMemset(big, 0x22, need));
        bigBytes = need;
      }
      u32x4 *l = reinterpret_cast<u32x4 *>(lin);
#define SECT(SC, UU, XX) hipLaunchKernelGGL((sect_copy<SC, UU, XX>), dim3(blocks), dim3(256), 0, st, l, big, lg, S)
      if (scatter) {
        if (U == 1) { if (xr) SECT(true, 1, true); else SECT(true, 1, false); }
        else { if (xr) SECT(true, 4, true); else SECT(true, 4, false); }
      } else {
        if (U == 1) { if (xr) SECT(false, 1, true); else SECT(false, 1, false); }
        else { if (xr) SECT(false, 4, true); else SECT(false, 4, false); }
      }
#undef SECT
    };
    cases.push_back(c);
  };
  // (U = 4 measured slower than U = 1 on every shape, round 3: kept for A/B)
  for (auto bs : {std::pair<uint32_t, uint32_t>{64, 128}, {64, 256}, {64, 512}, {64, 1024}, {64, 4096}, {128, 256},
                  {128, 512}, {256, 512}, {256, 1024}, {256, 4096}, {512, 1024}, {512, 2048}, {512, 4096},
                  {1024, 2048}, {1024, 4096}, {1024, 8192}, {2048, 4096}, {2048, 8192}, {4096, 8192},
                  {4096, 16384}})
    for (bool xr : {false, true}) add_sect(true, bs.first, bs.second, 1, xr);
  add_sect(true, 64, 512, 4, false);
  for (uint32_t S : {512u, 4096u}) add_sect(false, 64, S, 1, false);
  add_sect(false, 512, 1024, 1, false);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (const Case &c : cases) {
    if (!only.empty() && c.name.find(only) == std::string::npos) continue;
    c.run(s); // warm
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < reps; ++r) c.run(s);
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double t = ms / reps * 1e-3;
    std::printf("{\"case\": \"%s\", \"ms\": %.4f, \"alg_bytes\": %.0f, \"line_bytes\": %.0f, \"alg_GBps\": %.1f, "
                "\"line_GBps\": %.1f}\n",
                c.name.c_str(), t * 1e3, c.algBytes, c.lineBytes, c.algBytes / t / 1e9, c.lineBytes / t / 1e9);
    std::fflush(stdout);
  }
  CK(hipFree(buf));
  CK(hipFree(sink));
  if (lin) CK(hipFree(lin));
  if (big) CK(hipFree(big));
  return 0;
}
