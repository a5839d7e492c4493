// tempi_amd/csrc/hip/pack_kernels.hip -- gfx950 gather (pack) / scatter
// (unpack) kernels for canonical strided objects, behind the C ABI in
// include/tempi_hip.h (tempi_hip_pack / tempi_hip_unpack).
//
// Replaces the reference's pack_2d/unpack_2d/pack_3d/unpack_3d<W> kernels
// (/root/reference/include/pack_kernels.cuh:19-120, :350-433), their launch
// planning (/root/reference/include/pack_config.hpp:33-37,
// /root/reference/src/internal/packer_3d.cu:19-78) and Packer1D's memcpy
// (/root/reference/src/internal/packer_1d.cu:16-49). Semantics are the MPI
// type-map order the oracle (oracle/typemap.c) restates.
//
// Design (MI355X-first, not a translation):
//  * OUTPUT-LINEAR: the packed side is one contiguous stream, so every lane
//    owns one 16-byte ALIGNED chunk of it and moves it with a single
//    global_{load,store}_dwordx4. Only the first and last chunk of a launch
//    can be partial; they take a per-word path.
//  * W-byte words on the strided side: W = the largest power of two <= 16
//    dividing both base addresses, the block length and every stride (the
//    reference picks W from block length and offset only: SURVEY F4). A chunk
//    is 16/W words, gathered from (or scattered to) up to 16/W rows and
//    transposed in registers into one wide store (or out of one wide load):
//    narrow blocks still produce full-width coalesced packed traffic.
//  * Index math is 32-bit with invariant-divisor magic numbers (Granlund-
//    Montgomery) for words-per-row and every dimension count; offsets are
//    64-bit (extents of several GiB are fine; the reference's are 32-bit, F6).
//    One decode per chunk, then an odometer step per row change.
//  * Grid: 128-thread workgroups (2 waves), one 16-byte chunk per lane for
//    16-byte words (a 1 GiB pack is 524288 workgroups: the dispatcher keeps
//    every CU full and no lane loops), two chunks per lane for 8-byte words;
//    grid-stride only beyond 2^20 workgroups. Packed-side accesses are nontemporal, and so are strided-side
//    ones when the word is 16 bytes: every byte is touched once. Measured on
//    MI355X (tools/kbench.cpp): +12% over plain loads/stores at 512-byte rows.
//  * Launches larger than 2^31 words are split on the host.
#include <hip/hip_runtime.h>

#include "tempi_hip.h"
#include "ticket.hpp"

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include <unistd.h>

namespace {

struct Magic {
  uint32_t mul;
  uint32_t s1;
  uint32_t s2;
};

// magic for n / d, exact for every 32-bit n (Hacker's Delight 10-8)
Magic make_magic(uint32_t d) {
  uint32_t l = 0;
  while ((uint64_t(1) << l) < d) ++l;
  const uint64_t m = ((((uint64_t(1) << l) - d) << 32) / d) + 1;
  Magic r;
  r.mul = uint32_t(m);
  r.s1 = l ? 1 : 0;
  r.s2 = l ? l - 1 : 0;
  return r;
}

__device__ __forceinline__ uint32_t mdiv(uint32_t n, const Magic &m) {
  const uint32_t t = __umulhi(n, m.mul);
  return (t + ((n - t) >> m.s1)) >> m.s2;
}

template <int W> struct Word;
template <> struct Word<1> { typedef uint8_t T; };
template <> struct Word<2> { typedef uint16_t T; };
template <> struct Word<4> { typedef uint32_t T; };
template <> struct Word<8> { typedef uint2 T; };
template <> struct Word<16> { typedef uint4 T; };

// tuning knobs (defaults are the measured best; tools/kbench.cpp sweeps them)
#ifndef TEMPI_UNROLL_16
#define TEMPI_UNROLL_16 1
#endif
#ifndef TEMPI_UNROLL_WIDE
#define TEMPI_UNROLL_WIDE 2
#endif
#ifndef TEMPI_UNROLL_NARROW
#define TEMPI_UNROLL_NARROW 1
#endif
#ifndef TEMPI_MAX_BLOCKS
#define TEMPI_MAX_BLOCKS (1 << 20)
#endif
#ifndef TEMPI_BLOCK
// 128-lane workgroups for the packers: against 256 on one box
// (tools/gpu_block_ab.sh, profiles/r01/block_ab_s9.jsonl) the 512-byte-row
// headline packs 6 223-6 288 vs 6 022-6 068 GB/s and unpacks 6 235-6 309 vs
// 6 075-6 092, 64-byte rows unpack 5 712 vs 4 685-4 887; 512 and 1024 are no
// better than 256. The copy kernels keep 256 (kCopyBlock)
#define TEMPI_BLOCK 128
#endif
#ifndef TEMPI_NT
// 0: plain; 1: nontemporal packed side; 2: nontemporal both sides;
// 3: packed side always, strided side when its words are 16 bytes (a
//    narrower word's line is re-read by the next word of the same lane)
#define TEMPI_NT 3
#endif
constexpr bool kNtPacked = TEMPI_NT >= 1;
// word widths (bit W/1: 1, 2, 4, 8) that use the interleaved, LDS-transposed
// kernels (pack_il_kernel / unpack_il_kernel); measured on MI355X
// (tools/kbench.cpp, profiles/r01/kbench_il_s2.jsonl): unpack gains for every
// width (1 B : 2 B x2.4, 24-byte halo rows +20%), pack only for 1-byte words
#ifndef TEMPI_PACK_IL_WIDTHS
#define TEMPI_PACK_IL_WIDTHS 1
#endif
#ifndef TEMPI_UNPACK_IL_WIDTHS
#define TEMPI_UNPACK_IL_WIDTHS (1 | 2 | 4 | 8)
#endif
constexpr bool il_width(bool pack, int w) {
  return w <= 8 && ((pack ? TEMPI_PACK_IL_WIDTHS : TEMPI_UNPACK_IL_WIDTHS) & w) != 0;
}
template <int W> struct NtStrided { static constexpr bool value = TEMPI_NT == 2 || (TEMPI_NT == 3 && W == 16); };
// the strided-side stores of the chunk-per-lane scatter (unpack_body):
// -1 as NtStrided, 0 plain, 1 nontemporal (A/B knob, tools/gpu_gap_ab.sh)
#ifndef TEMPI_NT_SCATTER
#define TEMPI_NT_SCATTER -1
#endif
template <int W> struct NtScatter {
  static constexpr bool value = TEMPI_NT_SCATTER < 0 ? NtStrided<W>::value : TEMPI_NT_SCATTER == 1;
};

// chunks each lane keeps in flight per grid-stride step
template <int W> struct Unroll {
  static constexpr int U = W == 16 ? TEMPI_UNROLL_16 : W == 8 ? TEMPI_UNROLL_WIDE : (W == 4 ? 2 : TEMPI_UNROLL_NARROW);
};

#ifndef TEMPI_XCD_MAP
#define TEMPI_XCD_MAP 1
#endif
// Workgroup -> tile for scatters that write sectors in part. The dispatcher
// deals workgroups round-robin over the 8 XCDs, so blocks b and b + 8 share
// an XCD and its L2 (MI355X_MICROARCH.md, "Workgroup dispatch, XCD
// placement"). With kXcdRange in the launch's flags, XCD slot b % 8 owns one
// contiguous eighth of the tiles and walks it in order, so neighbouring tiles
// meet in one L2: a strided-side line two tiles both write in part (a row or
// an unaligned plane crossing the tile edge) is merged there instead of
// reaching DRAM as two masked writes from two XCDs, each a read-modify-write
// (1 B : 2 B 3D unpack +10 %, 128 B : 144 +26 %, 24-B rows +8 %). Streams of
// whole lines keep the dealt order: eight streams an eighth of the object
// apart cost the headline unpack 6 % (profiles/r02/xcd_group_ab_s12.jsonl),
// as do shorter runs per XCD (16 tiles: -14 %). Placement is only a speed
// hint: the map is a bijection of [0, n) whatever the hardware does.
constexpr uint32_t kXcdRange = 1u << 31; // internal flag bit (never a TEMPI_HIP_ITEM_*)
__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t n, uint32_t flags) {
  if (!(flags & kXcdRange)) return b;
  const uint32_t x = b & 7, q = n >> 3, r = n & 7;
  return x * q + (x < r ? x : r) + (b >> 3);
}

// The end of a workgroup of a launch that stores its own completion ticket
// (ticket.hpp): every wave waits until its stores are acknowledged, then one
// lane per workgroup counts the workgroup, and the workgroup that completes
// the count stores the ticket for the host. A workgroup whose stores went
// through the L2 write-back (`fence`) first releases them at system scope (an
// L2 write-back of this XCD; the XCD L2s are not coherent with each other):
// the interposer takes a ticket only when the kernel writes device memory or
// TEMPI's coherent slabs, but a process with two HIP runtimes sees the other
// runtime's pinned host memory as device memory, and host-visible
// must hold for that too. A workgroup whose stores were all write-through
// (kWriteThrough: sc0 sc1, acknowledged once out of L2) needs no release.
// The waits are inline asm: ROCm 7.2 may drop its own wait after the release's
// write-back when it can prove the wave's counters empty, and the count would
// then overtake the write-back (MI355X_MICROARCH.md, "Compiler hazard").
// sg.flag == nullptr (uniform): nothing to do.
using tempi_ticket::Sig;
__device__ __forceinline__ void wg_signal(const Sig &sg, bool fence) {
  if (!sg.flag) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    if (fence) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    using namespace tempi_ticket;
    const uint32_t k = blockIdx.x % kShards;
    const uint32_t old = __hip_atomic_fetch_add(sg.counter + k * kCounterStride, 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_SYSTEM);
    if (old + 1u == sg.target[k]) { // the last workgroup of its shard
      const uint32_t top = __hip_atomic_fetch_add(sg.counter + kShards * kCounterStride, 1u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_SYSTEM);
      if (top + 1u == sg.top) __hip_atomic_store(sg.flag, sg.ticket, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

constexpr int kBlock = TEMPI_BLOCK;
// the interleaved tiles index whole 64-lane waves (tile + wave * 64, j * 64 + lane over kBlock entries)
static_assert(kBlock % 64 == 0 && kBlock >= 64 && kBlock <= 1024, "packer workgroups are whole 64-lane waves");

// TEMPI_LAUNCH_CHECK=1: every launch is followed by a
// stream synchronisation; a launch that faults is reported with the kernel,
// its grid and the descriptor(s) of the entry point that launched it, and the
// process aborts there -- instead of a later, unrelated call (another
// runtime's copy, say) reporting a sticky error. A diagnostic mode: it
// serialises every call.
bool launch_check() {
  static const bool on = [] {
    const char *e = std::getenv("TEMPI_LAUNCH_CHECK");
    return e && std::strtol(e, nullptr, 10) != 0;
  }();
  return on;
}
thread_local std::string gDesc; // what the current entry point launches (only kept under launch_check())
void check_launch(const char *kernel, const dim3 &grid, hipStream_t s) {
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e == hipSuccess) return;
  std::fprintf(stderr, "[TEMPI_LAUNCH_CHECK] %s, grid %u x %u: %s (%d) -- %s\n", kernel, grid.x, grid.y,
               hipGetErrorString(e), int(e), gDesc.c_str());
  std::fflush(stderr);
  std::abort();
}
std::string describe(const tempi_hip_desc &d, const void *a, const void *b) {
  std::string r = "{" + std::to_string(uintptr_t(a)) + " <- " + std::to_string(uintptr_t(b)) + ": block " +
                  std::to_string(d.block);
  for (int k = 0; k < d.ndims && k < TEMPI_HIP_MAX_DIMS; ++k)
    r += " (" + std::to_string(d.counts[k]) + " x " + std::to_string(d.strides[k]) + ")";
  return r + "}";
}
#define TEMPI_LAUNCH(K, G, B, SH, S, ...)                                                                          \
  do {                                                                                                             \
    hipLaunchKernelGGL(K, G, B, SH, S, __VA_ARGS__);                                                               \
    if (launch_check()) check_launch(#K, G, S);                                                                    \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// plain or nontemporal (streaming) access; HIP's uint2/uint4 are structs, so
// the builtins see their native vector form
template <typename T> struct NativeOf { typedef T type; };
template <> struct NativeOf<uint4> { typedef u32x4 type; };
template <> struct NativeOf<uint2> { typedef u32x2 type; };

template <typename T> __device__ __forceinline__ T ld(const T *p, bool nt) {
  if (nt) {
    typedef typename NativeOf<T>::type N;
    N v = __builtin_nontemporal_load(reinterpret_cast<const N *>(p));
    T r;
    __builtin_memcpy(&r, &v, sizeof r);
    return r;
  }
  return *p;
}
template <typename T> __device__ __forceinline__ void st(T *p, const T &v, bool nt) {
  if (nt) {
    typedef typename NativeOf<T>::type N;
    N n;
    __builtin_memcpy(&n, &v, sizeof n);
    __builtin_nontemporal_store(n, reinterpret_cast<N *>(p));
  } else {
    *p = v;
  }
}

template <int ND> struct KArgs {
  char *chunk0;   // 16-byte aligned address of packed chunk 0 (<= packed start)
  char *strided;  // first byte of the strided object
  uint32_t nwords;  // packed words
  uint32_t head;    // words between chunk0 and the first packed word
  uint32_t nchunks; // 16-byte chunks covering the packed range
  uint32_t wpr;     // words per block (row)
  Magic mwpr;
  // strided dimensions, INNERMOST FIRST
  uint32_t cnt[ND > 0 ? ND : 1];
  Magic mcnt[ND > 0 ? ND : 1];
  uint32_t flags;  // TEMPI_HIP_ITEM_* of the item (sits in what was padding)
  int64_t stride[ND > 0 ? ND : 1];
  int64_t wrap[ND > 0 ? ND : 1]; // cnt[k] * stride[k]
};

// Packed bytes that live in another process's memory (an IPC-mapped slab,
// possibly on another GPU: TEMPI_HIP_ITEM_REMOTE) are read with system-scope
// loads (sc0 sc1). The slab is reused for later messages, and a plain load
// could return a line this GPU's L2 kept from an earlier message in it. The
// buffer form keeps the loads counted by hipcc; its base is the first active
// lane's address (wave-uniform), which every call site keeps lowest.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t remote_rsrc(const void *p, uint32_t *off) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(uint32_t(a));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(uint32_t(a >> 32));
  const uint64_t base = (uint64_t(hi) << 32) | lo;
  *off = uint32_t(a - base);
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(base), 0, 0x7fffffff, 0x00020000);
}
constexpr int kSysScope = 1 | 16; // cache policy sc0 | sc1
template <typename T> __device__ __forceinline__ T ld_remote(const T *p) {
  uint32_t off;
  const __amdgpu_buffer_rsrc_t r = remote_rsrc(p, &off);
  T v;
  if constexpr (sizeof(T) == 16) {
    u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(r, int(off), 0, kSysScope);
    __builtin_memcpy(&v, &x, 16);
  } else if constexpr (sizeof(T) == 8) {
    u32x2 x = __builtin_amdgcn_raw_buffer_load_b64(r, int(off), 0, kSysScope);
    __builtin_memcpy(&v, &x, 8);
  } else if constexpr (sizeof(T) == 4) {
    uint32_t x = __builtin_amdgcn_raw_buffer_load_b32(r, int(off), 0, kSysScope);
    __builtin_memcpy(&v, &x, 4);
  } else if constexpr (sizeof(T) == 2) {
    uint16_t x = __builtin_amdgcn_raw_buffer_load_b16(r, int(off), 0, kSysScope);
    __builtin_memcpy(&v, &x, 2);
  } else {
    uint8_t x = __builtin_amdgcn_raw_buffer_load_b8(r, int(off), 0, kSysScope);
    __builtin_memcpy(&v, &x, 1);
  }
  return v;
}
// a load of packed bytes on the unpack side
template <typename T, int ND> __device__ __forceinline__ T ld_packed(const KArgs<ND> &a, const T *p, bool nt) {
  if (a.flags & TEMPI_HIP_ITEM_REMOTE) return ld_remote(p);
  return ld(p, nt);
}

// A gather whose completion ticket is folded into it (wg_signal) stores its
// 16-byte packed chunks write-through (sc0 sc1: the line leaves L2 as it is
// written, at the plain store's rate), so that only the workgroups holding the
// object's partial first / last chunk, stored word by word, release L2 at the
// end. The store's buffer base is the wave's first active lane, whose chunk is
// the lowest (chunks ascend with the lane). Internal flag bit, never a
// TEMPI_HIP_ITEM_*. The store path exists only in the WTC ("write-through
// compiled") instantiations of the kernels, which the host picks for folded
// launches alone: compiled into every kernel, it cost the large 3D narrow-row
// gathers a third of their rate (2 B : 18, 1 205 -> 810-832 GB/s; register
// pressure of the unused path, profiles/r04/kab_218_r4s1.jsonl).
constexpr uint32_t kWriteThrough = 1u << 30;
template <bool WTC> __device__ __forceinline__ void st_packed(uint32_t flags, uint4 *p, const uint4 &v) {
  if constexpr (WTC) {
    if (flags & kWriteThrough) {
      uint32_t off;
      const __amdgpu_buffer_rsrc_t r = remote_rsrc(p, &off);
      u32x4 x;
      __builtin_memcpy(&x, &v, 16);
      __builtin_amdgcn_raw_buffer_store_b128(x, r, int(off), 0, kSysScope);
      return;
    }
  }
  st(p, v, kNtPacked);
}

// the scatter's store of one strided-side word: write-through for 16-byte
// words of a folded launch (the host sets kWriteThrough only when every
// stride is >= 0 and the object spans < 2 GiB, so a wave's addresses ascend
// with the lane from its first active lane and fit the buffer offset)
template <int W, bool WTC>
__device__ __forceinline__ void st_scatter(uint32_t flags, typename Word<W>::T *p, const typename Word<W>::T &v) {
  if constexpr (W == 16 && WTC) {
    if (flags & kWriteThrough) {
      st_packed<true>(flags, p, v);
      return;
    }
  }
  st(p, v, NtScatter<W>::value);
}

// row index -> byte offset of the row, plus the odometer digits
template <int ND>
__device__ __forceinline__ int64_t row_offset(uint32_t row, const KArgs<ND> &a,
                                              uint32_t *dig) {
  int64_t off = 0;
#pragma unroll
  for (int k = 0; k < ND; ++k) {
    if (k == ND - 1) {
      dig[k] = row;
      off += int64_t(row) * a.stride[k];
    } else {
      const uint32_t q = mdiv(row, a.mcnt[k]);
      const uint32_t d = row - q * a.cnt[k];
      dig[k] = d;
      off += int64_t(d) * a.stride[k];
      row = q;
    }
  }
  return off;
}

template <int ND>
__device__ __forceinline__ void next_row(int64_t &off, uint32_t *dig,
                                         const KArgs<ND> &a) {
#pragma unroll
  for (int k = 0; k < ND; ++k) {
    off += a.stride[k];
    if (k == ND - 1 || ++dig[k] < a.cnt[k]) return;
    dig[k] = 0;
    off -= a.wrap[k];
  }
}

// byte offset (in the strided object) of packed word q
template <int W, int ND>
__device__ __forceinline__ int64_t word_offset(uint32_t q, const KArgs<ND> &a) {
  const uint32_t row = mdiv(q, a.mwpr);
  const uint32_t w = q - row * a.wpr;
  uint32_t dig[ND > 0 ? ND : 1];
  return row_offset<ND>(row, a, dig) + int64_t(w) * W;
}

// ND >= 2: true when rows [row, lastRow] all lie in one run of the innermost
// dimension (dig[0] is row's innermost digit), so that moving from one of
// them to the next is a single add of stride[0] -- no odometer carry. Only a
// chunk (or wave) straddling the end of a run needs the full odometer: the
// carry test and its wrap were what made narrow 3D rows slower than the same
// bytes in 2D (2 B : 18 pack 753 vs 1 091 GB/s).
template <int ND>
__device__ __forceinline__ bool one_run(uint32_t row, uint32_t lastRow, const uint32_t *dig, const KArgs<ND> &a) {
  return ND <= 1 || dig[0] + (lastRow - row) < a.cnt[0];
}

template <int W, bool PACK> struct ChunkT {
  static constexpr int CW = 16 / W;
  typedef typename Word<W>::T WT;
  union U {
    uint4 v;
    WT w[CW];
  };
};

// words of one partial chunk, one at a time (first / last chunk only)
template <int W, int ND, bool PACK>
__device__ void partial_chunk(uint32_t c, const KArgs<ND> &a) {
  typedef typename Word<W>::T WT;
  constexpr int CW = 16 / W;
  const int64_t q0 = int64_t(c) * CW - a.head;
  for (int j = 0; j < CW; ++j) {
    const int64_t q = q0 + j;
    if (q < 0 || q >= int64_t(a.nwords)) continue;
    WT *pk = reinterpret_cast<WT *>(a.chunk0 + size_t(c) * 16) + j;
    WT *sp = reinterpret_cast<WT *>(a.strided + word_offset<W, ND>(uint32_t(q), a));
    if (PACK)
      *pk = *sp;
    else
      *sp = ld_packed(a, pk, false);
  }
}

// workgroup `blk` of `nblk` working on one object (grid-stride over its
// chunks, U chunks per lane per step; U = 1 makes workgroup blk handle exactly
// chunks [blk * kBlock, (blk + 1) * kBlock) when nblk covers the object)
template <int W, int ND, bool WTC, int U = Unroll<W>::U>
__device__ __forceinline__ void pack_body(const KArgs<ND> &a, uint32_t blk, uint32_t nblk) {
  typedef typename Word<W>::T WT;
  constexpr int CW = 16 / W;
  typedef typename ChunkT<W, true>::U Buf;
  const uint32_t step = nblk * (kBlock * U);
  for (uint32_t base = blk * (kBlock * U); base < a.nchunks; base += step) {
    Buf buf[U];
    bool full[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t c = base + u * kBlock + threadIdx.x;
      const int64_t q0 = int64_t(c) * CW - a.head;
      full[u] = c < a.nchunks && q0 >= 0 && q0 + CW <= int64_t(a.nwords);
      if (full[u]) {
        uint32_t w;
        uint32_t dig[ND > 0 ? ND : 1];
        const uint32_t q = uint32_t(q0);
        const uint32_t row = mdiv(q, a.mwpr);
        w = q - row * a.wpr;
        int64_t off = row_offset<ND>(row, a, dig);
        bool run = CW == 1;
        if constexpr (ND >= 2 && CW > 1 && CW <= 8) run = one_run<ND>(row, mdiv(q + (CW - 1), a.mwpr), dig, a);
        else if constexpr (CW > 1 && CW <= 8) run = true;
        // (1-byte words keep one loop: two 16-load copies of it double the
        // registers of every kernel that inlines this body, for its rare
        // partial tiles; their hot paths are the interleaved / dense kernels)
        if (ND >= 1 && CW > 1 && run && a.wpr == 1) {
          // one word per row (block == W, uniform): every word is the next
          // row, one add apart -- no word-in-row bookkeeping at all
#pragma unroll
          for (int j = 0; j < CW; ++j) {
            buf[u].w[j] = ld(reinterpret_cast<const WT *>(a.strided + off), NtStrided<W>::value);
            if constexpr (ND >= 1) off += a.stride[0];
          }
        } else if (run) {
#pragma unroll
          for (int j = 0; j < CW; ++j) {
            buf[u].w[j] = ld(reinterpret_cast<const WT *>(a.strided + off + int64_t(w) * W), NtStrided<W>::value);
            if (j + 1 < CW && ++w == a.wpr) {
              w = 0;
              if constexpr (ND >= 1) off += a.stride[0];
            }
          }
        } else {
#pragma unroll
          for (int j = 0; j < CW; ++j) {
            buf[u].w[j] = ld(reinterpret_cast<const WT *>(a.strided + off + int64_t(w) * W), NtStrided<W>::value);
            if (j + 1 < CW && ++w == a.wpr) {
              w = 0;
              next_row<ND>(off, dig, a);
            }
          }
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t c = base + u * kBlock + threadIdx.x;
      if (full[u]) {
        st_packed<WTC>(a.flags, reinterpret_cast<uint4 *>(a.chunk0 + size_t(c) * 16), buf[u].v);
      } else if (c < a.nchunks) {
        partial_chunk<W, ND, true>(c, a);
      }
    }
  }
}

template <int W, int ND, bool WTC, int U = Unroll<W>::U>
__device__ __forceinline__ void unpack_body(const KArgs<ND> &a, uint32_t blk, uint32_t nblk) {
  typedef typename Word<W>::T WT;
  constexpr int CW = 16 / W;
  typedef typename ChunkT<W, false>::U Buf;
  const uint32_t step = nblk * (kBlock * U);
  for (uint32_t base = blk * (kBlock * U); base < a.nchunks; base += step) {
    Buf buf[U];
    bool full[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t c = base + u * kBlock + threadIdx.x;
      const int64_t q0 = int64_t(c) * CW - a.head;
      full[u] = c < a.nchunks && q0 >= 0 && q0 + CW <= int64_t(a.nwords);
      if (full[u]) buf[u].v = ld_packed(a, reinterpret_cast<const uint4 *>(a.chunk0 + size_t(c) * 16), kNtPacked);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t c = base + u * kBlock + threadIdx.x;
      if (full[u]) {
        const int64_t q0 = int64_t(c) * CW - a.head;
        uint32_t dig[ND > 0 ? ND : 1];
        const uint32_t q = uint32_t(q0);
        const uint32_t row = mdiv(q, a.mwpr);
        uint32_t w = q - row * a.wpr;
        int64_t off = row_offset<ND>(row, a, dig);
        // (1-byte words keep one loop: two 16-load copies of it double the
        // registers of every kernel that inlines this body, for its rare
        // partial tiles; their hot paths are the interleaved / dense kernels)
        if (CW == 1 || (CW <= 8 && one_run<ND>(row, mdiv(q + (CW - 1), a.mwpr), dig, a))) {
#pragma unroll
          for (int j = 0; j < CW; ++j) {
            st_scatter<W, WTC>(a.flags, reinterpret_cast<WT *>(a.strided + off + int64_t(w) * W), buf[u].w[j]);
            if (j + 1 < CW && ++w == a.wpr) {
              w = 0;
              if constexpr (ND >= 1) off += a.stride[0];
            }
          }
        } else {
#pragma unroll
          for (int j = 0; j < CW; ++j) {
            st_scatter<W, WTC>(a.flags, reinterpret_cast<WT *>(a.strided + off + int64_t(w) * W), buf[u].w[j]);
            if (j + 1 < CW && ++w == a.wpr) {
              w = 0;
              next_row<ND>(off, dig, a);
            }
          }
        }
      } else if (c < a.nchunks) {
        partial_chunk<W, ND, false>(c, a);
      }
    }
  }
}

// a workgroup of a write-through gather that still needs the release: the
// first and last tiles hold the object's partial chunks (folded launches never
// grid-stride: at most TEMPI_FOLD_MAX_BLOCKS_WT workgroups, one tile each)
__device__ __forceinline__ bool needs_release(uint32_t flags, uint32_t tile, uint32_t ntiles) {
  return !(flags & kWriteThrough) || tile == 0 || tile + 1 == ntiles;
}

template <int W, int ND, bool WTC>
__global__ __launch_bounds__(kBlock) void pack_kernel(const KArgs<ND> a, const Sig sg) {
  const uint32_t tile = xcd_tile(blockIdx.x, gridDim.x, a.flags);
  pack_body<W, ND, WTC>(a, tile, gridDim.x);
  wg_signal(sg, needs_release(a.flags, tile, gridDim.x));
}

template <int W, int ND, bool WTC>
__global__ __launch_bounds__(kBlock) void unpack_kernel(const KArgs<ND> a, const Sig sg) {
  const uint32_t tile = xcd_tile(blockIdx.x, gridDim.x, a.flags);
  unpack_body<W, ND, WTC>(a, tile, gridDim.x);
  wg_signal(sg, needs_release(a.flags, tile, gridDim.x));
}

// ------------------------------------------- wave-interleaved scatter (unpack)
//
// For 1- and 2-byte words the chunk-per-lane scatter has every store
// instruction of a wave touch 64 different rows, 16/W rows apart, so each
// cache line of the strided side is written by 16/W separate instructions.
// Here the workgroup's kBlock x 16 bytes of packed input is staged in LDS (one 16-byte
// load per lane), and store instruction j of a wave writes the 64 CONSECUTIVE
// words j*64 .. j*64+63 of the wave's 1 KiB: neighbouring rows, so one
// instruction covers a line and every line is written once. Tiles holding the
// object's partial first / last chunk take the chunk-per-lane path.
template <int W, int ND>
__device__ __forceinline__ void unpack_il_tile(const KArgs<ND> &a, uint32_t tileIdx, uint32_t ntiles) {
  typedef typename Word<W>::T WT;
  constexpr int CW = 16 / W;
  __shared__ uint4 tile[kBlock];
  const uint32_t c0 = tileIdx * kBlock;
  const uint32_t c1 = min(c0 + uint32_t(kBlock), a.nchunks);
  const bool clean = c1 - c0 == uint32_t(kBlock) && int64_t(c0) * CW - a.head >= 0 &&
                     int64_t(c1) * CW - a.head <= int64_t(a.nwords);
  if (!clean) { // uniform: this tile's chunks, one per lane
    unpack_body<W, ND, false, 1>(a, tileIdx, ntiles);
    return;
  }
  tile[threadIdx.x] = ld_packed(a, reinterpret_cast<const uint4 *>(a.chunk0 + size_t(c0 + threadIdx.x) * 16), kNtPacked);
  __syncthreads();
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const WT *src = reinterpret_cast<const WT *>(tile + wave * 64);
  const uint32_t qw = uint32_t(int64_t(c0 + wave * 64) * CW - a.head); // first word of this wave
  if constexpr (ND >= 2 && ND <= 3) { // the wave's rows in one innermost run (uniform): one decode for the wave
    uint32_t dig0[ND];
    const uint32_t r0 = mdiv(qw, a.mwpr);
    const int64_t base0 = row_offset<ND>(r0, a, dig0);
    if (one_run<ND>(r0, mdiv(qw + uint32_t(64 * CW - 1), a.mwpr), dig0, a)) {
#pragma unroll
      for (int j = 0; j < CW; ++j) {
        const uint32_t t = uint32_t(j) * 64 + lane;
        const uint32_t row = mdiv(qw + t, a.mwpr);
        const uint32_t w = qw + t - row * a.wpr;
        st(reinterpret_cast<WT *>(a.strided + base0 + int64_t(row - r0) * a.stride[0] + int64_t(w) * W), src[t],
           false);
      }
      return;
    }
  }
#pragma unroll
  for (int j = 0; j < CW; ++j) {
    const uint32_t t = uint32_t(j) * 64 + lane;
    const uint32_t q = qw + t;
    const uint32_t row = mdiv(q, a.mwpr);
    const uint32_t w = q - row * a.wpr;
    uint32_t dig[ND > 0 ? ND : 1];
    const int64_t off = row_offset<ND>(row, a, dig) + int64_t(w) * W;
    st(reinterpret_cast<WT *>(a.strided + off), src[t], false);
  }
}

// the gather twin of unpack_il_kernel: load instruction j of a wave reads 64
// consecutive words (neighbouring rows), the words are transposed through LDS,
// and every lane writes one 16-byte packed chunk
template <int W, int ND, bool WTC>
__device__ __forceinline__ void pack_il_tile(const KArgs<ND> &a, uint32_t tileIdx, uint32_t ntiles) {
  typedef typename Word<W>::T WT;
  constexpr int CW = 16 / W;
  __shared__ uint4 tile[kBlock];
  const uint32_t c0 = tileIdx * kBlock;
  const uint32_t c1 = min(c0 + uint32_t(kBlock), a.nchunks);
  const bool clean = c1 - c0 == uint32_t(kBlock) && int64_t(c0) * CW - a.head >= 0 &&
                     int64_t(c1) * CW - a.head <= int64_t(a.nwords);
  if (!clean) { // uniform: this tile's chunks, one per lane
    pack_body<W, ND, WTC, 1>(a, tileIdx, ntiles);
    return;
  }
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  WT *dst = reinterpret_cast<WT *>(tile + wave * 64);
  const uint32_t qw = uint32_t(int64_t(c0 + wave * 64) * CW - a.head);
  WT v[CW];
  bool decoded = false;
  if constexpr (ND >= 2 && ND <= 3) { // the wave's rows in one innermost run (uniform): one decode for the wave
    uint32_t dig0[ND];
    const uint32_t r0 = mdiv(qw, a.mwpr);
    const int64_t base0 = row_offset<ND>(r0, a, dig0);
    if (one_run<ND>(r0, mdiv(qw + uint32_t(64 * CW - 1), a.mwpr), dig0, a)) {
#pragma unroll
      for (int j = 0; j < CW; ++j) {
        const uint32_t q = qw + uint32_t(j) * 64 + lane;
        const uint32_t row = mdiv(q, a.mwpr);
        const uint32_t w = q - row * a.wpr;
        v[j] = *reinterpret_cast<const WT *>(a.strided + base0 + int64_t(row - r0) * a.stride[0] + int64_t(w) * W);
      }
      decoded = true;
    }
  }
  if (!decoded) {
#pragma unroll
    for (int j = 0; j < CW; ++j) {
      const uint32_t q = qw + uint32_t(j) * 64 + lane;
      const uint32_t row = mdiv(q, a.mwpr);
      const uint32_t w = q - row * a.wpr;
      uint32_t dig[ND > 0 ? ND : 1];
      v[j] = *reinterpret_cast<const WT *>(a.strided + row_offset<ND>(row, a, dig) + int64_t(w) * W);
    }
  }
#pragma unroll
  for (int j = 0; j < CW; ++j) dst[uint32_t(j) * 64 + lane] = v[j];
  __syncthreads();
  st_packed<WTC>(a.flags, reinterpret_cast<uint4 *>(a.chunk0 + size_t(c0 + threadIdx.x) * 16), tile[threadIdx.x]);
}

template <int W, int ND, bool WTC>
__global__ __launch_bounds__(kBlock) void pack_il_kernel(const KArgs<ND> a, const Sig sg) {
  const uint32_t tile = xcd_tile(blockIdx.x, gridDim.x, a.flags);
  pack_il_tile<W, ND, WTC>(a, tile, gridDim.x);
  wg_signal(sg, needs_release(a.flags, tile, gridDim.x));
}
template <int W, int ND> __global__ __launch_bounds__(kBlock) void unpack_il_kernel(const KArgs<ND> a, const Sig sg) {
  unpack_il_tile<W, ND>(a, xcd_tile(blockIdx.x, gridDim.x, a.flags), gridDim.x);
  wg_signal(sg, true);
}

// ------------------------------------------------- dense-window gather (pack)
//
// Narrow rows packed tightly (1- or 2-byte words, inner stride
// s <= kDenseRatio * b): every 64-byte DRAM sector of the strided side holds
// payload, so reading the whole window costs no more HBM traffic than reading
// the rows, but the per-word path spends one 1/2/4-byte load instruction per
// row. Here a workgroup's kBlock x 16 bytes of packed output covers rows [rl, rh] of one
// inner segment, whose window the workgroup streams into LDS
// with 16-byte coalesced loads (<= kBlock*16*kDenseRatio + s bytes); each lane then gathers its 16 output bytes
// from LDS (ds_read_u8) and writes them with one 16-byte store -- the "LDS
// staging to transpose narrow strided blocks into wide contiguous writes" of
// the design. A tile whose rows straddle two segments of an outer dimension
// takes the per-word path (pack_body). The window's aligned 16-byte ends lie
// in the 16-byte chunks holding the first / last payload byte, and every gap
// inside it is shorter than 64 bytes between two payload bytes, so no byte
// outside pages the type already touches is read. Byte-for-byte identical to
// pack_body (type-map order).
#ifndef TEMPI_DENSE_RATIO
#define TEMPI_DENSE_RATIO 4
#endif
constexpr int kDenseRatio = TEMPI_DENSE_RATIO;
// Each lane's gather starts at a lane-dependent dword of its 16 bytes: without
// that, lane L's k-th byte read sits near L * 16 * s / b, for s / b = 2 on 4
// of a 32-lane group's banks (8-way conflicts; SQ_LDS_BANK_CONFLICT 7x lower
// with the rotation, profiles/r05/dense_lds_pmc_s16.txt).
#ifndef TEMPI_DENSE_ROT
#define TEMPI_DENSE_ROT 1
#endif
constexpr int kDenseLds = kBlock * 16 * kDenseRatio + 512;
constexpr int kDenseMaxBlock = 32;
// a workgroup's window must fit the CU's 160 KiB of LDS with room for a
// second workgroup on the CU (so <= 64 KiB)
static_assert(kDenseLds <= 64 * 1024, "dense window too large for LDS");

template <int ND, bool WTC>
__device__ __forceinline__ void pack_dense_tile(const KArgs<ND> &a, uint32_t blk) {
  __shared__ uint4 win[kDenseLds / 16];
  const uint32_t c0 = blk * kBlock; // first chunk of this tile
  const uint32_t c1 = min(c0 + uint32_t(kBlock), a.nchunks);
  // packed bytes of the tile (W = 1: words are bytes)
  const int64_t qlo = max(int64_t(c0) * 16 - int64_t(a.head), int64_t(0));
  const int64_t qhi = min(int64_t(c1) * 16 - int64_t(a.head), int64_t(a.nwords)) - 1;
  const uint32_t rl = mdiv(uint32_t(qlo), a.mwpr), rh = mdiv(uint32_t(qhi), a.mwpr);
  bool oneSegment = true;
  if (ND >= 2) oneSegment = mdiv(rl, a.mcnt[0]) == mdiv(rh, a.mcnt[0]);
  if (!oneSegment) { // uniform: the per-word path for this tile only
    pack_body<1, ND, WTC, 1>(a, blk, gridDim.x);
    return;
  }
  uint32_t dig[ND > 0 ? ND : 1];
  const int64_t offLo = row_offset<ND>(rl, a, dig);
  const char *first = a.strided + offLo;
  const char *A = reinterpret_cast<const char *>(reinterpret_cast<uintptr_t>(first) & ~uintptr_t(15));
  const int64_t span = int64_t(rh - rl) * a.stride[0] + a.wpr; // bytes from first row to end of last
  const int64_t winEnd = (first - A) + span;                  // bytes from A
  const uint32_t nvec = uint32_t((winEnd + 15) / 16);
  for (uint32_t v = threadIdx.x; v < nvec; v += kBlock)
    win[v] = ld(reinterpret_cast<const uint4 *>(A) + v, true);
  __syncthreads();
  const unsigned char *w8 = reinterpret_cast<const unsigned char *>(win);
  const uint32_t base = uint32_t(first - A);
  const uint32_t c = c0 + threadIdx.x;
  if (c >= c1) return;
  const int64_t q0 = int64_t(c) * 16 - a.head;
  const int64_t stride = a.stride[0];
  if (q0 >= 0 && q0 + 16 <= int64_t(a.nwords)) {
    uint32_t row = mdiv(uint32_t(q0), a.mwpr);
    uint32_t w = uint32_t(q0) - row * a.wpr;
    int64_t idx = int64_t(base) + int64_t(row - rl) * stride + w;
    union {
      uint4 v;
      unsigned char b[16];
      uint32_t d[4];
    } out;
#if TEMPI_DENSE_ROT
    // lanes 4k..4k+3 start their 16 bytes at dword k % 4 and wrap, so one
    // ds_read_u8 instruction spreads its addresses over 4x more banks; the
    // dwords are rotated back into place before the store
    const uint32_t rot = (threadIdx.x >> 2) & 3, wrapAt = 16 - 4 * rot;
    const uint32_t w0 = w;
    const int64_t idx0 = idx;
    {
      const uint32_t qs = uint32_t(q0) + 4 * rot;
      const uint32_t rs = mdiv(qs, a.mwpr);
      w = qs - rs * a.wpr;
      idx = int64_t(base) + int64_t(rs - rl) * stride + w;
    }
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      if (uint32_t(m) == wrapAt) {
        idx = idx0;
        w = w0;
      }
      out.b[m] = w8[idx];
      if (++w == a.wpr) {
        w = 0;
        idx += stride - int64_t(a.wpr) + 1;
      } else {
        ++idx;
      }
    }
    // slot dword i holds output dword (i + rot) % 4
    uint32_t d0 = out.d[0], d1 = out.d[1], d2 = out.d[2], d3 = out.d[3];
    if (rot & 1) {
      const uint32_t t = d3;
      d3 = d2; d2 = d1; d1 = d0; d0 = t;
    }
    if (rot & 2) {
      uint32_t t = d0; d0 = d2; d2 = t;
      t = d1; d1 = d3; d3 = t;
    }
    out.d[0] = d0; out.d[1] = d1; out.d[2] = d2; out.d[3] = d3;
#else
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      out.b[j] = w8[idx];
      if (++w == a.wpr) {
        w = 0;
        idx += stride - int64_t(a.wpr) + 1;
      } else {
        ++idx;
      }
    }
#endif
    st_packed<WTC>(a.flags, reinterpret_cast<uint4 *>(a.chunk0 + size_t(c) * 16), out.v);
  } else { // first / last chunk of the object: only its bytes
    for (int j = 0; j < 16; ++j) {
      const int64_t q = q0 + j;
      if (q < 0 || q >= int64_t(a.nwords)) continue;
      const uint32_t row = mdiv(uint32_t(q), a.mwpr);
      const uint32_t w = uint32_t(q) - row * a.wpr;
      a.chunk0[size_t(c) * 16 + size_t(j)] = w8[int64_t(base) + int64_t(row - rl) * stride + w];
    }
  }
}

template <int ND, bool WTC>
__global__ __launch_bounds__(kBlock) void pack_dense_kernel(const KArgs<ND> a, const Sig sg) {
  const uint32_t tile = xcd_tile(blockIdx.x, gridDim.x, a.flags);
  pack_dense_tile<ND, WTC>(a, tile);
  wg_signal(sg, needs_release(a.flags, tile, gridDim.x));
}

// Many objects in ONE launch (e.g. the 26 x nQuants faces of a halo step):
// the descriptors travel in the kernel arguments (<= 4 KiB), each object owns
// a contiguous range of workgroups, and a workgroup finds its object with a
// uniform binary search over the range starts. This replaces one launch
// (~7 us of host time on MI355X/ROCm 7.2) per message by one per batch.
constexpr int kBatchBytes = 3584;
template <int ND> struct BatchArgs {
  static constexpr int kMax = int((kBatchBytes - 8) / (sizeof(KArgs<ND>) + 4));
  uint32_t nitems;
  uint32_t first[kMax + 1]; // first workgroup of each object; first[nitems] = total
  KArgs<ND> item[kMax];
};

template <int ND> __device__ __forceinline__ uint32_t find_item(const BatchArgs<ND> &b, uint32_t blk) {
  uint32_t lo = 0, hi = b.nitems;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (blk >= b.first[mid])
      lo = mid;
    else
      hi = mid;
  }
  return lo;
}

// (sg: a completion ticket folded into the launch, as in the single-object
// kernels; a workgroup's partial chunks are its item's first / last tile)
template <int W, int ND, bool WTC>
__global__ __launch_bounds__(kBlock) void pack_batch_kernel(const BatchArgs<ND> b, const Sig sg) {
  const uint32_t i = find_item<ND>(b, blockIdx.x), n = b.first[i + 1] - b.first[i];
  const uint32_t blk = xcd_tile(blockIdx.x - b.first[i], n, b.item[i].flags); // (within the item: balanced)
  pack_body<W, ND, WTC>(b.item[i], blk, n);
  wg_signal(sg, needs_release(b.item[i].flags, blk, n));
}

template <int W, int ND, bool WTC>
__global__ __launch_bounds__(kBlock) void pack_il_batch_kernel(const BatchArgs<ND> b, const Sig sg) {
  const uint32_t i = find_item<ND>(b, blockIdx.x), n = b.first[i + 1] - b.first[i];
  const uint32_t blk = xcd_tile(blockIdx.x - b.first[i], n, b.item[i].flags); // (within the item: balanced)
  pack_il_tile<W, ND, WTC>(b.item[i], blk, n);
  wg_signal(sg, needs_release(b.item[i].flags, blk, n));
}
template <int W, int ND>
__global__ __launch_bounds__(kBlock) void unpack_il_batch_kernel(const BatchArgs<ND> b, const Sig sg) {
  const uint32_t i = find_item<ND>(b, blockIdx.x), n = b.first[i + 1] - b.first[i];
  const uint32_t blk = xcd_tile(blockIdx.x - b.first[i], n, b.item[i].flags); // (within the item: balanced)
  unpack_il_tile<W, ND>(b.item[i], blk, n);
  wg_signal(sg, true);
}

template <int W, int ND, bool WTC>
__global__ __launch_bounds__(kBlock) void unpack_batch_kernel(const BatchArgs<ND> b, const Sig sg) {
  const uint32_t i = find_item<ND>(b, blockIdx.x), n = b.first[i + 1] - b.first[i];
  const uint32_t blk = xcd_tile(blockIdx.x - b.first[i], n, b.item[i].flags); // (within the item: balanced)
  unpack_body<W, ND, WTC>(b.item[i], blk, n);
  wg_signal(sg, needs_release(b.item[i].flags, blk, n));
}

// ---------------------------------------------------------------- host side

struct Norm {
  int64_t block;
  int nd;                  // outermost first
  int64_t cnt[TEMPI_HIP_MAX_DIMS];
  int64_t str[TEMPI_HIP_MAX_DIMS];
};

// drop unit dims, fold a dense innermost dim into the block, merge adjacent
// dims whose strides line up -- every step preserves type-map order
bool normalise(const tempi_hip_desc *d, Norm *n) {
  if (d->ndims < 0 || d->ndims > TEMPI_HIP_MAX_DIMS || d->block < 0) return false;
  n->block = d->block;
  n->nd = 0;
  for (int k = 0; k < d->ndims; ++k) {
    if (d->counts[k] < 0) return false;
    if (d->counts[k] == 1) continue;
    n->cnt[n->nd] = d->counts[k];
    n->str[n->nd] = d->strides[k];
    n->nd++;
  }
  bool changed = true;
  while (changed) {
    changed = false;
    if (n->nd && n->str[n->nd - 1] == n->block) {
      n->block *= n->cnt[n->nd - 1];
      n->nd--;
      changed = true;
    }
    for (int k = 0; k + 1 < n->nd; ++k) {
      if (n->str[k] == n->cnt[k + 1] * n->str[k + 1]) {
        n->cnt[k] *= n->cnt[k + 1];
        n->str[k] = n->str[k + 1];
        for (int j = k + 1; j + 1 < n->nd; ++j) {
          n->cnt[j] = n->cnt[j + 1];
          n->str[j] = n->str[j + 1];
        }
        n->nd--;
        changed = true;
        break;
      }
    }
  }
  return true;
}

int64_t norm_bytes(const Norm &n) {
  int64_t b = n.block;
  for (int k = 0; k < n.nd; ++k) b *= n.cnt[k];
  return b;
}

int word_width(uintptr_t packed, uintptr_t first, const Norm &n) {
  uint64_t g = 16 | packed | first | uint64_t(n.block);
  for (int k = 0; k < n.nd; ++k) {
    const int64_t s = n.str[k];
    g |= uint64_t(s < 0 ? -s : s);
  }
  // lowest set bit of the OR = largest power of two dividing all of them
  return int(g & (~g + 1));
}

// kXcdRange when a scatter onto this strided side writes sectors in part
// (block, a stride or the base not a multiple of the 32-byte sector) AND
// neighbouring rows share lines (gap < 128 B), with rows below kXcdMaxBlock:
// isolated rows (the halo's x faces) have nothing to merge, and long rows
// are whole-line streams, which the dealt order serves better.
// (a build with -DTEMPI_XCD_MAP=0: never, for A/B runs)
#ifndef TEMPI_XCD_MAX_BLOCK
#define TEMPI_XCD_MAX_BLOCK 1024
#endif
// Rows of whole 64-byte sectors that leave part of every 4 KiB page of the
// strided side untouched (inner stride >= 4 KiB, rows < 4 KiB), and 64-byte
// rows with gaps >= 128 B: in the dealt order the eight XCDs write one narrow
// window at a time, whose addresses keep the same bits below 4 KiB, so only
// part of the HBM channels take the writes; one contiguous range per XCD puts
// eight far-apart windows in flight instead. Measured on MI355X (round 3,
// profiles/r03/gap3_ab_s4.jsonl, 1 GiB, kernel time): unpack 512:4096 +33 %,
// 1024:8192 +20 %, 1024:4096 +15 %, 3D 2048:4096 +14 %, 256:4096 +13 %,
// 2048:8192 +12 %, 64:4096 +7 %, 64:512 +6 %; the same shapes' bare access
// pattern (tools/calib.hip sect_copy, sect3_s4.jsonl) +5 to +41 %. Rows of
// 4 KiB or more (whole pages: 4096:8192 -5 %), and strides below 4 KiB
// (512:1024 -5 %, 128:256 -4 %), keep the dealt order.
// TEMPI_XCD_PAGES=0 turns the rule off; TEMPI_XCD_PAGES_PACK=1 applies it to
// gathers too (A/B).
#ifndef TEMPI_XCD_PAGES
#define TEMPI_XCD_PAGES 1
#endif
#ifndef TEMPI_XCD_PAGES_PACK
#define TEMPI_XCD_PAGES_PACK 0
#endif
bool partial_pages(const Norm &n) {
  if (n.nd == 0 || n.block % 64) return false;
  const int64_t inner = n.str[n.nd - 1];
  if (inner < n.block) return false;
  if (n.block == 64 && inner - n.block >= 128) return true;
  return inner >= 4096 && n.block < 4096 && inner - n.block >= 128;
}

// One exception above TEMPI_XCD_MAX_BLOCK: 2D rows of
// 4-8 KiB a few bytes apart (the sweep's 4096 : 4112). Each row's last line
// is shared with the next row's first, and in the dealt order the two halves
// come from workgroups on different XCDs: two partial-line writes (32-byte
// requests, 2.1 per row, profiles/r06/kpmc_rowends_s3.txt) instead of one
// line. Mapped: unpack +6 to +9.5 % (5.54 -> 5.90 TB/s); the same rule on
// 1 and 2 KiB rows and on the 3D forms of all three costs 0.5-2 %
// (profiles/r06/xcd_4112_ab_s5.jsonl, xcd_ab_wide_s6.jsonl), so it stays
// this narrow.
bool wide_shared_line_rows(const Norm &n) { return n.nd == 1 && n.block >= 4096 && n.block < 8192; }

uint32_t xcd_flag(const char *first, const Norm &n, bool pack) {
  if (!TEMPI_XCD_MAP) return 0;
  if (TEMPI_XCD_PAGES && (!pack || TEMPI_XCD_PAGES_PACK) && partial_pages(n)) return kXcdRange;
  if (pack || n.nd == 0 || (n.block >= TEMPI_XCD_MAX_BLOCK && !wide_shared_line_rows(n))) return 0;
  const int64_t inner = n.str[n.nd - 1];
  if (inner < n.block || inner - n.block >= 128) return 0;
  uint64_t g = reinterpret_cast<uintptr_t>(first) | uint64_t(n.block);
  for (int k = 0; k < n.nd; ++k) g |= uint64_t(n.str[k] < 0 ? -n.str[k] : n.str[k]);
  return (g & 31) ? kXcdRange : 0;
}

// TEMPI_HIP_ITEM_* of the object make_args is describing (set around each
// item by run_batch; 0 for the single-object entry points)
thread_local uint32_t gItemFlags = 0;

// the completion-ticket fold offered to this thread's next single-object
// launch (the *_ticket entry points set it around their launch)
thread_local tempi_ticket::Fold *gFold = nullptr;
// a 16-byte-word scatter may store write-through (st_scatter): every stride
// >= 0 and the object's span below 2 GiB
bool scatter_write_through(const Norm &n) {
  int64_t span = n.block;
  for (int k = 0; k < n.nd; ++k) {
    if (n.str[k] < 0) return false;
    span += (n.cnt[k] - 1) * n.str[k];
  }
  return span < (int64_t(1) << 31);
}

// the kernel's Sig for a launch of `blocks` workgroups: the fold when one is
// offered and the grid is small enough (counted on the host as the kernel
// will count on the device), else none
Sig take_fold_from(tempi_ticket::Fold *f, uint32_t blocks, bool writeThrough) {
  using tempi_ticket::kShards;
  Sig sg{};
  if (!f || f->taken || !f->t || !f->t->counter || blocks == 0 ||
      blocks > (writeThrough ? f->max_blocks_wt : f->max_blocks))
    return sg;
  uint32_t *counted = f->t->counted;
  for (uint32_t k = 0; k < uint32_t(kShards); ++k) { // workgroups b with b % kShards == k
    if (blocks > k) counted[k] += (blocks - k + kShards - 1) / kShards;
    sg.target[k] = counted[k];
  }
  counted[kShards] += blocks < uint32_t(kShards) ? blocks : uint32_t(kShards); // shards that get a workgroup
  sg.top = counted[kShards];
  f->taken = true;
  sg.counter = f->t->counter;
  sg.flag = f->t->dev;
  sg.ticket = f->ticket;
  return sg;
}
Sig take_fold(uint32_t blocks, bool writeThrough) { return take_fold_from(gFold, blocks, writeThrough); }

// descriptor + workgroup count of one object
template <int W, int ND>
void make_args(char *packed, char *first, const Norm &n, KArgs<ND> *out, uint32_t *blocks) {
  KArgs<ND> &a = *out;
  a = KArgs<ND>{};
  const uint64_t nwords = uint64_t(norm_bytes(n)) / W;
  const uint32_t head = uint32_t((reinterpret_cast<uintptr_t>(packed) & 15) / W);
  constexpr int CW = 16 / W;
  a.chunk0 = packed - size_t(head) * W;
  a.strided = first;
  a.flags = gItemFlags;
  a.nwords = uint32_t(nwords);
  a.head = head;
  a.nchunks = uint32_t((nwords + head + CW - 1) / CW);
  a.wpr = uint32_t(n.block / W);
  a.mwpr = make_magic(a.wpr);
  for (int k = 0; k < ND; ++k) {
    const int src = n.nd - 1 - k; // innermost first
    a.cnt[k] = uint32_t(n.cnt[src]);
    a.mcnt[k] = make_magic(a.cnt[k]);
    a.stride[k] = n.str[src];
    a.wrap[k] = n.cnt[src] * n.str[src];
  }
  constexpr int U = Unroll<W>::U;
  uint64_t b = (uint64_t(a.nchunks) + kBlock * U - 1) / (kBlock * U);
  if (b > TEMPI_MAX_BLOCKS) b = TEMPI_MAX_BLOCKS; // grid-stride beyond
  *blocks = uint32_t(b);
}

template <int W, int ND>
int launch_nd(bool pack, char *packed, char *first, const Norm &n, hipStream_t s) {
  KArgs<ND> a;
  uint32_t blocks;
  make_args<W, ND>(packed, first, n, &a, &blocks);
  if (blocks == 0) return 0;
  a.flags |= xcd_flag(first, n, pack);
  const bool wt = pack || (W == 16 && scatter_write_through(n));
  const Sig sg = take_fold(blocks, wt);
  if (sg.flag && wt) a.flags |= kWriteThrough;
  // (a scatter stores write-through only with 16-byte words: no WTC twin below)
  constexpr bool kScatterWT = W == 16;
  const bool wtc = (a.flags & kWriteThrough) != 0;
  if (pack) {
    auto *k = wtc ? pack_kernel<W, ND, true> : pack_kernel<W, ND, false>;
    TEMPI_LAUNCH(k, dim3(blocks), dim3(kBlock), 0, s, a, sg);
  } else {
    auto *k = wtc ? unpack_kernel<W, ND, kScatterWT> : unpack_kernel<W, ND, false>;
    TEMPI_LAUNCH(k, dim3(blocks), dim3(kBlock), 0, s, a, sg);
  }
  return int(hipGetLastError());
}

struct Job {
  char *packed, *first;
  Norm n;
  uint32_t flags;
};

// fold: offered to this group's last launch (the caller passes it to the
// batch's last group only, so that the ticket follows every launch of it)
template <int W, int ND>
int launch_batch_nd(bool pack, const std::vector<Job> &jobs, hipStream_t s, tempi_ticket::Fold *fold) {
  const bool il = il_width(pack, W); // il kernels: one kBlock x 16-byte tile per workgroup
  BatchArgs<ND> b;
  bool wt[BatchArgs<ND>::kMax]; // item may store write-through if the launch folds a ticket
  b.nitems = 0;
  uint32_t total = 0;
  auto flush = [&](bool last) -> int {
    if (!b.nitems) return 0;
    b.first[b.nitems] = total;
    Sig sg{};
    bool wtc = false; // some item stores write-through: the WTC instantiation
    if (last && fold && total) {
      bool all = true;
      for (uint32_t k = 0; k < b.nitems; ++k) all &= wt[k];
      sg = take_fold_from(fold, total, all);
      if (sg.flag)
        for (uint32_t k = 0; k < b.nitems; ++k)
          if (wt[k]) {
            b.item[k].flags |= kWriteThrough;
            wtc = true;
          }
    }
    constexpr bool kScatterWT = W == 16;
    if (total && b.nitems == 1) {
      // one item (a lone small message): the single-object kernel, same body,
      // whose arguments are the item alone instead of the 3.5 KiB batch
      const KArgs<ND> &a = b.item[0];
      if (il)
        if (pack)
          TEMPI_LAUNCH((wtc ? pack_il_kernel<W, ND, true> : pack_il_kernel<W, ND, false>), dim3(total),
                             dim3(kBlock), 0, s, a, sg);
        else
          TEMPI_LAUNCH((unpack_il_kernel<W, ND>), dim3(total), dim3(kBlock), 0, s, a, sg);
      else if (pack)
        TEMPI_LAUNCH((wtc ? pack_kernel<W, ND, true> : pack_kernel<W, ND, false>), dim3(total), dim3(kBlock),
                           0, s, a, sg);
      else
        TEMPI_LAUNCH((wtc ? unpack_kernel<W, ND, kScatterWT> : unpack_kernel<W, ND, false>), dim3(total),
                           dim3(kBlock), 0, s, a, sg);
    } else if (total) {
      if (il)
        if (pack)
          TEMPI_LAUNCH((wtc ? pack_il_batch_kernel<W, ND, true> : pack_il_batch_kernel<W, ND, false>),
                             dim3(total), dim3(kBlock), 0, s, b, sg);
        else
          TEMPI_LAUNCH((unpack_il_batch_kernel<W, ND>), dim3(total), dim3(kBlock), 0, s, b, sg);
      else if (pack)
        TEMPI_LAUNCH((wtc ? pack_batch_kernel<W, ND, true> : pack_batch_kernel<W, ND, false>), dim3(total),
                           dim3(kBlock), 0, s, b, sg);
      else
        TEMPI_LAUNCH((wtc ? unpack_batch_kernel<W, ND, kScatterWT> : unpack_batch_kernel<W, ND, false>),
                           dim3(total), dim3(kBlock), 0, s, b, sg);
    }
    b.nitems = 0;
    total = 0;
    return int(hipGetLastError());
  };
  for (const Job &j : jobs) {
    KArgs<ND> a;
    uint32_t blocks;
    gItemFlags = j.flags;
    make_args<W, ND>(j.packed, j.first, j.n, &a, &blocks);
    gItemFlags = 0;
    a.flags |= xcd_flag(j.first, j.n, pack);
    if (il) blocks = (a.nchunks + kBlock - 1) / kBlock;
    if (!blocks) continue;
    if (uint64_t(total) + blocks >= (uint64_t(1) << 31))
      if (int e = flush(false)) return e;
    b.first[b.nitems] = total;
    b.item[b.nitems] = a;
    // gathers write whole packed chunks; scatters of 16-byte words write-through
    // only where st_scatter allows it (the il scatters never: narrow words)
    wt[b.nitems] = pack || (!il && W == 16 && scatter_write_through(j.n));
    b.nitems++;
    total += blocks;
    if (b.nitems == uint32_t(BatchArgs<ND>::kMax))
      if (int e = flush(false)) return e;
  }
  return flush(true);
}

template <int W>
int launch_batch_w(bool pack, int nd, const std::vector<Job> &jobs, hipStream_t s, tempi_ticket::Fold *fold) {
  switch (nd) {
  case 0: return launch_batch_nd<W, 0>(pack, jobs, s, fold);
  case 1: return launch_batch_nd<W, 1>(pack, jobs, s, fold);
  case 2: return launch_batch_nd<W, 2>(pack, jobs, s, fold);
  case 3: return launch_batch_nd<W, 3>(pack, jobs, s, fold);
  case 4: return launch_batch_nd<W, 4>(pack, jobs, s, fold);
  case 5: return launch_batch_nd<W, 5>(pack, jobs, s, fold);
  default: return int(hipErrorInvalidValue);
  }
}

template <int W>
int launch_w(bool pack, char *packed, char *first, const Norm &n, hipStream_t s) {
  switch (n.nd) {
  case 0: return launch_nd<W, 0>(pack, packed, first, n, s);
  case 1: return launch_nd<W, 1>(pack, packed, first, n, s);
  case 2: return launch_nd<W, 2>(pack, packed, first, n, s);
  case 3: return launch_nd<W, 3>(pack, packed, first, n, s);
  case 4: return launch_nd<W, 4>(pack, packed, first, n, s);
  case 5: return launch_nd<W, 5>(pack, packed, first, n, s);
  default: return int(hipErrorInvalidValue);
  }
}

#ifndef TEMPI_DENSE
#define TEMPI_DENSE 1
#endif
// narrow rows packed tightly enough for pack_dense_kernel (see there)
bool dense_ok(const Norm &n, int w) {
  // measured (tools/kbench.cpp): wins for 1- and 2-byte words at stride <= 4
  // blocks (1 B : 2 B 2.3x, 3 B : 7 B +11%); 4-byte words are already at the
  // sector bound on the per-word path, and wider windows lose
  if (!TEMPI_DENSE || w > 2 || n.nd < 1 || n.block > kDenseMaxBlock) return false;
  const int64_t s = n.str[n.nd - 1], b = n.block; // innermost dimension
  if (s <= 0 || s > kDenseRatio * b || s - b >= 64) return false; // (gaps inside sectors the type touches)
  // outer dimensions: inner segments long enough that few tiles straddle two
  return n.nd == 1 || n.cnt[n.nd - 1] * b >= 4 * 4096;
}

template <int ND> int launch_dense_nd(char *packed, char *first, const Norm &n, hipStream_t s) {
  KArgs<ND> a;
  uint32_t blocks;
  make_args<1, ND>(packed, first, n, &a, &blocks);
  if (blocks == 0) return 0;
  const Sig sg = take_fold(blocks, true);
  if (sg.flag) a.flags |= kWriteThrough;
  auto *k = sg.flag ? pack_dense_kernel<ND, true> : pack_dense_kernel<ND, false>;
  TEMPI_LAUNCH(k, dim3(blocks), dim3(kBlock), 0, s, a, sg);
  return int(hipGetLastError());
}

int launch_dense(char *packed, char *first, const Norm &n, hipStream_t s) {
  switch (n.nd) {
  case 1: return launch_dense_nd<1>(packed, first, n, s);
  case 2: return launch_dense_nd<2>(packed, first, n, s);
  case 3: return launch_dense_nd<3>(packed, first, n, s);
  case 4: return launch_dense_nd<4>(packed, first, n, s);
  case 5: return launch_dense_nd<5>(packed, first, n, s);
  default: return int(hipErrorInvalidValue);
  }
}

template <int W, int ND> int launch_il_nd(bool pack, char *packed, char *first, const Norm &n, hipStream_t s) {
  KArgs<ND> a;
  uint32_t blocks;
  make_args<W, ND>(packed, first, n, &a, &blocks);
  blocks = (a.nchunks + kBlock - 1) / kBlock; // one tile per workgroup, no grid-stride
  if (blocks == 0) return 0;
  a.flags |= xcd_flag(first, n, pack);
  const Sig sg = take_fold(blocks, pack);
  if (sg.flag && pack) a.flags |= kWriteThrough;
  if (pack) {
    auto *k = sg.flag ? pack_il_kernel<W, ND, true> : pack_il_kernel<W, ND, false>;
    TEMPI_LAUNCH(k, dim3(blocks), dim3(kBlock), 0, s, a, sg);
  } else {
    TEMPI_LAUNCH((unpack_il_kernel<W, ND>), dim3(blocks), dim3(kBlock), 0, s, a, sg);
  }
  return int(hipGetLastError());
}

template <int W> int launch_il(bool pack, char *packed, char *first, const Norm &n, hipStream_t s) {
  switch (n.nd) {
  case 0: return launch_il_nd<W, 0>(pack, packed, first, n, s);
  case 1: return launch_il_nd<W, 1>(pack, packed, first, n, s);
  case 2: return launch_il_nd<W, 2>(pack, packed, first, n, s);
  case 3: return launch_il_nd<W, 3>(pack, packed, first, n, s);
  case 4: return launch_il_nd<W, 4>(pack, packed, first, n, s);
  case 5: return launch_il_nd<W, 5>(pack, packed, first, n, s);
  default: return int(hipErrorInvalidValue);
  }
}

int launch_one(bool pack, char *packed, char *first, const Norm &n, hipStream_t s) {
  const int w = word_width(reinterpret_cast<uintptr_t>(packed),
                           reinterpret_cast<uintptr_t>(first), n);
  if (pack && dense_ok(n, w)) return launch_dense(packed, first, n, s);
  if (il_width(pack, w)) {
    switch (w) {
    case 1: return launch_il<1>(pack, packed, first, n, s);
    case 2: return launch_il<2>(pack, packed, first, n, s);
    case 4: return launch_il<4>(pack, packed, first, n, s);
    case 8: return launch_il<8>(pack, packed, first, n, s);
    default: break;
    }
  }
  switch (w) {
  case 1: return launch_w<1>(pack, packed, first, n, s);
  case 2: return launch_w<2>(pack, packed, first, n, s);
  case 4: return launch_w<4>(pack, packed, first, n, s);
  case 8: return launch_w<8>(pack, packed, first, n, s);
  default: return launch_w<16>(pack, packed, first, n, s);
  }
}

constexpr int64_t kMaxLaunchBytes = int64_t(1) << 31; // words < 2^31 at W = 1

// split anything a single 32-bit-indexed launch cannot cover
int launch_split(bool pack, char *packed, char *first, const Norm &n, hipStream_t s) {
  const int64_t bytes = norm_bytes(n);
  if (bytes == 0) return 0;
  if (bytes < kMaxLaunchBytes) {
    // every dimension count must fit in 32 bits too
    bool ok = true;
    for (int k = 0; k < n.nd; ++k) ok &= n.cnt[k] < (int64_t(1) << 32);
    if (ok) return launch_one(pack, packed, first, n, s);
  }
  if (n.nd == 0) { // one huge contiguous block: cut it into pieces
    const int64_t piece = int64_t(1) << 30;
    for (int64_t o = 0; o < n.block; o += piece) {
      Norm p = n;
      p.block = (n.block - o < piece) ? n.block - o : piece;
      if (int e = launch_one(pack, packed + o, first + o, p, s)) return e;
    }
    return 0;
  }
  // split the outermost dimension into groups that fit
  const int64_t per = bytes / n.cnt[0];
  Norm inner = n;
  if (per >= kMaxLaunchBytes / 2) { // recurse one level down per outer index
    inner.nd = n.nd - 1;
    for (int k = 0; k < inner.nd; ++k) {
      inner.cnt[k] = n.cnt[k + 1];
      inner.str[k] = n.str[k + 1];
    }
    for (int64_t i = 0; i < n.cnt[0]; ++i)
      if (int e = launch_split(pack, packed + i * per, first + i * n.str[0], inner, s)) return e;
    return 0;
  }
  const int64_t group = (kMaxLaunchBytes / 2) / per;
  for (int64_t i = 0; i < n.cnt[0]; i += group) {
    inner.cnt[0] = (n.cnt[0] - i < group) ? n.cnt[0] - i : group;
    if (int e = launch_split(pack, packed + i * per, first + i * n.str[0], inner, s)) return e;
  }
  return 0;
}

// fold (optional): a completion ticket, offered to the batch's LAST launch
// only: the stream runs launches in order, so its ticket follows all of them
int run_batch(bool pack, const tempi_hip_batch_item *items, int n, hipStream_t s,
              tempi_ticket::Fold *fold = nullptr) {
  if (launch_check()) {
    gDesc = std::string(pack ? "pack" : "unpack") + " batch of " + std::to_string(n) + ":";
    for (int i = 0; i < n; ++i)
      gDesc += " " + (pack ? describe(items[i].desc, items[i].packed, items[i].first)
                           : describe(items[i].desc, items[i].first, items[i].packed));
  }
  // group by (word width, rank): one launch per group and per kMax objects
  std::vector<Job> groups[5][TEMPI_HIP_MAX_DIMS + 1];
  for (int i = 0; i < n; ++i) {
    Job j;
    j.packed = static_cast<char *>(items[i].packed);
    j.first = static_cast<char *>(items[i].first);
    j.flags = pack ? 0u : items[i].flags & TEMPI_HIP_ITEM_REMOTE; // (gathers read the strided side only)
    if (!normalise(&items[i].desc, &j.n)) return int(hipErrorInvalidValue);
    const int64_t bytes = norm_bytes(j.n);
    if (bytes == 0) continue;
    if (bytes >= kMaxLaunchBytes) { // too big for one 32-bit-indexed item
      gItemFlags = j.flags;
      const int e = launch_split(pack, j.packed, j.first, j.n, s);
      gItemFlags = 0;
      if (e) return e;
      continue;
    }
    const int w = word_width(reinterpret_cast<uintptr_t>(j.packed), reinterpret_cast<uintptr_t>(j.first), j.n);
    const int wi = w == 1 ? 0 : w == 2 ? 1 : w == 4 ? 2 : w == 8 ? 3 : 4;
    groups[wi][j.n.nd].push_back(j);
  }
  int lastGroup = -1;
  for (int g = 0; g < 5 * (TEMPI_HIP_MAX_DIMS + 1); ++g)
    if (!groups[g / (TEMPI_HIP_MAX_DIMS + 1)][g % (TEMPI_HIP_MAX_DIMS + 1)].empty()) lastGroup = g;
  for (int wi = 0; wi < 5; ++wi)
    for (int nd = 0; nd <= TEMPI_HIP_MAX_DIMS; ++nd) {
      const std::vector<Job> &g = groups[wi][nd];
      if (g.empty()) continue;
      tempi_ticket::Fold *f = wi * (TEMPI_HIP_MAX_DIMS + 1) + nd == lastGroup ? fold : nullptr;
      int e = 0;
      switch (wi) {
      case 0: e = launch_batch_w<1>(pack, nd, g, s, f); break;
      case 1: e = launch_batch_w<2>(pack, nd, g, s, f); break;
      case 2: e = launch_batch_w<4>(pack, nd, g, s, f); break;
      case 3: e = launch_batch_w<8>(pack, nd, g, s, f); break;
      default: e = launch_batch_w<16>(pack, nd, g, s, f); break;
      }
      if (e) return e;
    }
  return 0;
}

// ------------------------------------------------------ strided -> strided copy
//
// dst object <- src object, both describing the same bytes in type-map order
// (e.g. a halo face sent to the same process: the interior face of one buffer
// into the exterior face of another). No packed intermediate, so HBM sees the
// payload once each way instead of twice. Each side keeps its own shape: the
// virtual packed word q is decoded independently into a src and a dst offset.
//
// A workgroup owns kCopyBlock * 16/W consecutive words; word j of a lane is
// tileBase + j * kCopyBlock + lane, so every load/store instruction of a wave
// touches 64 consecutive words (coalesced whenever rows are longer than a few
// words). Each side has at most kCopyND dimensions after normalisation (the
// unbounded outermost one lives in the last slot; the unused slots in between
// have count 1, stride 0); anything deeper is reported unsupported and the
// caller packs + unpacks through a slab instead.
constexpr int kCopyND = 3;
// The copy kernels keep 256-lane workgroups: on the halo regions 128 measured
// 2-5 % slower (round 1, profiles/r01/block_ab_s9.jsonl), while the single-object packers gain
// from 128 (see TEMPI_BLOCK)
#ifndef TEMPI_COPY_BLOCK
#define TEMPI_COPY_BLOCK 256
#endif
constexpr int kCopyBlock = TEMPI_COPY_BLOCK;
static_assert(kCopyBlock % 64 == 0 && kCopyBlock >= 64 && kCopyBlock <= 1024,
              "copy kernels interleave whole 64-lane waves");

struct CSide {
  char *first;
  uint32_t wpr;
  Magic mwpr;
  uint32_t cnt[kCopyND - 1]; // the outermost slot is unbounded
  Magic mcnt[kCopyND - 1];
  int64_t stride[kCopyND];
};

struct CArgs {
  CSide s, d;
  // PAIRED items: a second (src, dst) of exactly the same two shapes, moved
  // by the same lanes right after the first. In a halo the two opposite faces
  // of one buffer pair up this way, and the sector one copy writes is the
  // sector the other just read (x faces: [0,24) and [24,48) of each row):
  // the write then lands on a line already in L2 and goes back to HBM whole,
  // instead of as a partial-sector write (a read-modify-write in DRAM)
  char *s2, *d2; // nullptr: not paired
  uint32_t nwords;
  uint32_t flags; // TEMPI_HIP_ITEM_REMOTE: the source is another process's memory
};

// A system-scope load through the flat global path: a relaxed atomic load at
// system scope, which gfx950 issues as global_load_* sc0 sc1 (the same cache
// policy as ld_remote's) and which the compiler tracks like any other load,
// so every load of a lane's words is in flight at once. (The source side of a
// copy may have any stride sign, so the wave-uniform buffer base of ld_remote
// cannot be used.) A 16-byte word is two 8-byte loads.
template <typename T> __device__ __forceinline__ T ld_sys(const T *p) {
  T v;
  if constexpr (sizeof(T) == 16) {
    const uint64_t *q = reinterpret_cast<const uint64_t *>(p);
    const uint64_t x[2] = {__hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM),
                           __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)};
    __builtin_memcpy(&v, x, 16);
  } else {
    typedef typename std::conditional<
        sizeof(T) == 8, uint64_t,
        typename std::conditional<sizeof(T) == 4, uint32_t,
                                  typename std::conditional<sizeof(T) == 2, uint16_t, uint8_t>::type>::type>::type U;
    const U x = __hip_atomic_load(reinterpret_cast<const U *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_memcpy(&v, &x, sizeof(T));
  }
  return v;
}
template <typename T> __device__ __forceinline__ T ld_src(const CArgs &a, const T *p, bool nt) {
  if (a.flags & TEMPI_HIP_ITEM_REMOTE) return ld_sys(p);
  return ld(p, nt);
}

template <int W> __device__ __forceinline__ int64_t side_offset(uint32_t q, const CSide &c) {
  uint32_t row = mdiv(q, c.mwpr);
  int64_t off = int64_t(q - row * c.wpr) * W;
#pragma unroll
  for (int k = 0; k < kCopyND - 1; ++k) {
    const uint32_t r2 = mdiv(row, c.mcnt[k]);
    off += int64_t(row - r2 * c.cnt[k]) * c.stride[k];
    row = r2;
  }
  return off + int64_t(row) * c.stride[kCopyND - 1];
}

#ifndef TEMPI_COPY_U
#define TEMPI_COPY_U 1
#endif
template <int W> __device__ __forceinline__ void copy_body(const CArgs &a, uint32_t blk, uint32_t nblk) {
  typedef typename Word<W>::T WT;
  constexpr int CW = 16 / W * TEMPI_COPY_U;
  constexpr bool nt = W == 16;
  const uint32_t tile = uint32_t(kCopyBlock) * CW;
  if (a.s2) {
    for (uint32_t base = blk * tile; base < a.nwords; base += nblk * tile) {
      WT v[CW], v2[CW];
      int64_t so[CW], dof[CW];
#pragma unroll
      for (int j = 0; j < CW; ++j) {
        const uint32_t q = base + uint32_t(j) * kCopyBlock + threadIdx.x;
        so[j] = q < a.nwords ? side_offset<W>(q, a.s) : 0;
        dof[j] = q < a.nwords ? side_offset<W>(q, a.d) : 0;
        if (q < a.nwords) {
          v[j] = ld_src(a, reinterpret_cast<const WT *>(a.s.first + so[j]), false);
          v2[j] = ld_src(a, reinterpret_cast<const WT *>(a.s2 + so[j]), false);
        }
      }
#pragma unroll
      for (int j = 0; j < CW; ++j) {
        const uint32_t q = base + uint32_t(j) * kCopyBlock + threadIdx.x;
        if (q < a.nwords) {
          st(reinterpret_cast<WT *>(a.d.first + dof[j]), v[j], false);
          st(reinterpret_cast<WT *>(a.d2 + dof[j]), v2[j], false);
        }
      }
    }
    return;
  }
  for (uint32_t base = blk * tile; base < a.nwords; base += nblk * tile) {
    WT v[CW];
#pragma unroll
    for (int j = 0; j < CW; ++j) {
      const uint32_t q = base + uint32_t(j) * kCopyBlock + threadIdx.x;
      if (q < a.nwords) v[j] = ld_src(a, reinterpret_cast<const WT *>(a.s.first + side_offset<W>(q, a.s)), nt);
    }
#pragma unroll
    for (int j = 0; j < CW; ++j) {
      const uint32_t q = base + uint32_t(j) * kCopyBlock + threadIdx.x;
      if (q < a.nwords) st(reinterpret_cast<WT *>(a.d.first + side_offset<W>(q, a.d)), v[j], nt);
    }
  }
}

// ---- the PEELED copy (kPeelItem items of the 8-byte-word launches)
//
// Both sides start 8 bytes past a 16-byte boundary, with rows of a multiple
// of 16 bytes at strides that are multiples of 16: the halo's y / z faces, 4
// KiB rows whose region starts 24 B into 512-B-aligned pitched rows. The
// plain plan moves those in 8-byte words (word_width ORs the bases), and a
// 1 GiB copy of that shape runs at 4.5-4.8 TB/s against 5.4 TB/s in 16-byte
// words (tools/kbench.cpp with KBENCH_OFFSET 24 / 32, profiles/r06/
// koff_s1.jsonl). Here the VIRTUAL byte v = b + 8 (b: the byte in type-map
// order) has v = address (mod 16) on both sides, so virtual chunk c (bytes
// b in [16c - 8, 16c + 8)) is one aligned dwordx4 on each side, unless its
// second half starts a row on either side (a row seam in its middle) or it is
// the first / last chunk (half outside the object): those move as two 8-byte
// halves. a.nwords counts 8-byte words (even), the sides' wpr too.
__device__ __forceinline__ int64_t side_offset_seam(uint32_t q0, const CSide &c, bool *seam) {
  uint32_t row = mdiv(q0, c.mwpr);
  const uint32_t w = q0 - row * c.wpr;
  *seam = w + 1 == c.wpr; // word q0 ends its row: the next word starts one
  int64_t off = int64_t(w) * 8;
#pragma unroll
  for (int k = 0; k < kCopyND - 1; ++k) {
    const uint32_t r2 = mdiv(row, c.mcnt[k]);
    off += int64_t(row - r2 * c.cnt[k]) * c.stride[k];
    row = r2;
  }
  return off + int64_t(row) * c.stride[kCopyND - 1];
}

__device__ __forceinline__ void copy_half(const CArgs &a, uint32_t q, const char *s, char *d) {
  const uint2 v = ld_src(a, reinterpret_cast<const uint2 *>(s + side_offset<8>(q, a.s)), false);
  st(reinterpret_cast<uint2 *>(d + side_offset<8>(q, a.d)), v, false);
}

// the peeled copy's whole chunks go nontemporal unless the item carries
// kCopyPlain (TEMPI_COPY_PEEL=2, an A/B switch)
constexpr uint32_t kCopyPlain = 1u << 29; // internal flag bit (never a TEMPI_HIP_ITEM_*)
__device__ void copy_body_peel(const CArgs &a, uint32_t blk, uint32_t nblk) {
  const uint32_t nchunks = a.nwords / 2 + 1;
  const bool nt = !(a.flags & kCopyPlain);
  for (uint32_t c = blk * kCopyBlock + threadIdx.x; c < nchunks; c += nblk * kCopyBlock) {
    const uint32_t q1 = 2 * c; // the 8-byte word of the chunk's second half
    bool ss = true, ds = true;
    int64_t so = 0, dof = 0;
    if (c > 0 && q1 < a.nwords) {
      so = side_offset_seam(q1 - 1, a.s, &ss);
      dof = side_offset_seam(q1 - 1, a.d, &ds);
    }
    if (!ss && !ds) { // one aligned 16-byte word on each side
      const uint4 v = ld_src(a, reinterpret_cast<const uint4 *>(a.s.first + so), nt);
      uint4 v2;
      if (a.s2) v2 = ld_src(a, reinterpret_cast<const uint4 *>(a.s2 + so), nt);
      st(reinterpret_cast<uint4 *>(a.d.first + dof), v, nt);
      if (a.s2) st(reinterpret_cast<uint4 *>(a.d2 + dof), v2, nt);
      continue;
    }
    for (int h = 0; h < 2; ++h) { // a seam, or the object's first / last chunk
      const uint32_t q = q1 - 1 + uint32_t(h);
      if ((h == 0 && c == 0) || q >= a.nwords) continue;
      copy_half(a, q, a.s.first, a.d.first);
      if (a.s2) copy_half(a, q, a.s2, a.d2);
    }
  }
}

// Peeled items travel in the 8-byte-word launches (their sides count 8-byte
// words too), flagged per item: a flush of a halo then stays ONE launch in
// which the x faces' isolated rows and the y / z faces' streams overlap.
// Launched on their own, after the 8-byte-word items, the peeled faces made
// the 1-rank 512^3 halo 6 % and the 2-rank one 8 % slower than no peel at all
// (profiles/r06/halo_peel_ab_n1_s4.jsonl, _n2_s4), although a 1 GiB copy of
// that row shape runs 13-25 % faster peeled; merged, the halo is within noise
// of no peel (halo_peel_merged_ab_n1_s5.jsonl).
constexpr uint32_t kPeelItem = 1u << 28; // internal flag bit (never a TEMPI_HIP_ITEM_*)
template <int W> __device__ __forceinline__ void copy_any(const CArgs &a, uint32_t blk, uint32_t nblk) {
  if constexpr (W == 8) {
    if (a.flags & kPeelItem) {
      copy_body_peel(a, blk, nblk);
      return;
    }
  }
  copy_body<W>(a, blk, nblk);
}

template <int W> __global__ __launch_bounds__(kCopyBlock) void copy_kernel(const CArgs a, const Sig sg) {
  copy_any<W>(a, xcd_tile(blockIdx.x, gridDim.x, a.flags), gridDim.x);
  wg_signal(sg, true);
}

constexpr int kCopyMax = int((kBatchBytes - 8) / (sizeof(CArgs) + 4));
struct CBatchArgs {
  uint32_t nitems;
  uint32_t first[kCopyMax + 1];
  CArgs item[kCopyMax];
};

template <int W> __global__ __launch_bounds__(kCopyBlock) void copy_batch_kernel(const CBatchArgs b, const Sig sg) {
  uint32_t lo = 0, hi = b.nitems;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (blockIdx.x >= b.first[mid])
      lo = mid;
    else
      hi = mid;
  }
  const uint32_t n = b.first[lo + 1] - b.first[lo];
  copy_any<W>(b.item[lo], xcd_tile(blockIdx.x - b.first[lo], n, b.item[lo].flags), n); // (within the item)
  wg_signal(sg, true);
}

bool make_side(char *first, const Norm &n, int W, CSide *c) {
  if (n.nd > kCopyND) return false;
  *c = CSide{};
  c->first = first;
  c->wpr = uint32_t(n.block / W);
  c->mwpr = make_magic(c->wpr);
  for (int k = 0; k < kCopyND - 1; ++k) {
    c->cnt[k] = 1;
    c->mcnt[k] = make_magic(1);
  }
  // innermost first into slots 0 .. nd-2; the outermost into the last slot
  for (int k = 0; k < n.nd; ++k) {
    const int src = n.nd - 1 - k;
    if (src == 0) {
      c->stride[kCopyND - 1] = n.str[0];
    } else {
      if (n.cnt[src] >= (int64_t(1) << 32)) return false;
      c->cnt[k] = uint32_t(n.cnt[src]);
      c->mcnt[k] = make_magic(c->cnt[k]);
      c->stride[k] = n.str[src];
    }
  }
  return true;
}

struct CopyJob {
  CArgs a;
  int w; // word width; 0: the peeled copy (16-byte chunks, 8-byte seam halves; launched with W = 8)
};

#ifndef TEMPI_COPY_PEEL
#define TEMPI_COPY_PEEL 1
#endif
// the peeled copy applies: 8-byte words only because both bases sit 8 bytes
// past a 16-byte boundary, every block and stride a multiple of 16
// (TEMPI_COPY_PEEL=0 in the environment turns it off, for A/B runs)
// (TEMPI_COPY_PEEL=2: peeled, with plain loads and stores)
int peel_mode() {
  static const int m = [] {
    const char *e = std::getenv("TEMPI_COPY_PEEL");
    return TEMPI_COPY_PEEL ? (e ? int(std::strtol(e, nullptr, 10)) : 1) : 0;
  }();
  return m;
}
bool peel_enabled() { return peel_mode() != 0; }
bool peel_ok(uintptr_t dst, uintptr_t src, const Norm &nd, const Norm &ns) {
  if (!peel_enabled() || (dst & 15) != 8 || (src & 15) != 8) return false;
  for (const Norm *n : {&nd, &ns}) {
    if (n->block % 16) return false;
    for (int k = 0; k < n->nd; ++k)
      if (n->str[k] % 16) return false;
  }
  return true;
}

// the copy as one kernel item, or false when it needs the pack + unpack route
bool plan_copy(void *dst, const void *src, const tempi_hip_desc *dd, const tempi_hip_desc *sd, CopyJob *job) {
  Norm nd, ns;
  if (!normalise(dd, &nd) || !normalise(sd, &ns)) return false;
  const int64_t bytes = norm_bytes(ns);
  if (bytes != norm_bytes(nd) || bytes >= kMaxLaunchBytes) return false;
  int w = word_width(reinterpret_cast<uintptr_t>(dst), reinterpret_cast<uintptr_t>(src), ns);
  const int wd = word_width(reinterpret_cast<uintptr_t>(dst), reinterpret_cast<uintptr_t>(src), nd);
  if (wd < w) w = wd;
  const bool peel = w == 8 && peel_ok(reinterpret_cast<uintptr_t>(dst), reinterpret_cast<uintptr_t>(src), nd, ns);
  if (!make_side(const_cast<char *>(static_cast<const char *>(src)), ns, w, &job->a.s)) return false;
  if (!make_side(static_cast<char *>(dst), nd, w, &job->a.d)) return false;
  job->a.nwords = uint32_t(bytes / w);
  if (peel) w = 0; // (the sides count 8-byte words, as the peeled body expects; launched with W = 8)
  job->a.flags = xcd_flag(static_cast<char *>(dst), nd, false) | (peel ? kPeelItem : 0u) |
                 (peel && peel_mode() == 2 ? kCopyPlain : 0u);
  job->a.s2 = job->a.d2 = nullptr;
  job->w = w;
  return true;
}

bool same_shape(const CSide &x, const CSide &y) {
  if (x.wpr != y.wpr) return false;
  for (int k = 0; k < kCopyND - 1; ++k)
    if (x.cnt[k] != y.cnt[k]) return false;
  for (int k = 0; k < kCopyND; ++k)
    if (x.stride[k] != y.stride[k]) return false;
  return true;
}

#ifndef TEMPI_COPY_PAIR
#define TEMPI_COPY_PAIR 1
#endif
// pair items of identical shapes (see CArgs::s2); greedy, order-preserving
std::vector<CopyJob> pair_jobs(const std::vector<CopyJob> &in) {
  if (!TEMPI_COPY_PAIR) return in;
  std::vector<CopyJob> out;
  std::vector<char> used(in.size(), 0);
  for (size_t i = 0; i < in.size(); ++i) {
    if (used[i]) continue;
    CopyJob j = in[i];
    for (size_t k = i + 1; k < in.size() && k < i + 64; ++k) {
      if (used[k] || in[k].a.nwords != j.a.nwords || in[k].a.flags != j.a.flags || !same_shape(in[k].a.s, j.a.s) ||
          !same_shape(in[k].a.d, j.a.d))
        continue;
      j.a.s2 = in[k].a.s.first;
      j.a.d2 = in[k].a.d.first;
      used[k] = 1;
      break;
    }
    out.push_back(j);
  }
  return out;
}

uint32_t copy_blocks(const CopyJob &j) {
  const uint64_t tile = j.w ? uint64_t(kCopyBlock) * (16 / j.w) * TEMPI_COPY_U : uint64_t(kCopyBlock);
  const uint64_t units = j.w ? uint64_t(j.a.nwords) : uint64_t(j.a.nwords) / 2 + 1; // (peeled: chunks)
  uint64_t b = (units + tile - 1) / tile;
  if (b > TEMPI_MAX_BLOCKS) b = TEMPI_MAX_BLOCKS;
  return uint32_t(b);
}

// fold: offered to this group's last launch (see run_batch)
template <int W> int launch_copy_group(const std::vector<CopyJob> &jobs, hipStream_t s, tempi_ticket::Fold *fold) {
  CBatchArgs b;
  b.nitems = 0;
  uint32_t total = 0;
  auto flush = [&](bool last) -> int {
    if (!b.nitems) return 0;
    b.first[b.nitems] = total;
    const Sig sg = last && fold ? take_fold_from(fold, total, false) : Sig{};
    if (b.nitems == 1)
      TEMPI_LAUNCH(copy_kernel<W>, dim3(total), dim3(kCopyBlock), 0, s, b.item[0], sg);
    else
      TEMPI_LAUNCH(copy_batch_kernel<W>, dim3(total), dim3(kCopyBlock), 0, s, b, sg);
    b.nitems = 0;
    total = 0;
    return int(hipGetLastError());
  };
  for (const CopyJob &j : jobs) {
    const uint32_t blocks = copy_blocks(j);
    if (!blocks) continue;
    if (uint64_t(total) + blocks >= (uint64_t(1) << 31))
      if (int e = flush(false)) return e;
    b.first[b.nitems] = total;
    b.item[b.nitems] = j.a;
    b.nitems++;
    total += blocks;
    if (b.nitems == uint32_t(kCopyMax))
      if (int e = flush(false)) return e;
  }
  return flush(true);
}

// the copy batch; fold: a completion ticket for its last launch (run_batch)
int copy_batch(const tempi_hip_copy_item *items, int n, void *stream, tempi_ticket::Fold *fold) {
  if (launch_check()) {
    gDesc = "copy batch of " + std::to_string(n) + ":";
    for (int i = 0; i < n; ++i)
      gDesc += " " + describe(items[i].dst, items[i].dst_first, nullptr) + " <- " +
               describe(items[i].src, items[i].src_first, nullptr) +
               ((items[i].flags & TEMPI_HIP_ITEM_REMOTE) ? " remote" : "");
  }
  std::vector<CopyJob> groups[5];
  for (int i = 0; i < n; ++i) {
    CopyJob j;
    if (!plan_copy(items[i].dst_first, items[i].src_first, &items[i].dst, &items[i].src, &j))
      return int(hipErrorInvalidValue);
    j.a.flags |= items[i].flags & TEMPI_HIP_ITEM_REMOTE;
    if (j.a.nwords == 0) continue;
    const int wi = j.w == 1 ? 0 : j.w == 2 ? 1 : j.w == 4 ? 2 : j.w == 8 || j.w == 0 ? 3 : 4;
    groups[wi].push_back(j);
  }
  hipStream_t s = static_cast<hipStream_t>(stream);
  int lastGroup = -1;
  for (int wi = 0; wi < 5; ++wi)
    if (!groups[wi].empty()) lastGroup = wi;
  for (int wi = 0; wi < 5; ++wi) {
    if (groups[wi].empty()) continue;
    tempi_ticket::Fold *f = wi == lastGroup ? fold : nullptr;
    int e = 0;
    switch (wi) {
    case 0: e = launch_copy_group<1>(pair_jobs(groups[wi]), s, f); break;
    case 1: e = launch_copy_group<2>(pair_jobs(groups[wi]), s, f); break;
    case 2: e = launch_copy_group<4>(pair_jobs(groups[wi]), s, f); break;
    case 3: e = launch_copy_group<8>(pair_jobs(groups[wi]), s, f); break;
    default: e = launch_copy_group<16>(pair_jobs(groups[wi]), s, f); break;
    }
    if (e) return e;
  }
  return 0;
}

} // namespace

extern "C" {

int tempi_hip_copy_supported(void *dst_first, const void *src_first, const tempi_hip_desc *dst,
                             const tempi_hip_desc *src) {
  CopyJob j;
  return plan_copy(dst_first, src_first, dst, src, &j) ? 1 : 0;
}

int tempi_hip_copy_word_width(void *dst_first, const void *src_first, const tempi_hip_desc *dst,
                              const tempi_hip_desc *src) {
  CopyJob j;
  return plan_copy(dst_first, src_first, dst, src, &j) ? j.w : -1;
}

int tempi_hip_copy_batch(const tempi_hip_copy_item *items, int n, void *stream) {
  return copy_batch(items, n, stream, nullptr);
}

int tempi_hip_pack(void *packed, const void *first, const tempi_hip_desc *d, void *stream) {
  if (launch_check()) gDesc = "pack " + describe(*d, packed, first);
  Norm n;
  if (!normalise(d, &n)) return int(hipErrorInvalidValue);
  return launch_split(true, static_cast<char *>(packed),
                      const_cast<char *>(static_cast<const char *>(first)), n,
                      static_cast<hipStream_t>(stream));
}

int tempi_hip_unpack(void *first, const void *packed, const tempi_hip_desc *d, void *stream) {
  if (launch_check()) gDesc = "unpack " + describe(*d, first, packed);
  Norm n;
  if (!normalise(d, &n)) return int(hipErrorInvalidValue);
  return launch_split(false, const_cast<char *>(static_cast<const char *>(packed)),
                      static_cast<char *>(first), n, static_cast<hipStream_t>(stream));
}

} // extern "C"

namespace {
// pack / unpack + a completion ticket: folded into the work kernel when the
// work is one launch of at most fold_max_blocks() workgroups, else the ticket
// kernel queued behind it. The mutex keeps tickets and folded counts in
// launch order on the stream.
int with_ticket(bool pack, char *packed, char *first, const tempi_hip_desc *d, hipStream_t s, const uint32_t **flag,
                uint32_t *ticket) {
  if (launch_check()) gDesc = std::string(pack ? "pack " : "unpack ") + "(ticket) " + describe(*d, packed, first);
  Norm n;
  if (!normalise(d, &n)) return int(hipErrorInvalidValue);
  bool single = norm_bytes(n) < kMaxLaunchBytes; // launch_split makes exactly one launch
  for (int k = 0; k < n.nd; ++k) single &= n.cnt[k] < (int64_t(1) << 32);
  std::lock_guard<std::mutex> lock(tempi_ticket::mutex());
  tempi_ticket::Ticket *t = tempi_ticket::of(s);
  if (!t) return int(hipErrorOutOfMemory);
  tempi_ticket::Fold fold;
  fold.t = t;
  fold.ticket = ++t->next;
  fold.max_blocks = single ? tempi_ticket::fold_max_blocks() : 0;
  fold.max_blocks_wt = single ? tempi_ticket::fold_max_blocks_wt() : 0;
  gFold = &fold;
  const int e = launch_split(pack, packed, first, n, s);
  gFold = nullptr;
  if (e) {
    if (fold.taken) t->broken = true; // the host counted a launch that never ran
    return e;
  }
  *flag = t->host;
  *ticket = fold.ticket;
  if (fold.taken) tempi_ticket::stats().folded++;
  return fold.taken ? 0 : int(tempi_ticket::queue_kernel(*t, s, fold.ticket));
}
// A batch with a completion ticket folded into its last launch (run_batch,
// copy_batch). When that launch is too large to fold, *flag stays NULL and
// the caller waits as it would without a ticket: a batch never costs a
// second launch (a queued ticket kernel per batch made the halo 1-3 %
// slower, round 2).
template <typename F> int batch_with_ticket(hipStream_t s, const uint32_t **flag, uint32_t *ticket, F &&run) {
  *flag = nullptr;
  *ticket = 0;
  std::lock_guard<std::mutex> lock(tempi_ticket::mutex());
  tempi_ticket::Ticket *t = tempi_ticket::of(s);
  if (!t) return run(nullptr);
  tempi_ticket::Fold fold;
  fold.t = t;
  fold.ticket = t->next + 1; // issued only if a launch takes it
  fold.max_blocks = tempi_ticket::fold_max_blocks();
  fold.max_blocks_wt = tempi_ticket::fold_max_blocks_wt();
  const int e = run(&fold);
  if (e) {
    if (fold.taken) t->broken = true; // the host counted a launch that may never run
    return e;
  }
  if (fold.taken) {
    t->next = fold.ticket;
    *flag = t->host;
    *ticket = fold.ticket;
    tempi_ticket::stats().folded++;
  }
  return 0;
}

// ------------------------------------------------------------ resident packer
//
// A synchronous MPI_Pack / MPI_Unpack of a small object (config 1: 512 KiB)
// was ~9 us, of which the kernel's gather is ~2: hipLaunchKernel 2.2-3.0 us,
// dispatch 2.2-2.6 before a wave runs, one-way visibility of the completion
// 1.2-1.35. The reference pays the same (a launch and a
// cudaStreamSynchronize: /root/reference/src/internal/packer_2d.cu:101-118).
// Here no launch is made per call: a kernel stays RESIDENT while calls keep
// coming. The host writes the request into pinned host memory; the kernel's
// leader wave polls it over the host link and hands it to the worker
// workgroups through device memory; each worker invalidates its caches (an
// acquire: the object may have been written by any other kernel, copy or the
// host since it last looked) and runs the same gather / scatter body as the
// launched kernels (pack_body / unpack_body, grid-stride over the workers);
// the last worker to finish stores the completion to pinned host memory.
// Measured on MI355X (tools/resident.hip, profiles/r06/resident_proto_s15.jsonl):
// 5.1 us per config-1 call against 9.2 through a launch.
//
// Records are 64 tagged 8-byte granules {data dword, sequence number}: one
// wave-wide load reads a whole record, and it is complete when every lane's
// tag is the number expected -- no separate flag, no ordering between the
// granule stores. Completion is the ticket fold (ticket.hpp): workers count
// themselves on kShards shard counters, the last of a shard on the top
// counter, the last of all stores the sequence number; the host keeps the
// counts and puts each request's targets in its record.
//
// Lifetime: the server is launched by the first call that can use it (that
// call pays about a launch, as before) on a stream of its own, and leaves after
// TEMPI_RESIDENT_IDLE_US (default 200) without a request, after 2 s in any
// case, or on an EXIT request (MPI_Finalize). Every wave has a bounded exit:
// the leader hands the workers an EXIT record as it leaves, and workers leave
// on that record alone (or 1 ms past the 2 s cap). A leader leaving stores the
// first sequence number it did not serve; a request that crossed its exit is
// posted again to a new instance (stream order puts the new one behind the
// old). A server that ended with a request neither served nor refused has its
// counters reset and the request posted again: packs and unpacks are
// idempotent. The server runs only between calls of a burst: an
// application's hipDeviceSynchronize may wait up to the idle time for it.
//
// The hand-off slot holds one record, so the leader overwrites it (with the
// next request or EXIT) only once every worker has counted itself on
// Dev::seen for the record there: a worker preempted or dispatched late would
// otherwise find a later tag than the one it waits for and sit out the cap,
// while a request that needed it never completed (four processes
// time-slicing one GPU: profiles/r06/NOTES.md s36). A worker counts itself
// right after its part of the completion, long before the host has seen the
// completion and posted the next request, so the leader's check (a load kept
// in flight beside its polls) costs a call nothing.
//
// Taken: single descriptors of <= 3 dims, at most TEMPI_RESIDENT_MAX_BYTES
// (default 2 MiB; 1- and 2-byte words TEMPI_RESIDENT_NARROW_MAX_BYTES, default
// 256 KiB: beyond, their interleaved / dense launches win), not under
// TEMPI_LAUNCH_CHECK. TEMPI_RESIDENT=0 (or
// tempi_hip_resident_enable(0)) turns it off.
namespace resident {
using tempi_ticket::kCounterStride;
using tempi_ticket::kShards;
constexpr uint32_t kOpPack = 1, kOpUnpack = 2, kOpExit = 3;
constexpr int kGranules = 64; // one per lane of a wave
// data dwords of a record
constexpr int kOp = 0;         // op | W << 8 | ND << 16 | kAgentAcquire
constexpr uint32_t kAgentAcquire = 1u << 24; // (A/B: TEMPI_RESIDENT_ACQUIRE=agent)
constexpr uint32_t kStamp = 1u << 25;        // (diagnostic: TEMPI_RESIDENT_STAMPS=1, Dev::stamp)
constexpr int kWorkers = 1;    // workers taking part (a multiple of kShards)
constexpr int kArgs = 2;       // KArgs<ND> (8-byte aligned)
constexpr int kLastWorker = 40;  // the worker holding the object's last chunk when it is partial (else ~0)
constexpr int kReleaseAll = 41;  // every worker stored through L2 (not write-through)
constexpr int kReleaseFirst = 42; // the first chunk is partial (worker 0 holds it)
constexpr int kTargets = 43;     // the shard counters' targets, then the top counter's
static_assert(kArgs * 4 + sizeof(KArgs<3>) <= kLastWorker * 4, "record layout");
static_assert(kTargets + kShards + 1 <= kGranules, "record layout");
constexpr uint64_t kTicksPerUs = 100; // wall_clock64 (s_memrealtime): 100 MHz
// chunks a lane has in flight per pass (A/B, profiles/r06/resident_u_ab_s19.jsonl:
// 1, 2 and 4 within noise of each other at config 1)
#ifndef TEMPI_RESIDENT_U
#define TEMPI_RESIDENT_U 1
#endif
constexpr int kResidentU = TEMPI_RESIDENT_U;
// one completion counter for all workers (a request has at most a few
// hundred) instead of the launched kernels' sharded fold: one atomic on the
// path instead of two, no slower in the A/B
#ifndef TEMPI_RESIDENT_FLAT
#define TEMPI_RESIDENT_FLAT 1
#endif
constexpr bool kResidentFlat = TEMPI_RESIDENT_FLAT != 0;
constexpr uint64_t kGrace = 1000 * kTicksPerUs;
// a fresh instance waits at least this long for its first request: the call
// that launched it posts right after the launch, and a host thread
// descheduled in between must not see its request refused twice (the call
// would then launch after all)
constexpr uint64_t kFirstIdle = 100 * kTicksPerUs;

struct Mail {                 // pinned, coherent, mapped host memory
  uint64_t req[kGranules];    // the request, tagged with its sequence number
  uint32_t done;              // the last request served
  uint32_t pad0[31];
  uint32_t exitw;             // the first request an exiting server left unserved
  uint32_t pad1[31];
};
struct Dev {                  // device memory, zeroed once
  uint64_t bcast[kGranules];  // the leader's hand-off to the workers
  uint32_t counter[(kShards + 1) * kCounterStride];
  // wall_clock64 of the last stamped request: the leader saw it; worker 0 saw
  // the hand-off, finished its acquire, finished its body; the completing
  // worker stored the completion
  uint64_t stamp[8];
  // records read, summed over the workers (a line of its own: one atomic per
  // worker and request, none of them on a call's path)
  uint32_t seen[32];
};

template <bool PACK, int W, int ND>
__device__ __forceinline__ void serve(const uint32_t *rec, uint32_t w, uint32_t nw) {
  KArgs<ND> a;
  __builtin_memcpy(&a, rec + kArgs, sizeof a);
  if constexpr (PACK)
    pack_body<W, ND, true, kResidentU>(a, w, nw);
  else
    unpack_body<W, ND, W == 16, kResidentU>(a, w, nw);
}

template <bool PACK, int W> __device__ __forceinline__ void serve_nd(uint32_t nd, const uint32_t *rec, uint32_t w,
                                                                    uint32_t nw) {
  switch (nd) {
  case 0: return serve<PACK, W, 0>(rec, w, nw);
  case 1: return serve<PACK, W, 1>(rec, w, nw);
  case 2: return serve<PACK, W, 2>(rec, w, nw);
  default: return serve<PACK, W, 3>(rec, w, nw);
  }
}

template <bool PACK> __device__ __forceinline__ void serve_w(uint32_t op, const uint32_t *rec, uint32_t w,
                                                            uint32_t nw) {
  const uint32_t W = (op >> 8) & 31, nd = (op >> 16) & 7;
  if (W == 16)
    serve_nd<PACK, 16>(nd, rec, w, nw);
  else if (W == 8)
    serve_nd<PACK, 8>(nd, rec, w, nw);
  else if (W == 4)
    serve_nd<PACK, 4>(nd, rec, w, nw);
  else if (W == 2)
    serve_nd<PACK, 2>(nd, rec, w, nw);
  else
    serve_nd<PACK, 1>(nd, rec, w, nw);
}

// block 0: the leader (one wave); blocks 1 .. gridDim.x - 1: the workers
__global__ __launch_bounds__(kBlock) void server_kernel(Mail *m, Dev *dv, uint32_t firstSeq, uint64_t idle,
                                                        uint64_t cap) {
  __shared__ __attribute__((aligned(16))) uint32_t rec[kGranules];
  const uint64_t t0 = wall_clock64();
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t expect = firstSeq;
  uint64_t last = t0;
  if (blockIdx.x == 0) {
    if (wave) return;
    // two polls of the host link in flight, so a request is seen about half
    // a round trip sooner; a poll older than the request it overlapped holds
    // an old tag and is passed over (four: no gain)
    bool leave = false;
    const uint32_t nWorkers = gridDim.x - 1;
    auto seen = [&]() { return __hip_atomic_load(&dv->seen[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    const uint32_t seen0 = seen(); // (the previous instance has ended: stream order)
    uint32_t handed = 0;           // records this leader handed out
    // every worker has read the record in the slot (s: a recent Dev::seen);
    // else wait for them, up to the cap
    auto all_read = [&](uint32_t s) {
      while (s - seen0 != handed * nWorkers) {
        if (int64_t(wall_clock64() - t0) > int64_t(cap)) return false;
        __builtin_amdgcn_s_sleep(1);
        s = seen();
      }
      return true;
    };
    auto take = [&](uint64_t g, uint32_t s) {
      if (__ballot(uint32_t(g >> 32) == expect) != ~0ull) return;
      leave = true;
      if (!all_read(s)) return; // (past the cap: left unserved, so posted again)
      const uint32_t op = __shfl(uint32_t(g), 0);
      if ((op & kStamp) && lane == 0) dv->stamp[0] = wall_clock64();
      __hip_atomic_store(&dv->bcast[lane], g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      ++expect;
      ++handed;
      last = wall_clock64();
      leave = (op & 3) == kOpExit;
    };
    auto poll = [&]() { return __hip_atomic_load(&m->req[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); };
    // each poll travels with a load of Dev::seen issued just after it, so
    // the count a request is checked against left no earlier than the poll
    uint64_t ga = poll();
    uint32_t sa = seen();
    for (;;) {
      const uint64_t gb = poll();
      const uint32_t sb = seen();
      take(ga, sa);
      if (leave) break;
      ga = poll();
      sa = seen();
      take(gb, sb);
      if (leave) break;
      const uint64_t now = wall_clock64();
      // (signed: a wave restored onto another XCD after a preemption reads
      // another XCD's clock, which may be behind the one it last read)
      const uint64_t limit = handed || idle >= kFirstIdle ? idle : kFirstIdle;
      if (int64_t(now - last) > int64_t(limit) || int64_t(now - t0) > int64_t(cap)) {
        // one fresh poll first: a request posted as the idle time ran out is
        // served, not refused (a refusal costs its call a launch)
        const uint32_t before = expect;
        const uint64_t g = poll();
        take(g, seen());
        if (leave) break;
        if (expect != before) continue;
        if (all_read(seen())) // (else past the cap: workers leave on theirs)
          __hip_atomic_store(&dv->bcast[lane], (uint64_t(expect) << 32) | (lane == 0 ? kOpExit : 0u),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_store(&m->exitw, expect, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  const uint32_t w = blockIdx.x - 1;
  for (;;) {
    if (wave == 0) {
      uint32_t d;
      for (;;) {
        const uint64_t g = __hip_atomic_load(&dv->bcast[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__ballot(uint32_t(g >> 32) == expect) == ~0ull) {
          d = uint32_t(g);
          break;
        }
        const uint64_t now = wall_clock64();
        // workers leave on the leader's EXIT record alone: one that left on a
        // clock of its own could miss a request the leader then hands out.
        // The cap is only the bound every wave reaches, a grace period after
        // the leader's own
        if (int64_t(now - t0) > int64_t(cap + kGrace)) {
          d = lane == 0 ? kOpExit : 0u;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      rec[lane] = d;
    }
    __syncthreads();
    const uint32_t op = rec[kOp], nw = rec[kWorkers], seq = expect;
    if ((op & 3) == kOpExit) return;
    ++expect;
    if (w < nw) {
      const bool stamp = (op & kStamp) && w == 0 && threadIdx.x == 0;
      if (stamp) dv->stamp[1] = wall_clock64();
      // acquire: nothing this CU cached before the request may be read
      if (threadIdx.x == 0) {
        if (op & kAgentAcquire)
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        else
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (stamp) dv->stamp[2] = wall_clock64();
      if ((op & 3) == kOpPack)
        serve_w<true>(op, rec, w, nw);
      else
        serve_w<false>(op, rec, w, nw);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (stamp) dv->stamp[3] = wall_clock64();
      if (threadIdx.x == 0) {
        // workers that stored through L2 (partial first / last chunks, scatters
        // of narrower words) write it back first (as wg_signal; an L2
        // write-back costs ~1.5 us on the call's path, so only those)
        if (rec[kReleaseAll] || (w == 0 && rec[kReleaseFirst]) || w == rec[kLastWorker]) {
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        const uint32_t k = kResidentFlat ? 0u : w % kShards;
        // (device counters only the GPU touches: agent scope)
        const uint32_t old = __hip_atomic_fetch_add(dv->counter + k * kCounterStride, 1u, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
        if (old + 1u == rec[kTargets + k]) {
          const uint32_t top = kResidentFlat ? 0u
                                             : __hip_atomic_fetch_add(dv->counter + kShards * kCounterStride, 1u,
                                                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (kResidentFlat || top + 1u == rec[kTargets + kShards]) {
            if (op & kStamp) dv->stamp[4] = wall_clock64();
            __hip_atomic_store(&m->done, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          }
        }
      }
    }
    // this worker is done with the record: the leader may overwrite it
    if (threadIdx.x == 0) __hip_atomic_fetch_add(&dv->seen[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = wall_clock64();
    __syncthreads(); // (every wave has read the record before wave 0 writes the next)
  }
}

bool env_flag(const char *name, bool dflt) {
  const char *e = std::getenv(name);
  return e ? std::strtol(e, nullptr, 10) != 0 : dflt;
}
int64_t env_int(const char *name, int64_t dflt) {
  const char *e = std::getenv(name);
  return e ? int64_t(std::strtoll(e, nullptr, 10)) : dflt;
}
std::atomic<int> &switched_on() { // TEMPI_RESIDENT, then tempi_hip_resident_enable
  static std::atomic<int> v{env_flag("TEMPI_RESIDENT", true) ? 1 : 0};
  return v;
}
bool enabled() { return switched_on().load(std::memory_order_relaxed) != 0; }
int64_t max_bytes() {
  static const int64_t v = env_int("TEMPI_RESIDENT_MAX_BYTES", int64_t(2) << 20);
  return v;
}
int64_t narrow_max_bytes() {
  static const int64_t v = env_int("TEMPI_RESIDENT_NARROW_MAX_BYTES", int64_t(256) << 10);
  return v;
}
// workers of a server: a multiple of kShards (a request takes up to all of them)
uint32_t workers() {
  static const uint32_t v = [] {
    int64_t n = env_int("TEMPI_RESIDENT_WORKERS", 96);
    n = n < kShards ? kShards : (n > 1024 ? 1024 : n);
    return uint32_t(n / kShards * kShards);
  }();
  return v;
}
uint64_t idle_ticks() {
  static const uint64_t v = uint64_t(std::max<int64_t>(env_int("TEMPI_RESIDENT_IDLE_US", 200), 1)) * kTicksPerUs;
  return v;
}
constexpr uint64_t kCapTicks = uint64_t(2000000) * kTicksPerUs; // 2 s
bool stamps() {
  static const bool v = env_flag("TEMPI_RESIDENT_STAMPS", false);
  return v;
}
bool agent_acquire() {
  static const bool v = [] {
    const char *e = std::getenv("TEMPI_RESIDENT_ACQUIRE");
    return e && std::strcmp(e, "agent") == 0;
  }();
  return v;
}

struct Server {
  bool ready = false, broken = false, running = false;
  hipStream_t stream = nullptr;
  Mail *host = nullptr, *mapped = nullptr;
  Dev *dev = nullptr;
  uint32_t seq = 0;                   // the last request posted
  uint32_t counted[kShards + 1] = {}; // the host's totals of the device counters
};
struct Stats {
  uint64_t served = 0, launches = 0, reposts = 0, lost = 0;
};
std::mutex &mutex() {
  static std::mutex m;
  return m;
}
Stats &stats() {
  static Stats s;
  return s;
}
constexpr int kMaxServers = 64; // devices a process may have a server on
Server &server(int device) {
  static Server s[kMaxServers];
  return s[device];
}

bool ready(Server &sv) {
  if (sv.ready || sv.broken) return sv.ready;
  void *h = nullptr, *d = nullptr, *dv = nullptr;
  // A kernel that stays running holds its hardware queue: any stream HIP maps
  // onto the same queue (at most GPU_MAX_HW_QUEUES = 4 per process) waits
  // behind it. Made at normal priority after TEMPI's streams, the server's
  // stream shared the null stream's queue (a kernel there waited out the
  // server); at high priority it shared none of the process's streams
  // (tools/queue_probe.hip, profiles/r06/queue_probe_s30.jsonl).
  int least = 0, greatest = 0;
  hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest);
  if (e == hipSuccess) e = hipStreamCreateWithPriority(&sv.stream, hipStreamNonBlocking, greatest);
  if (e == hipSuccess) e = hipHostMalloc(&h, sizeof(Mail), hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable);
  if (e == hipSuccess) e = hipHostGetDevicePointer(&d, h, 0);
  if (e == hipSuccess) e = hipMalloc(&dv, sizeof(Dev));
  if (e == hipSuccess) e = hipMemsetAsync(dv, 0, sizeof(Dev), sv.stream);
  if (e == hipSuccess) e = hipStreamSynchronize(sv.stream);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    if (dv) (void)hipFree(dv);
    if (h) (void)hipHostFree(h);
    if (sv.stream) (void)hipStreamDestroy(sv.stream);
    sv.stream = nullptr;
    (void)hipGetLastError();
    sv.broken = true;
    return false;
  }
  std::memset(h, 0, sizeof(Mail));
  sv.host = static_cast<Mail *>(h);
  sv.mapped = static_cast<Mail *>(d);
  sv.dev = static_cast<Dev *>(dv);
  sv.ready = true;
  return true;
}

void post(Server &sv, uint32_t seq, const uint32_t *d) {
  for (int i = 0; i < kGranules; ++i)
    __atomic_store_n(&sv.host->req[i], (uint64_t(seq) << 32) | d[i], __ATOMIC_RELAXED);
}

// 0: served; 1: the server left without serving it; 2: the server ended
// with it neither served nor refused; else a HIP error
int wait(Server &sv, uint32_t seq) {
  for (uint32_t spins = 1;; ++spins) {
    if (__atomic_load_n(&sv.host->done, __ATOMIC_ACQUIRE) == seq) return 0;
    if (__atomic_load_n(&sv.host->exitw, __ATOMIC_ACQUIRE) == seq) return 1;
    if ((spins & 1023) == 0) { // ~20 us of pause loops: a faulted server ends the wait
      const hipError_t e = hipStreamQuery(sv.stream);
      if (e == hipSuccess) { // ended: its last stores are visible now
        if (__atomic_load_n(&sv.host->done, __ATOMIC_ACQUIRE) == seq) return 0;
        if (__atomic_load_n(&sv.host->exitw, __ATOMIC_ACQUIRE) == seq) return 1;
        return 2;
      }
      if (e != hipErrorNotReady) return int(e);
      (void)hipGetLastError();
    }
    __builtin_ia32_pause();
  }
}

template <int W, int ND>
void make_record(bool pack, char *packed, char *first, const Norm &n, uint32_t *d) {
  KArgs<ND> a;
  uint32_t blocks;
  make_args<W, ND>(packed, first, n, &a, &blocks);
  if (pack || (W == 16 && scatter_write_through(n))) a.flags |= kWriteThrough;
  constexpr uint32_t tile = uint32_t(kBlock) * kResidentU; // chunks per worker step
  const uint32_t tiles = (a.nchunks + tile - 1) / tile;
  uint32_t nw = std::min<uint32_t>(workers(), (tiles + kShards - 1) / kShards * kShards);
  d[kOp] = (pack ? kOpPack : kOpUnpack) | uint32_t(W) << 8 | uint32_t(ND) << 16 | (agent_acquire() ? kAgentAcquire : 0u) |
             (stamps() ? kStamp : 0u);
  d[kWorkers] = nw;
  std::memcpy(d + kArgs, &a, sizeof a);
  constexpr uint32_t CW = 16 / W;
  const bool tailPartial = (uint64_t(a.head) + a.nwords) % CW != 0;
  d[kLastWorker] = tailPartial ? (tiles - 1) % nw : ~0u;
  d[kReleaseAll] = (a.flags & kWriteThrough) ? 0u : 1u;
  d[kReleaseFirst] = a.head != 0 ? 1u : 0u;
}

template <int W>
void make_record_w(bool pack, char *packed, char *first, const Norm &n, uint32_t *d) {
  switch (n.nd) {
  case 0: return make_record<W, 0>(pack, packed, first, n, d);
  case 1: return make_record<W, 1>(pack, packed, first, n, d);
  case 2: return make_record<W, 2>(pack, packed, first, n, d);
  default: return make_record<W, 3>(pack, packed, first, n, d);
  }
}

// serve one synchronous pack / unpack; *served = false: not taken (the caller
// launches as before)
int run_inner(bool pack, char *packed, char *first, const Norm &n, hipStream_t s, bool *served);
// (TEMPI_RESIDENT_DEBUG=1: report a HIP error the call left behind)
int run(bool pack, char *packed, char *first, const Norm &n, hipStream_t s, bool *served) {
  static const bool debug = env_flag("TEMPI_RESIDENT_DEBUG", false);
  const hipError_t pre = debug ? hipPeekAtLastError() : hipSuccess;
  const int e = run_inner(pack, packed, first, n, s, served);
  if (debug) {
    const hipError_t post = hipPeekAtLastError();
    if (post != hipSuccess)
      std::fprintf(stderr, "[resident] pid %d: HIP error %s (%d) pending after a call (before: %s), rc %d served %d, "
                   "%d dims, block %lld\n", int(getpid()), hipGetErrorString(post), int(post),
                   hipGetErrorString(pre), e, int(*served), n.nd, (long long)n.block);
  }
  return e;
}
int run_inner(bool pack, char *packed, char *first, const Norm &n, hipStream_t s, bool *served) {
  *served = false;
  if (!enabled() || launch_check() || n.nd > 3) return 0;
  const int64_t bytes = norm_bytes(n);
  if (bytes == 0 || bytes > max_bytes()) return 0;
  for (int k = 0; k < n.nd; ++k)
    if (n.cnt[k] >= (int64_t(1) << 32)) return 0;
  // 1- and 2-byte words move at a fraction of the rate on the chunk-per-lane
  // body (their launched kernels interleave through LDS): only small objects
  const int w = word_width(reinterpret_cast<uintptr_t>(packed), reinterpret_cast<uintptr_t>(first), n);
  if (w < 4 && bytes > narrow_max_bytes()) return 0;
  // (no order with TEMPI's earlier work on `s` is needed: a synchronous call
  // waited for its own, and an MPI_Isend / MPI_Irecv still in flight may not
  // share a buffer this call writes -- MPI's rule for the application --
  // while readers of one buffer do not conflict. HIP reports a stream busy for
  // ~5 us after a launched call's ticket is seen, so waiting for it here would
  // hand every call of a burst to a launch.)
  (void)s;
  int device = 0;
  if (hipGetDevice(&device) != hipSuccess || device < 0 || device >= kMaxServers) return 0;
  std::lock_guard<std::mutex> lock(mutex());
  Server &sv = server(device);
  if (!ready(sv)) return 0;
  uint32_t d[kGranules] = {};
  switch (w) {
  case 16: make_record_w<16>(pack, packed, first, n, d); break;
  case 8: make_record_w<8>(pack, packed, first, n, d); break;
  case 4: make_record_w<4>(pack, packed, first, n, d); break;
  case 2: make_record_w<2>(pack, packed, first, n, d); break;
  default: make_record_w<1>(pack, packed, first, n, d); break;
  }
  const uint32_t perShard = kResidentFlat ? 0u : d[kWorkers] / kShards;
  for (int k = 0; k < kShards; ++k) d[kTargets + k] = sv.counted[k] + perShard;
  d[kTargets + kShards] = sv.counted[kShards] + (kResidentFlat ? 0u : uint32_t(kShards));
  if (kResidentFlat) d[kTargets] = sv.counted[0] + d[kWorkers];
  for (int attempt = 0; attempt < 2; ++attempt) {
    if (!sv.running) {
      hipLaunchKernelGGL(server_kernel, dim3(1 + workers()), dim3(kBlock), 0, sv.stream, sv.mapped, sv.dev,
                         sv.seq + 1, idle_ticks(), kCapTicks);
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) return int(e);
      sv.running = true;
      stats().launches++;
    }
    const uint32_t seq = ++sv.seq;
    post(sv, seq, d);
    const int r = wait(sv, seq);
    if (r == 0) {
      for (int k = 0; k <= kShards; ++k) sv.counted[k] = d[kTargets + k];
      stats().served++;
      *served = true;
      return 0;
    }
    sv.running = false;
    if (r == 2) { // workers may have counted part of it: start the counts again
      stats().lost++;
      hipError_t e = hipMemsetAsync(sv.dev->counter, 0, sizeof(sv.dev->counter), sv.stream);
      if (e == hipSuccess) e = hipStreamSynchronize(sv.stream);
      if (e != hipSuccess) {
        (void)hipGetLastError();
        sv.broken = true;
        return int(e);
      }
      for (uint32_t &c : sv.counted) c = 0;
      for (int k = 0; k < kShards; ++k) d[kTargets + k] = perShard;
      d[kTargets + kShards] = kResidentFlat ? 0u : uint32_t(kShards);
      if (kResidentFlat) d[kTargets] = d[kWorkers];
    } else if (r != 1) { // a fault: the counters are unknown from here on
      sv.broken = true;
      return r;
    }
    stats().reposts++; // it crossed the server's exit: post it to a new one
  }
  return 0;
}

// MPI_Finalize: an EXIT request to every running server, then its stream drains
void stop_all() {
  std::lock_guard<std::mutex> lock(mutex());
  for (int dv = 0; dv < kMaxServers; ++dv) {
    Server &sv = server(dv);
    if (!sv.ready || !sv.running) continue;
    uint32_t d[kGranules] = {};
    d[kOp] = kOpExit;
    post(sv, ++sv.seq, d);
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(dv);
    (void)hipStreamSynchronize(sv.stream);
    (void)hipSetDevice(cur);
    (void)hipGetLastError();
    sv.running = false;
  }
}
} // namespace resident

} // namespace

extern "C" {

int tempi_hip_pack_ticket(void *packed, const void *first, const tempi_hip_desc *d, void *stream,
                          const uint32_t **flag, uint32_t *ticket) {
  return with_ticket(true, static_cast<char *>(packed), const_cast<char *>(static_cast<const char *>(first)), d,
                     static_cast<hipStream_t>(stream), flag, ticket);
}

int tempi_hip_unpack_ticket(void *first, const void *packed, const tempi_hip_desc *d, void *stream,
                            const uint32_t **flag, uint32_t *ticket) {
  return with_ticket(false, const_cast<char *>(static_cast<const char *>(packed)), static_cast<char *>(first), d,
                     static_cast<hipStream_t>(stream), flag, ticket);
}

int tempi_hip_pack_batch_ticket(const tempi_hip_batch_item *items, int n, void *stream, const uint32_t **flag,
                                uint32_t *ticket) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  return batch_with_ticket(s, flag, ticket, [&](tempi_ticket::Fold *f) { return run_batch(true, items, n, s, f); });
}

int tempi_hip_unpack_batch_ticket(const tempi_hip_batch_item *items, int n, void *stream, const uint32_t **flag,
                                  uint32_t *ticket) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  return batch_with_ticket(s, flag, ticket, [&](tempi_ticket::Fold *f) { return run_batch(false, items, n, s, f); });
}

int tempi_hip_copy_batch_ticket(const tempi_hip_copy_item *items, int n, void *stream, const uint32_t **flag,
                                uint32_t *ticket) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  return batch_with_ticket(s, flag, ticket, [&](tempi_ticket::Fold *f) { return copy_batch(items, n, stream, f); });
}

int tempi_hip_pack_resident(void *packed, const void *first, const tempi_hip_desc *d, void *stream, int *served) {
  *served = 0;
  Norm n;
  if (!normalise(d, &n)) return int(hipErrorInvalidValue);
  bool s = false;
  const int e = resident::run(true, static_cast<char *>(packed), const_cast<char *>(static_cast<const char *>(first)),
                              n, static_cast<hipStream_t>(stream), &s);
  *served = s ? 1 : 0;
  return e;
}

int tempi_hip_unpack_resident(void *first, const void *packed, const tempi_hip_desc *d, void *stream, int *served) {
  *served = 0;
  Norm n;
  if (!normalise(d, &n)) return int(hipErrorInvalidValue);
  bool s = false;
  const int e = resident::run(false, const_cast<char *>(static_cast<const char *>(packed)), static_cast<char *>(first),
                              n, static_cast<hipStream_t>(stream), &s);
  *served = s ? 1 : 0;
  return e;
}

void tempi_hip_resident_stats(uint64_t *served, uint64_t *launches, uint64_t *reposts) {
  std::lock_guard<std::mutex> lock(resident::mutex());
  if (served) *served = resident::stats().served;
  if (launches) *launches = resident::stats().launches;
  if (reposts) *reposts = resident::stats().reposts;
}

uint64_t tempi_hip_resident_lost(void) {
  std::lock_guard<std::mutex> lock(resident::mutex());
  return resident::stats().lost;
}

void tempi_hip_resident_stop(void) { resident::stop_all(); }

int tempi_hip_resident_enable(int on) { return resident::switched_on().exchange(on ? 1 : 0); }

int tempi_hip_resident_stamps(uint64_t *out) {
  int device = 0;
  hipError_t e = hipGetDevice(&device);
  if (e == hipSuccess && (device < 0 || device >= resident::kMaxServers)) e = hipErrorInvalidDevice;
  if (e != hipSuccess) return int(e);
  std::lock_guard<std::mutex> lock(resident::mutex());
  resident::Server &sv = resident::server(device);
  if (e == hipSuccess && !sv.ready) e = hipErrorNotReady;
  if (e == hipSuccess) e = hipMemcpy(out, sv.dev->stamp, 5 * sizeof(uint64_t), hipMemcpyDeviceToHost);
  return int(e);
}

int tempi_hip_pack_batch(const tempi_hip_batch_item *items, int n, void *stream) {
  return run_batch(true, items, n, static_cast<hipStream_t>(stream));
}

int tempi_hip_unpack_batch(const tempi_hip_batch_item *items, int n, void *stream) {
  return run_batch(false, items, n, static_cast<hipStream_t>(stream));
}

int64_t tempi_hip_desc_bytes(const tempi_hip_desc *d) {
  Norm n;
  if (!normalise(d, &n)) return -1;
  return norm_bytes(n);
}

int tempi_hip_word_width(const void *packed, const void *first, const tempi_hip_desc *d) {
  Norm n;
  if (!normalise(d, &n)) return -1;
  return word_width(reinterpret_cast<uintptr_t>(packed), reinterpret_cast<uintptr_t>(first), n);
}

} // extern "C"
