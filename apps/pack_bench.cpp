// apps/pack_bench.cpp -- the reference's two packer-level benchmarks, at the
// C-ABI boundary (include/tempi_hip.h), without MPI:
//
//   bench_pack (/root/reference/bin/bench_pack.cpp:28-86, 103-262): 2D byte
//     vectors of `target` packed bytes, rows of 1-256 B at a 512-B stride,
//     targets 64 B - 4 MiB; pack and unpack through the packer with the packed
//     side in pinned mapped host memory ("oneshot": the kernel writes host
//     memory across PCIe) or in device memory ("device"). Wall time of one
//     synchronous call (launch + stream synchronise), trimean over ITERS.
//   bench_pack_kernels (/root/reference/bin/bench_pack_kernels.cu:28-113,
//     120-190): targets 1 KiB and 1 MiB, count 1 and 2 objects of extent
//     (rows - 1) * stride + block laid end to end, strides 16 and 256, rows
//     of 1-256 B; the pack kernel alone, timed with HIP events around the
//     launch, trimean of 30, packed side device or pinned host. (The
//     reference divides event milliseconds by 1024; times here
//     are in microseconds.)
//
// Strided byte i holds i & 0xFF (a fill kernel); the first pack of every
// point is checked byte for byte against the type map, and the first unpack
// is read back and checked in the same way.
//
// usage: pack_bench [ITERS] [--packer] [--kernels] [--max-target BYTES]
//        one JSON object per point on stdout
#include <hip/hip_runtime.h>

#include "tempi_hip.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace {

#define CK(x)                                                                                      \
  do {                                                                                             \
    int e_ = (x);                                                                                  \
    if (e_) {                                                                                      \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, tempi_hip_error_string(e_));  \
      std::exit(2);                                                                                \
    }                                                                                              \
  } while (0)

__global__ void fill_pattern(unsigned char *p, size_t n) {
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
    p[i] = (unsigned char)(i & 0xFF);
}

double trimean(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  auto pct = [&](double p) {
    const double idx = p * double(v.size() - 1);
    const size_t lo = size_t(std::floor(idx)), hi = size_t(std::ceil(idx));
    return v[lo] + (v[hi] - v[lo]) * (idx - double(lo));
  };
  return (pct(0.25) + 2 * pct(0.5) + pct(0.75)) / 4;
}

// one 2D object shape: `count` elements `ext` bytes apart, each `rows` rows
// of `block` bytes `stride` apart
struct Shape {
  int64_t rows, block, stride, count, ext;
  tempi_hip_desc desc() const {
    tempi_hip_desc d{};
    d.block = block;
    d.ndims = 2;
    d.counts[0] = count;
    d.strides[0] = ext;
    d.counts[1] = rows;
    d.strides[1] = stride;
    return d;
  }
  int64_t packed() const { return rows * block * count; }
  int64_t span() const { return (count - 1) * ext + (rows - 1) * stride + block; }
  // strided offset of packed byte k
  int64_t offset(int64_t k) const {
    const int64_t e = k / (rows * block), r = (k / block) % rows, b = k % block;
    return e * ext + r * stride + b;
  }
};

struct Buffers {
  unsigned char *strided = nullptr; // device
  unsigned char *packed = nullptr;  // device, or the device alias of pinned host memory
  unsigned char *host = nullptr;    // pinned host (oneshot), else nullptr
};

Buffers alloc(const Shape &s, bool oneshot) {
  Buffers b;
  CK(tempi_hip_malloc(reinterpret_cast<void **>(&b.strided), size_t(s.span())));
  if (oneshot) {
    void *h = nullptr, *d = nullptr;
    CK(tempi_hip_host_alloc(&h, &d, size_t(s.packed())));
    b.host = static_cast<unsigned char *>(h);
    b.packed = static_cast<unsigned char *>(d);
  } else {
    CK(tempi_hip_malloc(reinterpret_cast<void **>(&b.packed), size_t(s.packed())));
  }
  hipLaunchKernelGGL(fill_pattern, dim3(1024), dim3(256), 0, 0, b.strided, size_t(s.span()));
  CK(int(hipDeviceSynchronize()));
  return b;
}

void release(const Buffers &b) {
  tempi_hip_free(b.strided);
  if (b.host)
    tempi_hip_host_free(b.host);
  else
    tempi_hip_free(b.packed);
}

// the packed bytes against the strided pattern (byte i = i & 0xFF)
long check_packed(const Shape &s, const Buffers &b) {
  std::vector<unsigned char> g(size_t(s.packed()));
  if (b.host)
    std::memcpy(g.data(), b.host, g.size());
  else
    CK(tempi_hip_memcpy(g.data(), b.packed, g.size()));
  long errors = 0;
  for (int64_t k = 0; k < s.packed(); ++k) errors += g[size_t(k)] != (unsigned char)(s.offset(k) & 0xFF);
  return errors;
}

// the strided side after unpacking the packed pattern (byte k = 7k + 3)
long check_strided(const Shape &s, const Buffers &b) {
  std::vector<unsigned char> g(size_t(s.span()));
  CK(tempi_hip_memcpy(g.data(), b.strided, g.size()));
  long errors = 0;
  for (int64_t k = 0; k < s.packed(); ++k) {
    const int64_t o = s.offset(k);
    errors += g[size_t(o)] != (unsigned char)((k * 7 + 3) & 0xFF);
  }
  return errors;
}

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void print(const char *bench, const char *dst, const char *op, int64_t target, const Shape &s, double us,
           int iters, long errors) {
  const double mib = double(s.packed()) / 1024.0 / 1024.0;
  std::printf("{\"bench\": \"%s\", \"dst\": \"%s\", \"op\": \"%s\", \"target\": %lld, \"count\": %lld, "
              "\"block\": %lld, \"stride\": %lld, \"packed\": %lld, \"us\": %.3f, \"MiBps\": %.1f, \"iters\": %d, "
              "\"errors\": %ld}\n",
              bench, dst, op, (long long)target, (long long)s.count, (long long)s.block, (long long)s.stride,
              (long long)s.packed(), us, mib / (us * 1e-6), iters, errors);
  std::fflush(stdout);
}

// bench_pack: synchronous pack and unpack calls, wall time
long packer_point(void *stream, int64_t target, int64_t block, bool oneshot, int iters) {
  Shape s{target / block, block, 512, 1, 0};
  s.ext = (s.rows - 1) * s.stride + s.block;
  const tempi_hip_desc d = s.desc();
  Buffers b = alloc(s, oneshot);
  std::vector<double> tp, tu;
  long errors = 0;
  for (int it = 0; it < iters + 2; ++it) { // 2 warm-up calls
    double t0 = now_s();
    CK(tempi_hip_pack(b.packed, b.strided, &d, stream));
    CK(tempi_hip_stream_synchronize(stream));
    double t1 = now_s();
    if (it == 0) {
      errors += check_packed(s, b);
      // a different packed pattern for the unpack's check
      std::vector<unsigned char> p(size_t(s.packed()));
      for (size_t k = 0; k < p.size(); ++k) p[k] = (unsigned char)((k * 7 + 3) & 0xFF);
      if (b.host)
        std::memcpy(b.host, p.data(), p.size());
      else
        CK(tempi_hip_memcpy(b.packed, p.data(), p.size()));
    }
    double t2 = now_s();
    CK(tempi_hip_unpack(b.strided, b.packed, &d, stream));
    CK(tempi_hip_stream_synchronize(stream));
    double t3 = now_s();
    if (it == 0) errors += check_strided(s, b);
    if (it >= 2) {
      tp.push_back(t1 - t0);
      tu.push_back(t3 - t2);
    }
  }
  const char *dst = oneshot ? "oneshot" : "device";
  print("bench_pack", dst, "pack", target, s, trimean(tp) * 1e6, iters, errors);
  print("bench_pack", dst, "unpack", target, s, trimean(tu) * 1e6, iters, errors);
  release(b);
  return errors;
}

// bench_pack_kernels: the pack kernel alone, HIP events around the launch
long kernel_point(void *stream, void *e0, void *e1, int64_t target, int64_t count, int64_t stride, int64_t block,
                  bool oneshot) {
  const int iters = 30;
  Shape s{target / block, block, stride, count, 0};
  s.ext = (s.rows - 1) * s.stride + s.block; // objects end to end (bench_pack_kernels.cu:32)
  const tempi_hip_desc d = s.desc();
  Buffers b = alloc(s, oneshot);
  std::vector<double> t;
  long errors = 0;
  for (int it = 0; it < iters + 1; ++it) {
    CK(tempi_hip_event_record(e0, stream));
    CK(tempi_hip_pack(b.packed, b.strided, &d, stream));
    CK(tempi_hip_event_record(e1, stream));
    CK(tempi_hip_event_synchronize(e1));
    float ms = 0;
    CK(tempi_hip_event_elapsed_ms(&ms, e0, e1));
    if (it == 0)
      errors += check_packed(s, b);
    else
      t.push_back(double(ms) * 1e3);
  }
  print("bench_pack_kernels", oneshot ? "oneshot" : "device", "pack", target, s, trimean(t), iters, errors);
  release(b);
  return errors;
}

} // namespace

int main(int argc, char **argv) {
  int iters = argc > 1 && argv[1][0] != '-' ? std::max(1, std::atoi(argv[1])) : 200;
  bool packer = false, kernels = false;
  int64_t maxTarget = int64_t(1) << 40;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--packer")) packer = true;
    if (!std::strcmp(argv[i], "--kernels")) kernels = true;
    if (!std::strcmp(argv[i], "--max-target") && i + 1 < argc) maxTarget = std::atoll(argv[++i]);
  }
  if (!packer && !kernels) packer = kernels = true;
  void *stream, *e0, *e1;
  CK(tempi_hip_stream_create(&stream));
  CK(tempi_hip_event_create(&e0, 1));
  CK(tempi_hip_event_create(&e1, 1));
  long errors = 0;
  if (packer) {
    const int64_t targets[] = {64, 256, 1024, 4096, 16384, 65536, 262144, 1048576, 4 * 1048576};
    const int64_t contigs[] = {1, 2, 4, 8, 12, 16, 20, 24, 32, 64, 128, 256};
    for (bool oneshot : {true, false})
      for (int64_t target : targets)
        for (int64_t contig : contigs)
          if (target <= maxTarget)
            errors += packer_point(stream, target, std::min(contig, target), oneshot, iters);
  }
  if (kernels) {
    const int64_t blocks[] = {1, 2, 4, 6, 8, 12, 16, 20, 24, 28, 32, 64, 96, 128, 256};
    for (bool oneshot : {false, true})
      for (int64_t target : {int64_t(1024), int64_t(1048576)})
        for (int64_t count : {1, 2})
          for (int64_t stride : {16, 256})
            for (int64_t block : blocks)
              if (target / block > 0 && stride >= block && target <= maxTarget)
                errors += kernel_point(stream, e0, e1, target, count, stride, block, oneshot);
  }
  tempi_hip_event_destroy(e0);
  tempi_hip_event_destroy(e1);
  tempi_hip_stream_destroy(stream);
  return errors ? 3 : 0;
}
