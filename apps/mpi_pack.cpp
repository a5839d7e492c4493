// apps/mpi_pack.cpp -- the reference's headline MPI_Pack benchmark
// (/root/reference/bin/bench_mpi_pack.cpp:24-95, 120-190): one rank, 2D byte
// objects of `target` packed bytes per element (1 KiB, 1 MiB, 4 MiB), count
// 1 and 2, rows of 1-512 B at a 512-B stride, built three ways
// (MPI_Type_vector, MPI_Type_create_hvector, MPI_Type_create_subarray:
// /root/reference/support/type.cpp:216-242); MPI_Pack then MPI_Unpack of the
// whole object, wall time per call (MPI_Wtime), trimean over ITERS, reported
// as the reference does in MiB/s of packed bytes. Buffers are device memory
// (hipMalloc), or pageable host memory with --host (with TEMPI_DISABLE=1:
// the library's own CPU path, the reference's comparison). Source byte i is
// i & 0xFF; every point's first pack is checked byte for byte against the
// type map.
//
// usage: mpiexec -n 1 mpi_pack ITERS [--host] [--factory NAME] [--min-target BYTES] [--max-target BYTES]
//                                   [--shape N:BL:STRIDE] [--pin]
//        one JSON object per point. --shape times that one vector(N, BL, STRIDE) of MPI_BYTE at count 1
//        (BASELINE config 1 is 1024:512:1024); --pin runs on one core (the first of the affinity mask).
#include <hip/hip_runtime.h>
#include <mpi.h>

#include <algorithm>
#include <sched.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define HIPCHECK(x)                                                                                \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) {                                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));              \
      MPI_Abort(MPI_COMM_WORLD, 1);                                                                \
    }                                                                                              \
  } while (0)

namespace {

MPI_Datatype make_vector(int n, int bl, int stride) {
  MPI_Datatype t;
  MPI_Type_vector(n, bl, stride, MPI_BYTE, &t);
  return t;
}
MPI_Datatype make_hvector(int n, int bl, int stride) {
  MPI_Datatype t;
  MPI_Type_create_hvector(n, bl, stride, MPI_BYTE, &t);
  return t;
}
MPI_Datatype make_subarray(int n, int bl, int stride) {
  int sizes[2] = {n, stride}, subs[2] = {n, bl}, starts[2] = {0, 0};
  MPI_Datatype t;
  MPI_Type_create_subarray(2, sizes, subs, starts, MPI_ORDER_C, MPI_BYTE, &t);
  return t;
}

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

} // namespace

int main(int argc, char **argv) {
  MPI_Init(&argc, &argv);
  const int iters = argc > 1 ? std::max(1, std::atoi(argv[1])) : 100;
  bool host = false;
  const char *only = nullptr;
  bool shape = false;
  int shapeN = 0, shapeBl = 0, shapeStride = 0;
  long minTarget = 0, maxTarget = 1L << 30;
  for (int i = 2; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--host")) host = true;
    if (!std::strcmp(argv[i], "--max-target") && i + 1 < argc) maxTarget = std::atol(argv[++i]);
    if (!std::strcmp(argv[i], "--min-target") && i + 1 < argc) minTarget = std::atol(argv[++i]);
    if (!std::strcmp(argv[i], "--factory") && i + 1 < argc) only = argv[++i];
    if (!std::strcmp(argv[i], "--shape") && i + 1 < argc) {
      shape = true;
      std::sscanf(argv[++i], "%d:%d:%d", &shapeN, &shapeBl, &shapeStride);
    }
    if (!std::strcmp(argv[i], "--pin")) {
      cpu_set_t m;
      if (sched_getaffinity(0, sizeof m, &m) == 0)
        for (int c = 0; c < CPU_SETSIZE; ++c)
          if (CPU_ISSET(c, &m)) {
            cpu_set_t one;
            CPU_ZERO(&one);
            CPU_SET(c, &one);
            sched_setaffinity(0, sizeof one, &one);
            break;
          }
    }
  }
  struct Factory {
    const char *name;
    MPI_Datatype (*make)(int, int, int);
  };
  const Factory factories[] = {{"vector", make_vector}, {"hvector", make_hvector}, {"subarray", make_subarray}};
  long errorsTotal = 0;
  std::vector<int> targets = {1024, 1024 * 1024, 4 * 1024 * 1024}, counts = {1, 2},
                   blocks = {1, 2, 4, 8, 32, 64, 128, 256, 512};
  if (shape) {
    targets = {shapeN * shapeBl};
    counts = {1};
    blocks = {shapeBl};
    only = "vector";
  }
  const int stride = shape ? shapeStride : 512;
  for (int target : targets)
    for (int count : counts)
      for (int bl : blocks)
        for (const Factory &f : factories) {
          if ((only && std::strcmp(only, f.name)) || target > maxTarget || target < minTarget) continue;
          const int n = target / bl;
          MPI_Datatype t = f.make(n, bl, stride);
          MPI_Type_commit(&t);
          MPI_Aint lb, ext;
          MPI_Type_get_extent(t, &lb, &ext);
          int psize = 0;
          MPI_Pack_size(count, t, MPI_COMM_WORLD, &psize);
          const size_t span = size_t(ext) * size_t(count);
          char *src, *dst;
          if (host) {
            src = static_cast<char *>(std::malloc(span));
            dst = static_cast<char *>(std::malloc(size_t(psize)));
            if (!src || !dst) {
              std::fprintf(stderr, "mpi_pack: cannot allocate %zu host bytes\n", span);
              MPI_Abort(MPI_COMM_WORLD, 1);
            }
            for (size_t i = 0; i < span; ++i) src[i] = char(i & 0xFF);
          } else {
            HIPCHECK(hipMalloc(&src, span));
            HIPCHECK(hipMalloc(&dst, size_t(psize)));
            hipLaunchKernelGGL(fill_pattern, dim3(4096), dim3(256), 0, 0, reinterpret_cast<unsigned char *>(src), span);
            HIPCHECK(hipDeviceSynchronize());
          }
          std::vector<double> tp, tu;
          long errors = 0;
          for (int it = 0; it < iters + 2; ++it) { // 2 warm-up calls
            int pos = 0;
            double t0 = MPI_Wtime();
            MPI_Pack(src, count, t, dst, psize, &pos, MPI_COMM_WORLD);
            double t1 = MPI_Wtime();
            if (it == 0) { // the packed bytes: element e, row r, byte b
              std::vector<unsigned char> g(static_cast<size_t>(psize));
              if (host)
                std::memcpy(g.data(), dst, g.size());
              else
                HIPCHECK(hipMemcpy(g.data(), dst, g.size(), hipMemcpyDeviceToHost));
              size_t k = 0;
              for (int e = 0; e < count; ++e)
                for (int r = 0; r < n; ++r)
                  for (int b = 0; b < bl; ++b, ++k)
                    errors += g[k] != (unsigned char)((size_t(e) * size_t(ext) + size_t(r) * size_t(stride) +
                                                       size_t(b)) & 0xFF);
            }
            pos = 0;
            double t2 = MPI_Wtime();
            MPI_Unpack(dst, psize, &pos, src, count, t, MPI_COMM_WORLD);
            double t3 = MPI_Wtime();
            if (it >= 2) {
              tp.push_back(t1 - t0);
              tu.push_back(t3 - t2);
            }
          }
          const double p = std::max(trimean(tp), 1e-9), u = std::max(trimean(tu), 1e-9); // (timer ticks)
          const double mib = double(psize) / 1024.0 / 1024.0;
          std::printf("{\"target\": %d, \"count\": %d, \"block\": %d, \"stride\": %d, \"factory\": \"%s\", "
                      "\"packed\": %d, \"pack_us\": %.3f, \"unpack_us\": %.3f, \"pack_MiBps\": %.1f, "
                      "\"unpack_MiBps\": %.1f, \"iters\": %d, \"errors\": %ld, \"buffers\": \"%s\", "
                      "\"tempi\": %s}\n",
                      target, count, bl, stride, f.name, psize, p * 1e6, u * 1e6, mib / p, mib / u, iters, errors,
                      host ? "host" : "device", std::getenv("TEMPI_DISABLE") ? "false" : "true");
          std::fflush(stdout);
          errorsTotal += errors;
          if (host) {
            std::free(src);
            std::free(dst);
          } else {
            HIPCHECK(hipFree(src));
            HIPCHECK(hipFree(dst));
          }
          MPI_Type_free(&t);
        }
  MPI_Finalize();
  return errorsTotal ? 3 : 0;
}
