// apps/pingpong_nd.cpp -- strided MPI_Send / MPI_Recv ping-pong of device
// buffers between ranks 0 and 1 (config 3).
//
// Workload of the reference's bench_mpi_pingpong_nd (/root/reference/bin/
// bench_mpi_pingpong_nd.cpp:146-197): MPI_Type_vector(total/bl, bl, 512,
// MPI_BYTE), count 1, rank 0 -> 1 -> 0, one-way time = trimean(round trip)/2.
// The method comes from the environment (TEMPI_DATATYPE_*). --check verifies
// the bytes that arrived on every iteration's last hop.
//
// usage: pingpong_nd ITERS TOTAL_BYTES BLOCK [STRIDE] [--check]
#include <hip/hip_runtime.h>
#include <mpi.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define HIPCHECK(x)                                                                                \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) {                                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));              \
      MPI_Abort(MPI_COMM_WORLD, 1);                                                                \
    }                                                                                              \
  } while (0)

static double trimean(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  auto pct = [&](double p) {
    const double idx = p * double(v.size() - 1);
    const size_t lo = size_t(std::floor(idx)), hi = size_t(std::ceil(idx));
    return v[lo] + (v[hi] - v[lo]) * (idx - double(lo));
  };
  return (pct(0.25) + 2 * pct(0.5) + pct(0.75)) / 4;
}

int main(int argc, char **argv) {
  MPI_Init(&argc, &argv);
  int rank, size;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &size);
  bool check = false;
  std::vector<long> pos;
  for (int i = 1; i < argc; ++i) {
    if (std::string(argv[i]) == "--check")
      check = true;
    else
      pos.push_back(std::atol(argv[i]));
  }
  if (size < 2 || pos.size() < 3) {
    if (!rank) std::fprintf(stderr, "usage: %s ITERS TOTAL BLOCK [STRIDE] [--check] (2+ ranks)\n", argv[0]);
    MPI_Abort(MPI_COMM_WORLD, 1);
  }
  const int iters = int(pos[0]);
  const long total = pos[1], bl = pos[2], stride = pos.size() > 3 ? pos[3] : 512;
  const int nblocks = int(total / bl);
  int ndev = 0;
  HIPCHECK(hipGetDeviceCount(&ndev));
  HIPCHECK(hipSetDevice(rank % ndev));

  MPI_Datatype t;
  MPI_Type_vector(nblocks, int(bl), int(stride), MPI_BYTE, &t);
  MPI_Type_commit(&t);
  MPI_Aint lb, ext;
  MPI_Type_get_extent(t, &lb, &ext);
  char *buf;
  HIPCHECK(hipMalloc(&buf, size_t(ext)));
  std::vector<unsigned char> h(static_cast<size_t>(ext));
  for (size_t i = 0; i < h.size(); ++i) h[i] = (unsigned char)((i * 131 + size_t(rank) * 7) & 0xFF);
  HIPCHECK(hipMemcpy(buf, h.data(), h.size(), hipMemcpyHostToDevice));

  std::vector<double> times;
  long errors = 0;
  for (int i = 0; i < iters + 2; ++i) {
    MPI_Barrier(MPI_COMM_WORLD);
    const double t0 = MPI_Wtime();
    if (rank == 0) {
      MPI_Send(buf, 1, t, 1, 0, MPI_COMM_WORLD);
      MPI_Recv(buf, 1, t, 1, 0, MPI_COMM_WORLD, MPI_STATUS_IGNORE);
    } else if (rank == 1) {
      MPI_Recv(buf, 1, t, 0, 0, MPI_COMM_WORLD, MPI_STATUS_IGNORE);
      MPI_Send(buf, 1, t, 0, 0, MPI_COMM_WORLD);
    }
    const double el = MPI_Wtime() - t0;
    if (i >= 2) times.push_back(el);
  }
  if (check && rank < 2) {
    // after the exchanges every block holds rank 0's original bytes; the
    // gaps keep each rank's own pattern
    std::vector<unsigned char> g(static_cast<size_t>(ext));
    HIPCHECK(hipMemcpy(g.data(), buf, g.size(), hipMemcpyDeviceToHost));
    for (long b = 0; b < nblocks; ++b)
      for (long k = 0; k < stride && b * stride + k < long(ext); ++k) {
        const size_t i = size_t(b * stride + k);
        const unsigned char exp0 = (unsigned char)((i * 131) & 0xFF);
        const unsigned char mine = (unsigned char)((i * 131 + size_t(rank) * 7) & 0xFF);
        const unsigned char exp = k < bl ? exp0 : mine;
        if (g[i] != exp) ++errors;
      }
  }
  MPI_Allreduce(MPI_IN_PLACE, &errors, 1, MPI_LONG, MPI_SUM, MPI_COMM_WORLD);
  if (rank == 0) {
    const double oneway = trimean(times) / 2;
    std::printf("{\"total\": %ld, \"block\": %ld, \"stride\": %ld, \"iters\": %d, \"oneway_us\": %.2f, "
                "\"GBps\": %.3f, \"checked\": %s, \"errors\": %ld, \"method\": \"%s\"}\n",
                total, bl, stride, iters, oneway * 1e6, double(total) / oneway / 1e9, check ? "true" : "false",
                errors, std::getenv("TEMPI_DATATYPE_ONESHOT") ? "ONESHOT" : std::getenv("TEMPI_DATATYPE_STAGED") ? "STAGED" : std::getenv("TEMPI_DATATYPE_IPC") ? "IPC" : std::getenv("TEMPI_DATATYPE_DEVICE") ? "DEVICE" : std::getenv("TEMPI_DISABLE") ? "LIBRARY" : "AUTO");
    std::fflush(stdout);
  }
  MPI_Type_free(&t);
  HIPCHECK(hipFree(buf));
  MPI_Finalize();
  return errors ? 3 : 0;
}
