// apps/bench_lib.cpp -- configs 3 and 5 as library calls (libtempi_apps.so),
// so that bench.py can run them inside the driver's torch.distributed launch
// and the CLIs (apps/pingpong_nd.cpp, apps/alltoallv_sparse.cpp) under mpiexec.
//
// tempi_bench_pingpong: the reference's bench_mpi_pingpong_nd
//   (/root/reference/bin/bench_mpi_pingpong_nd.cpp:146-197):
//   MPI_Type_vector(total/bl, bl, stride, MPI_BYTE), count 1, device buffers,
//   rank 0 -> 1 -> 0 with MPI_Send / MPI_Recv; one-way time = trimean of the
//   round trips / 2. Ranks other than 0 and 1 only take part in the barriers.
//   check: every block holds rank 0's bytes afterwards, every gap its owner's.
//
// tempi_bench_pingpong_1d: the reference's bench_mpi_pingpong_1d
//   (/root/reference/bin/bench_mpi_pingpong_1d.cpp:29-100, 119-165): MPI_BYTE
//   count = total, device buffers, every rank r < size/2 paired with
//   r + size/2 (all pairs at once), MPI_Send then MPI_Recv (the partner
//   Recv then Send); time = max over ranks per iteration, trimean, one-way =
//   half of it. check: every rank's receive buffer holds its partner's bytes.
//
// tempi_bench_alltoallv: the reference's bench_alltoallv_random_sparse
//   (/root/reference/bin/bench_alltoallv_random_sparse.cpp:100-222): an
//   MPI_BYTE MPI_Alltoallv of device buffers whose counts are the matrix of
//   SquareMat::make_random_sparse(size, round(density*size), 1, 10, scale,
//   seed) (/root/reference/support/squaremat.cpp:52-75, restated here with
//   the same srand/rand and std::shuffle(default_random_engine) calls, so the
//   matrix is the reference's own); time = max over ranks, min over
//   iterations, as there. check: every received byte is the sender's pattern.
//
// tempi_bench_nbr_alltoallv: the reference's bench_nbr_alltoallv_random_sparse
//   (/root/reference/bin/bench_nbr_alltoallv_random_sparse.cpp:100-330): the
//   same matrix as a distributed graph (MPI_Dist_graph_create_adjacent over
//   the nonzeros, weights = bytes, reorder = 1 as there, so TEMPI_PLACEMENT_*
//   places the ranks), then MPI_BYTE MPI_Neighbor_alltoallv of device buffers
//   with graph rank q sending row q of the matrix. Reported as there: setup
//   (graph creation) and teardown (MPI_Comm_free) times, min over iterations
//   of the max over ranks, and the pattern's bytes between and within nodes
//   (:40-97) under the placement that was made.
//
// tempi_bench_sync_phases: where one synchronous MPI_Pack of BASELINE config 1
//   (MPI_Type_vector(1024, 512, 1024, MPI_BYTE), 512 KiB, device buffers) spends
//   its time on this box, all in C (no Python): the interposed call end to
//   end, and its phases at libtempi_hip's C ABI -- pointer classification of
//   both sides, the launch (host time of tempi_hip_pack_ticket), the wait for
//   the ticket the kernel stores; the kernel alone between HIP events (200
//   back-to-back launches); and MPICH's own MPI_Pack of the same type on host
//   buffers (TEMPI hands host buffers to the library). Medians over `reps`.
#include <hip/hip_runtime.h>
#include <mpi.h>

#include "tempi_hip.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <random>
#include <vector>

#define HIPCHECK(x)                                                                                \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) {                                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));              \
      MPI_Abort(MPI_COMM_WORLD, 1);                                                                \
    }                                                                                              \
  } while (0)

#define EXPORT extern "C" __attribute__((visibility("default")))

namespace {

double trimean(std::vector<double> v) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  auto pct = [&](double p) {
    const double idx = p * double(v.size() - 1);
    const size_t lo = size_t(std::floor(idx)), hi = size_t(std::ceil(idx));
    return v[lo] + (v[hi] - v[lo]) * (idx - double(lo));
  };
  return (pct(0.25) + 2 * pct(0.5) + pct(0.75)) / 4;
}

const char *method_name() {
  if (std::getenv("TEMPI_DATATYPE_ONESHOT")) return "ONESHOT";
  if (std::getenv("TEMPI_DATATYPE_STAGED")) return "STAGED";
  if (std::getenv("TEMPI_DATATYPE_IPC")) return "IPC";
  if (std::getenv("TEMPI_DATATYPE_DEVICE")) return "DEVICE";
  if (std::getenv("TEMPI_DISABLE")) return "LIBRARY";
  return "AUTO";
}

// SquareMat::make_random_sparse (row-major ranks x ranks)
std::vector<int64_t> random_sparse(int ranks, int rowNnz, int lb, int ub, int scale, int seed) {
  srand(unsigned(seed));
  std::default_random_engine dre(static_cast<std::default_random_engine::result_type>(seed));
  rowNnz = std::min(rowNnz, ranks);
  std::vector<int64_t> mat(size_t(ranks) * size_t(ranks), 0);
  std::vector<size_t> rowInd(static_cast<size_t>(ranks));
  std::iota(rowInd.begin(), rowInd.end(), size_t(0));
  for (int r = 0; r < ranks; ++r) {
    std::shuffle(rowInd.begin(), rowInd.end(), dre);
    for (int i = 0; i < rowNnz; ++i) mat[size_t(r) * size_t(ranks) + rowInd[size_t(i)]] = (lb + rand() % (ub - lb)) * scale;
  }
  return mat;
}

__host__ __device__ inline unsigned char a2av_byte(int64_t i, int src, int dst) {
  return (unsigned char)((i * 31 + src * 7 + dst * 13) & 0xFF);
}

// TEMPI_BENCH_HOST=1: the same workload on pageable host memory -- the
// library path the reference takes for host buffers (with TEMPI_DISABLE=1:
// the host MPI alone, bench.py's CPU baselines)
bool host_buffers() {
  const char *e = std::getenv("TEMPI_BENCH_HOST");
  return e && *e && *e != '0';
}
void *buf_alloc(size_t n) {
  void *p = nullptr;
  if (host_buffers())
    p = std::aligned_alloc(4096, (std::max<size_t>(n, 1) + 4095) / 4096 * 4096);
  else
    HIPCHECK(hipMalloc(&p, std::max<size_t>(n, 1)));
  return p;
}
void buf_free(void *p) {
  if (host_buffers())
    std::free(p);
  else
    HIPCHECK(hipFree(p));
}
// bytes between a host vector and a benchmark buffer (either kind)
void buf_copy(void *dst, const void *src, size_t n) {
  if (host_buffers())
    std::memcpy(dst, src, n);
  else
    HIPCHECK(hipMemcpy(dst, src, n, hipMemcpyDefault));
}

} // namespace

EXPORT int tempi_bench_pingpong(int iters, long total, long bl, long stride, int check, int setDevice, char *json,
                                int jsonCap) {
  int rank, size;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &size);
  if (size < 2 || bl <= 0 || total < bl || stride < bl) return 2;
  const int nblocks = int(total / bl);
  if (setDevice) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0; // (host buffers need no GPU)
    if (ndev > 0) HIPCHECK(hipSetDevice(rank % ndev));
  }
  MPI_Datatype t;
  MPI_Type_vector(nblocks, int(bl), int(stride), MPI_BYTE, &t);
  MPI_Type_commit(&t);
  MPI_Aint lb, ext;
  MPI_Type_get_extent(t, &lb, &ext);
  char *buf = static_cast<char *>(buf_alloc(size_t(ext)));
  std::vector<unsigned char> h(static_cast<size_t>(ext));
  for (size_t i = 0; i < h.size(); ++i) h[i] = (unsigned char)((i * 131 + size_t(rank) * 7) & 0xFF);
  buf_copy(buf, h.data(), h.size());

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
    // every block now holds rank 0's original bytes; the gaps keep each
    // rank's own pattern
    std::vector<unsigned char> g(static_cast<size_t>(ext));
    buf_copy(g.data(), buf, g.size());
    for (long b = 0; b < nblocks; ++b)
      for (long k = 0; k < stride && b * stride + k < long(ext); ++k) {
        const size_t i = size_t(b * stride + k);
        const unsigned char exp0 = (unsigned char)((i * 131) & 0xFF);
        const unsigned char mine = (unsigned char)((i * 131 + size_t(rank) * 7) & 0xFF);
        if (g[i] != (k < bl ? exp0 : mine)) ++errors;
      }
  }
  MPI_Allreduce(MPI_IN_PLACE, &errors, 1, MPI_LONG, MPI_SUM, MPI_COMM_WORLD);
  if (rank == 0 && json && jsonCap > 0) {
    const double oneway = trimean(times) / 2;
    std::snprintf(json, size_t(jsonCap),
                  "{\"total\": %ld, \"block\": %ld, \"stride\": %ld, \"iters\": %d, \"oneway_us\": %.2f, "
                  "\"GBps\": %.3f, \"checked\": %s, \"errors\": %ld, \"method\": \"%s\", \"buffers\": \"%s\"}",
                  total, bl, stride, iters, oneway * 1e6, double(total) / oneway / 1e9, check ? "true" : "false",
                  errors, method_name(), host_buffers() ? "host" : "device");
  }
  MPI_Type_free(&t);
  buf_free(buf);
  return errors ? 3 : 0;
}

// block d of buf (displ[d], count[d] bytes) gets the pattern of src -> dst[d]
// (dst == nullptr: d itself)
EXPORT int tempi_bench_pingpong_1d(int iters, long total, int check, int setDevice, char *json, int jsonCap) {
  int rank, size;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &size);
  if (size < 2 || total <= 0 || total > (1L << 30)) return 2;
  if (setDevice) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0; // (host buffers need no GPU)
    if (ndev > 0) HIPCHECK(hipSetDevice(rank % ndev));
  }
  const int half = size / 2;
  const int partner = rank < half ? rank + half : (rank < 2 * half ? rank - half : -1); // odd size: the last idles
  char *src = static_cast<char *>(buf_alloc(size_t(total)));
  char *dst = static_cast<char *>(buf_alloc(size_t(total)));
  std::vector<unsigned char> h(static_cast<size_t>(total));
  for (size_t i = 0; i < h.size(); ++i) h[i] = (unsigned char)((i * 7 + size_t(rank) * 31) & 0xFF);
  buf_copy(src, h.data(), h.size());
  std::vector<double> times;
  for (int i = 0; i < iters + 2; ++i) {
    MPI_Barrier(MPI_COMM_WORLD);
    const double t0 = MPI_Wtime();
    if (partner >= 0 && rank < half) {
      MPI_Send(src, int(total), MPI_BYTE, partner, 0, MPI_COMM_WORLD);
      MPI_Recv(dst, int(total), MPI_BYTE, partner, 0, MPI_COMM_WORLD, MPI_STATUS_IGNORE);
    } else if (partner >= 0) {
      MPI_Recv(dst, int(total), MPI_BYTE, partner, 0, MPI_COMM_WORLD, MPI_STATUS_IGNORE);
      MPI_Send(src, int(total), MPI_BYTE, partner, 0, MPI_COMM_WORLD);
    }
    double el = MPI_Wtime() - t0;
    MPI_Allreduce(MPI_IN_PLACE, &el, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
    if (i >= 2) times.push_back(el);
  }
  long errors = 0;
  if (check && partner >= 0) {
    std::vector<unsigned char> g(static_cast<size_t>(total));
    buf_copy(g.data(), dst, g.size());
    for (size_t i = 0; i < g.size(); ++i) errors += g[i] != (unsigned char)((i * 7 + size_t(partner) * 31) & 0xFF);
  }
  MPI_Allreduce(MPI_IN_PLACE, &errors, 1, MPI_LONG, MPI_SUM, MPI_COMM_WORLD);
  if (rank == 0 && json && jsonCap > 0) {
    const double oneway = trimean(times) / 2;
    std::snprintf(json, size_t(jsonCap),
                  "{\"total\": %ld, \"pairs\": %d, \"iters\": %d, \"oneway_us\": %.2f, \"pair_GBps\": %.3f, "
                  "\"aggregate_GBps\": %.3f, \"checked\": %s, \"errors\": %ld, \"method\": \"%s\", "
                  "\"buffers\": \"%s\"}",
                  total, half, iters, oneway * 1e6, double(total) / oneway / 1e9,
                  double(half) * double(total) / oneway / 1e9, check ? "true" : "false", errors, method_name(),
                  host_buffers() ? "host" : "device");
  }
  buf_free(src);
  buf_free(dst);
  return errors ? 3 : 0;
}

// tempi_bench_isend: the reference's bench_mpi_isend
// (/root/reference/bin/bench_mpi_isend.cpp:21-83): ranks 0 and 1 ping-pong
// `tags` overlapping contiguous MPI_BYTE messages of `bytes` each (device
// buffers) -- rank 0 MPI_Isend's all of them and MPI_Waitall's, then posts
// the MPI_Irecv's for the replies; rank 1 the other way round. Reported as
// there: 2 x bytes / trimean(round trip) in MiB/s (:130), plus every received
// byte checked when `check` (the reference checks none).
EXPORT int tempi_bench_isend(int iters, long bytes, int tags, int check, char *json, int jsonCap) {
  int rank, size;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &size);
  if (size < 2 || bytes <= 0 || bytes > (1L << 30) || tags < 1) return 2;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0; // (host buffers need no GPU)
  if (ndev > 0) HIPCHECK(hipSetDevice(rank % ndev));
  const bool active = rank < 2;
  const int peer = 1 - rank;
  std::vector<char *> srcs(static_cast<size_t>(tags)), dsts(static_cast<size_t>(tags));
  std::vector<unsigned char> h(static_cast<size_t>(bytes));
  for (int t = 0; t < tags; ++t) {
    srcs[size_t(t)] = static_cast<char *>(buf_alloc(size_t(bytes)));
    dsts[size_t(t)] = static_cast<char *>(buf_alloc(size_t(bytes)));
    for (size_t i = 0; i < h.size(); ++i) h[i] = (unsigned char)((i * 13 + size_t(t) * 7 + size_t(rank) * 101) & 0xFF);
    buf_copy(srcs[size_t(t)], h.data(), h.size());
  }
  std::vector<MPI_Request> reqs(static_cast<size_t>(tags));
  std::vector<double> times;
  auto sends = [&] {
    for (int t = 0; t < tags; ++t) MPI_Isend(srcs[size_t(t)], int(bytes), MPI_BYTE, peer, t, MPI_COMM_WORLD, &reqs[size_t(t)]);
    MPI_Waitall(tags, reqs.data(), MPI_STATUSES_IGNORE);
  };
  auto recvs = [&] {
    for (int t = 0; t < tags; ++t) MPI_Irecv(dsts[size_t(t)], int(bytes), MPI_BYTE, peer, t, MPI_COMM_WORLD, &reqs[size_t(t)]);
    MPI_Waitall(tags, reqs.data(), MPI_STATUSES_IGNORE);
  };
  for (int i = 0; i < iters + 2; ++i) {
    MPI_Barrier(MPI_COMM_WORLD);
    const double t0 = MPI_Wtime();
    if (active && rank == 0) {
      sends();
      recvs();
    } else if (active) {
      recvs();
      sends();
    }
    double el = MPI_Wtime() - t0;
    MPI_Allreduce(MPI_IN_PLACE, &el, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
    if (i >= 2) times.push_back(el);
  }
  long errors = 0;
  if (check && active) {
    std::vector<unsigned char> g(static_cast<size_t>(bytes));
    for (int t = 0; t < tags; ++t) {
      buf_copy(g.data(), dsts[size_t(t)], g.size());
      for (size_t i = 0; i < g.size(); ++i)
        errors += g[i] != (unsigned char)((i * 13 + size_t(t) * 7 + size_t(peer) * 101) & 0xFF);
    }
  }
  MPI_Allreduce(MPI_IN_PLACE, &errors, 1, MPI_LONG, MPI_SUM, MPI_COMM_WORLD);
  if (rank == 0 && json && jsonCap > 0) {
    const double rt = trimean(times);
    std::snprintf(json, size_t(jsonCap),
                  "{\"bytes\": %ld, \"tags\": %d, \"iters\": %d, \"roundtrip_us\": %.2f, \"MiBps\": %.2f, "
                  "\"checked\": %s, \"errors\": %ld, \"method\": \"%s\", \"buffers\": \"%s\"}",
                  bytes, tags, iters, rt * 1e6, 2.0 * double(bytes) / 1024 / 1024 / rt, check ? "true" : "false", errors,
                  method_name(), host_buffers() ? "host" : "device");
  }
  for (int t = 0; t < tags; ++t) {
    buf_free(srcs[size_t(t)]);
    buf_free(dsts[size_t(t)]);
  }
  return errors ? 3 : 0;
}

__global__ void a2av_fill(unsigned char *buf, const int64_t *displ, const int64_t *count, const int *dst, int n,
                          int src) {
  for (int d = 0; d < n; ++d)
    for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < count[d]; i += int64_t(gridDim.x) * blockDim.x)
      buf[displ[d] + i] = a2av_byte(i, src, dst ? dst[d] : d);
}

namespace {
// blocks (displ, count) of a benchmark buffer get the patterns src -> dst[d]
void fill_blocks(unsigned char *buf, const std::vector<int> &displ, const std::vector<int> &count,
                 const std::vector<int> &dst, int src) {
  const size_t n = displ.size();
  if (host_buffers()) {
    for (size_t d = 0; d < n; ++d)
      for (int64_t i = 0; i < count[d]; ++i) buf[displ[d] + i] = a2av_byte(i, src, dst[d]);
    return;
  }
  if (!n) return;
  std::vector<int64_t> hd(displ.begin(), displ.end()), hc(count.begin(), count.end());
  int64_t *dd, *dc;
  int *dr;
  HIPCHECK(hipMalloc(&dd, sizeof(int64_t) * n));
  HIPCHECK(hipMalloc(&dc, sizeof(int64_t) * n));
  HIPCHECK(hipMalloc(&dr, sizeof(int) * n));
  HIPCHECK(hipMemcpy(dd, hd.data(), sizeof(int64_t) * n, hipMemcpyHostToDevice));
  HIPCHECK(hipMemcpy(dc, hc.data(), sizeof(int64_t) * n, hipMemcpyHostToDevice));
  HIPCHECK(hipMemcpy(dr, dst.data(), sizeof(int) * n, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(a2av_fill, dim3(256), dim3(256), 0, 0, buf, dd, dc, dr, int(n), src);
  HIPCHECK(hipDeviceSynchronize());
  HIPCHECK(hipFree(dd));
  HIPCHECK(hipFree(dc));
  HIPCHECK(hipFree(dr));
}

void fill_byte(void *buf, int v, size_t n) {
  if (host_buffers())
    std::memset(buf, v, n);
  else
    HIPCHECK(hipMemset(buf, v, n));
}

// node of every rank of comm, by world rank: TEMPI_FAKE_NODE_SIZE groups of
// consecutive world ranks (the nodes TEMPI's placement sees in tests), else
// the ranks sharing memory with it
std::vector<int> node_of_ranks(MPI_Comm comm) {
  int wr = 0, size = 0;
  MPI_Comm_rank(MPI_COMM_WORLD, &wr);
  MPI_Comm_size(comm, &size);
  int node = wr;
  const char *f = std::getenv("TEMPI_FAKE_NODE_SIZE");
  if (f && std::atoi(f) > 0) {
    node = wr / std::atoi(f);
  } else {
    MPI_Comm shm;
    MPI_Comm_split_type(MPI_COMM_WORLD, MPI_COMM_TYPE_SHARED, 0, MPI_INFO_NULL, &shm);
    MPI_Allreduce(MPI_IN_PLACE, &node, 1, MPI_INT, MPI_MIN, shm);
    MPI_Comm_free(&shm);
  }
  std::vector<int> ids(static_cast<size_t>(size));
  MPI_Allgather(&node, 1, MPI_INT, ids.data(), 1, MPI_INT, comm);
  std::vector<int> distinct(ids);
  std::sort(distinct.begin(), distinct.end());
  distinct.erase(std::unique(distinct.begin(), distinct.end()), distinct.end());
  for (int &i : ids) i = int(std::lower_bound(distinct.begin(), distinct.end(), i) - distinct.begin());
  return ids; // 0 .. nodes - 1
}
} // namespace

EXPORT int tempi_bench_alltoallv(int iters, int scale, double density, int seed, int check, int setDevice,
                                 char *json, int jsonCap) {
  int rank, size;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &size);
  if (setDevice) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0; // (host buffers need no GPU)
    if (ndev > 0) HIPCHECK(hipSetDevice(rank % ndev));
  }
  const int rowNnz = int(density * size + 0.5);
  const std::vector<int64_t> mat = random_sparse(size, rowNnz, 1, 10, scale, seed);
  auto M = [&](int r, int c) { return mat[size_t(r) * size_t(size) + size_t(c)]; };
  std::vector<int> sc(static_cast<size_t>(size)), rc(static_cast<size_t>(size)), sd(static_cast<size_t>(size)), rd(static_cast<size_t>(size));
  int64_t sbytes = 0, rbytes = 0, maxPair = 0, total = 0;
  for (int p = 0; p < size; ++p) {
    sc[size_t(p)] = int(M(rank, p));
    rc[size_t(p)] = int(M(p, rank));
    sd[size_t(p)] = int(sbytes);
    rd[size_t(p)] = int(rbytes);
    sbytes += sc[size_t(p)];
    rbytes += rc[size_t(p)];
  }
  for (int r = 0; r < size; ++r)
    for (int c = 0; c < size; ++c) {
      total += M(r, c);
      if (r != c) maxPair = std::max(maxPair, M(r, c));
    }
  // busiest link: bytes out of (or into) one GPU to other GPUs
  int64_t maxOut = 0;
  for (int r = 0; r < size; ++r) {
    int64_t o = 0, in = 0;
    for (int c = 0; c < size; ++c)
      if (c != r) {
        o += M(r, c);
        in += M(c, r);
      }
    maxOut = std::max(maxOut, std::max(o, in));
  }
  unsigned char *sbuf = static_cast<unsigned char *>(buf_alloc(size_t(sbytes)));
  unsigned char *rbuf = static_cast<unsigned char *>(buf_alloc(size_t(rbytes)));
  if (host_buffers()) {
    for (int d = 0; d < size; ++d)
      for (int64_t i = 0; i < sc[size_t(d)]; ++i) sbuf[sd[size_t(d)] + i] = a2av_byte(i, rank, d);
    std::memset(rbuf, 0xEE, size_t(std::max<int64_t>(rbytes, 1)));
  } else {
    std::vector<int64_t> hd(static_cast<size_t>(size)), hc(static_cast<size_t>(size));
    for (int p = 0; p < size; ++p) {
      hd[size_t(p)] = sd[size_t(p)];
      hc[size_t(p)] = sc[size_t(p)];
    }
    int64_t *dd, *dc;
    HIPCHECK(hipMalloc(&dd, sizeof(int64_t) * size_t(size)));
    HIPCHECK(hipMalloc(&dc, sizeof(int64_t) * size_t(size)));
    HIPCHECK(hipMemcpy(dd, hd.data(), sizeof(int64_t) * size_t(size), hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(dc, hc.data(), sizeof(int64_t) * size_t(size), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(a2av_fill, dim3(256), dim3(256), 0, 0, sbuf, dd, dc, nullptr, size, rank);
    HIPCHECK(hipMemset(rbuf, 0xEE, size_t(std::max<int64_t>(rbytes, 1))));
    HIPCHECK(hipDeviceSynchronize());
    HIPCHECK(hipFree(dd));
    HIPCHECK(hipFree(dc));
  }
  std::vector<double> times;
  for (int i = 0; i < iters + 1; ++i) {
    MPI_Barrier(MPI_COMM_WORLD);
    const double t0 = MPI_Wtime();
    MPI_Alltoallv(sbuf, sc.data(), sd.data(), MPI_BYTE, rbuf, rc.data(), rd.data(), MPI_BYTE, MPI_COMM_WORLD);
    double el = MPI_Wtime() - t0;
    MPI_Allreduce(MPI_IN_PLACE, &el, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
    if (i >= 1) times.push_back(el);
  }
  long errors = 0;
  if (check) {
    std::vector<unsigned char> h(size_t(std::max<int64_t>(rbytes, 1)));
    buf_copy(h.data(), rbuf, h.size());
    for (int p = 0; p < size; ++p)
      for (int64_t i = 0; i < rc[size_t(p)]; ++i)
        if (h[size_t(rd[size_t(p)] + i)] != a2av_byte(i, p, rank)) ++errors;
    MPI_Allreduce(MPI_IN_PLACE, &errors, 1, MPI_LONG, MPI_SUM, MPI_COMM_WORLD);
  }
  if (rank == 0 && json && jsonCap > 0) {
    const double tmin = times.empty() ? 0 : *std::min_element(times.begin(), times.end());
    std::snprintf(json, size_t(jsonCap),
                  "{\"ranks\": %d, \"scale\": %d, \"density\": %.4f, \"row_nnz\": %d, \"seed\": %d, \"iters\": %d, "
                  "\"min_us\": %.2f, \"trimean_us\": %.2f, \"total_bytes\": %lld, \"max_pairwise_bytes\": %lld, "
                  "\"max_gpu_out_or_in_bytes\": %lld, \"checked\": %s, \"errors\": %ld, \"buffers\": \"%s\"}",
                  size, scale, density, rowNnz, seed, iters, tmin * 1e6, trimean(times) * 1e6, (long long)total,
                  (long long)maxPair, (long long)maxOut, check ? "true" : "false", errors,
                  host_buffers() ? "host" : "device");
  }
  buf_free(sbuf);
  buf_free(rbuf);
  return errors ? 3 : 0;
}

EXPORT int tempi_bench_nbr_alltoallv(int iters, int scale, double density, int seed, int reorder, int check,
                                     int setDevice, char *json, int jsonCap) {
  int wrank, size;
  MPI_Comm_rank(MPI_COMM_WORLD, &wrank);
  MPI_Comm_size(MPI_COMM_WORLD, &size);
  if (setDevice) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0; // (host buffers need no GPU)
    if (ndev > 0) HIPCHECK(hipSetDevice(wrank % ndev));
  }
  const int rowNnz = int(density * size + 0.5);
  const std::vector<int64_t> mat = random_sparse(size, rowNnz, 1, 10, scale, seed);
  auto M = [&](int r, int c) { return mat[size_t(r) * size_t(size) + size_t(c)]; };
  // the graph: this process's row and column of the matrix
  // (bench_nbr_alltoallv_random_sparse.cpp:143-152)
  std::vector<int> sources, sourceweights, destinations, destweights;
  for (int i = 0; i < size; ++i) {
    if (M(wrank, i)) {
      destinations.push_back(i);
      destweights.push_back(int(M(wrank, i)));
    }
    if (M(i, wrank)) {
      sources.push_back(i);
      sourceweights.push_back(int(M(i, wrank)));
    }
  }
  MPI_Comm graph;
  MPI_Barrier(MPI_COMM_WORLD);
  double t0 = MPI_Wtime();
  MPI_Dist_graph_create_adjacent(MPI_COMM_WORLD, int(sources.size()), sources.data(), sourceweights.data(),
                                 int(destinations.size()), destinations.data(), destweights.data(), MPI_INFO_NULL,
                                 reorder, &graph);
  double setup = MPI_Wtime() - t0;
  MPI_Allreduce(MPI_IN_PLACE, &setup, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
  // after placement this process is graph rank q and plays row q
  // (:232-259): its neighbours as the graph reports them
  int q = 0;
  MPI_Comm_rank(graph, &q);
  int indeg = 0, outdeg = 0, weighted = 0;
  MPI_Dist_graph_neighbors_count(graph, &indeg, &outdeg, &weighted);
  std::vector<int> in(static_cast<size_t>(indeg)), out(static_cast<size_t>(outdeg));
  std::vector<int> iw(size_t(indeg) + 1), ow(size_t(outdeg) + 1);
  MPI_Dist_graph_neighbors(graph, indeg, in.data(), iw.data(), outdeg, out.data(), ow.data());
  std::vector<int> sc, sd, rc, rd;
  int64_t sbytes = 0, rbytes = 0;
  for (int d : out) {
    sc.push_back(int(M(q, d)));
    sd.push_back(int(sbytes));
    sbytes += M(q, d);
  }
  for (int s : in) {
    rc.push_back(int(M(s, q)));
    rd.push_back(int(rbytes));
    rbytes += M(s, q);
  }
  // the pattern's bytes between and within nodes under this placement (:40-97)
  const std::vector<int> node = node_of_ranks(graph);
  const int nodes = *std::max_element(node.begin(), node.end()) + 1;
  std::vector<int64_t> nodeMat(size_t(nodes) * size_t(nodes), 0);
  int64_t maxPair = 0;
  for (int r = 0; r < size; ++r)
    for (int c = 0; c < size; ++c) {
      maxPair = std::max(maxPair, M(r, c));
      nodeMat[size_t(node[size_t(r)]) * size_t(nodes) + size_t(node[size_t(c)])] += M(r, c);
    }
  int64_t maxOn = 0, maxOff = 0, totOn = 0, totOff = 0;
  for (int i = 0; i < nodes; ++i) {
    int64_t off = 0;
    for (int j = 0; j < nodes; ++j) {
      const int64_t v = nodeMat[size_t(i) * size_t(nodes) + size_t(j)];
      if (i == j) {
        totOn += v;
        maxOn = std::max(maxOn, v);
      } else {
        off += v;
      }
    }
    totOff += off;
    maxOff = std::max(maxOff, off);
  }
  unsigned char *sbuf = static_cast<unsigned char *>(buf_alloc(size_t(sbytes)));
  unsigned char *rbuf = static_cast<unsigned char *>(buf_alloc(size_t(rbytes)));
  fill_blocks(sbuf, sd, sc, out, q);
  fill_byte(rbuf, 0xEE, size_t(std::max<int64_t>(rbytes, 1)));
  std::vector<double> times;
  for (int i = 0; i < iters + 1; ++i) {
    MPI_Barrier(MPI_COMM_WORLD);
    const double ts = MPI_Wtime();
    MPI_Neighbor_alltoallv(sbuf, sc.data(), sd.data(), MPI_BYTE, rbuf, rc.data(), rd.data(), MPI_BYTE, graph);
    double el = MPI_Wtime() - ts;
    MPI_Allreduce(MPI_IN_PLACE, &el, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
    if (i >= 1) times.push_back(el);
  }
  long errors = 0;
  if (check) {
    std::vector<unsigned char> h(size_t(std::max<int64_t>(rbytes, 1)));
    buf_copy(h.data(), rbuf, h.size());
    for (size_t k = 0; k < in.size(); ++k)
      for (int64_t i = 0; i < rc[k]; ++i)
        if (h[size_t(rd[k] + i)] != a2av_byte(i, in[k], q)) ++errors;
    MPI_Allreduce(MPI_IN_PLACE, &errors, 1, MPI_LONG, MPI_SUM, MPI_COMM_WORLD);
  }
  MPI_Barrier(MPI_COMM_WORLD);
  t0 = MPI_Wtime();
  MPI_Comm_free(&graph);
  double teardown = MPI_Wtime() - t0;
  MPI_Allreduce(MPI_IN_PLACE, &teardown, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
  if (wrank == 0 && json && jsonCap > 0) {
    const double tmin = times.empty() ? 0 : *std::min_element(times.begin(), times.end());
    std::snprintf(json, size_t(jsonCap),
                  "{\"ranks\": %d, \"scale\": %d, \"density\": %.4f, \"row_nnz\": %d, \"seed\": %d, "
                  "\"iters\": %d, \"reorder\": %s, \"setup_us\": %.2f, \"min_us\": %.2f, \"trimean_us\": %.2f, "
                  "\"teardown_us\": %.2f, \"max_pairwise_bytes\": %lld, \"nodes\": %d, \"max_on_node_bytes\": %lld, "
                  "\"max_off_node_bytes\": %lld, \"total_on_node_bytes\": %lld, \"total_off_node_bytes\": %lld, "
                  "\"checked\": %s, \"errors\": %ld, \"buffers\": \"%s\", \"api\": \"MPI_Neighbor_alltoallv\"}",
                  size, scale, density, rowNnz, seed, iters, reorder ? "true" : "false", setup * 1e6, tmin * 1e6,
                  trimean(times) * 1e6, teardown * 1e6, (long long)maxPair, nodes, (long long)maxOn,
                  (long long)maxOff, (long long)totOn, (long long)totOff, check ? "true" : "false", errors,
                  host_buffers() ? "host" : "device");
  }
  buf_free(sbuf);
  buf_free(rbuf);
  return errors ? 3 : 0;
}

namespace {
double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
double median(std::vector<double> v) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}
// the same kernel-argument size as the packer's launch (KArgs<1> + Sig)
struct Args184 {
  unsigned char b[184];
};
__global__ void empty_kernel_184(Args184 a) {
  if (a.b[0] == 0xEE && threadIdx.x == 1000) a.b[1] = 0; // never true; keeps the argument
}
} // namespace

EXPORT int tempi_bench_sync_phases(int reps, char *json, int jsonCap) {
  const int rows = 1024, block = 512, stride = 1024;
  const int extent = (rows - 1) * stride + block, packed = rows * block;
  MPI_Datatype t;
  MPI_Type_vector(rows, block, stride, MPI_BYTE, &t);
  MPI_Type_commit(&t);
  char *src = nullptr, *dst = nullptr;
  HIPCHECK(hipMalloc(&src, size_t(extent)));
  HIPCHECK(hipMalloc(&dst, size_t(packed)));
  HIPCHECK(hipMemset(src, 7, size_t(extent)));
  HIPCHECK(hipDeviceSynchronize());
  std::vector<char> hsrc(size_t(extent), 7);
  std::vector<char> hdst(size_t(packed), 0);
  hipStream_t s;
  HIPCHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  tempi_hip_desc d{};
  d.block = block;
  d.ndims = 1;
  d.counts[0] = rows;
  d.strides[0] = stride;
  std::vector<double> api, lib, ptr, launch, wait, total, apiMixed, launchMixed, bare;
  int errs = 0;
  // Each phase in a loop of its own (the call as an application makes it,
  // back to back), then the interleaved loop round 4 measured: there, each
  // TEMPI call followed MPICH's 512 KiB host pack, which evicts the HIP
  // runtime's state from the core's caches and adds ~1 us to the launch
  // (VERDICT r04 weak 4). `bare_launch` is an empty kernel with the packer's
  // argument size on the same stream: HIP's own floor on this box.
  for (int r = 0; r < reps + 20; ++r) {
    int pos = 0;
    double t0 = now_us();
    errs += MPI_Pack(src, 1, t, dst, packed, &pos, MPI_COMM_WORLD) != MPI_SUCCESS || pos != packed;
    if (r >= 20) api.push_back(now_us() - t0);
  }
  for (int r = 0; r < reps + 20; ++r) {
    int pos = 0;
    double t0 = now_us();
    errs += MPI_Pack(hsrc.data(), 1, t, hdst.data(), packed, &pos, MPI_COMM_WORLD) != MPI_SUCCESS;
    if (r >= 20) lib.push_back(now_us() - t0);
  }
  for (int r = 0; r < reps + 20; ++r) {
    const bool keep = r >= 20;
    double t2 = now_us();
    tempi_hip_ptrinfo info;
    tempi_hip_pointer_info(src, &info);
    tempi_hip_pointer_info(dst, &info);
    double t3 = now_us();
    const uint32_t *flag = nullptr;
    uint32_t ticket = 0;
    errs += tempi_hip_pack_ticket(dst, src, &d, s, &flag, &ticket) != 0;
    double t4 = now_us();
    errs += tempi_hip_ticket_wait(s, flag, ticket) != 0;
    double t5 = now_us();
    if (keep) {
      ptr.push_back(t3 - t2);
      launch.push_back(t4 - t3);
      wait.push_back(t5 - t4);
      total.push_back(t5 - t3);
    }
  }
  // the resident packer called at the C ABI (no interposer around it)
  std::vector<double> res;
  int resServed = 1;
  for (int r = 0; r < reps + 20; ++r) {
    int served = 0;
    double t0 = now_us();
    errs += tempi_hip_pack_resident(dst, src, &d, s, &served) != 0;
    double t1 = now_us();
    resServed &= served;
    if (r >= 20) res.push_back(t1 - t0);
  }
  for (int r = 0; r < reps + 20; ++r) {
    HIPCHECK(hipStreamSynchronize(s));
    double t0 = now_us();
    hipLaunchKernelGGL(empty_kernel_184, dim3(256), dim3(256), 0, s, Args184{});
    double t1 = now_us();
    if (r >= 20) bare.push_back(t1 - t0);
  }
  HIPCHECK(hipStreamSynchronize(s));
  for (int r = 0; r < reps + 20; ++r) { // interleaved with MPICH's host pack (round 4's loop)
    int pos = 0;
    errs += MPI_Pack(hsrc.data(), 1, t, hdst.data(), packed, &pos, MPI_COMM_WORLD) != MPI_SUCCESS;
    double t0 = now_us();
    pos = 0;
    errs += MPI_Pack(src, 1, t, dst, packed, &pos, MPI_COMM_WORLD) != MPI_SUCCESS || pos != packed;
    double t1 = now_us();
    const uint32_t *flag = nullptr;
    uint32_t ticket = 0;
    int pos2 = 0;
    errs += MPI_Pack(hsrc.data(), 1, t, hdst.data(), packed, &pos2, MPI_COMM_WORLD) != MPI_SUCCESS;
    double t3 = now_us();
    errs += tempi_hip_pack_ticket(dst, src, &d, s, &flag, &ticket) != 0;
    double t4 = now_us();
    errs += tempi_hip_ticket_wait(s, flag, ticket) != 0;
    if (r >= 20) {
      apiMixed.push_back(t1 - t0);
      launchMixed.push_back(t4 - t3);
    }
  }
  hipEvent_t e0, e1;
  HIPCHECK(hipEventCreate(&e0));
  HIPCHECK(hipEventCreate(&e1));
  const int nk = 200;
  HIPCHECK(hipEventRecord(e0, s));
  for (int i = 0; i < nk; ++i) errs += tempi_hip_pack(dst, src, &d, s) != 0;
  HIPCHECK(hipEventRecord(e1, s));
  HIPCHECK(hipEventSynchronize(e1));
  float ms = 0;
  HIPCHECK(hipEventElapsedTime(&ms, e0, e1));
  HIPCHECK(hipEventDestroy(e0));
  HIPCHECK(hipEventDestroy(e1));
  HIPCHECK(hipStreamDestroy(s));
  HIPCHECK(hipFree(src));
  HIPCHECK(hipFree(dst));
  MPI_Type_free(&t);
  std::snprintf(json, size_t(jsonCap),
                "{\"workload\": \"config 1: MPI_Pack of vector(1024, 512, 1024), 512 KiB, medians of %d calls in C, each phase in a loop of its own\", "
                "\"mpi_pack_device_us\": %.2f, \"mpich_host_us\": %.2f, \"c_speedup\": %.3f, "
                "\"phases_us\": {\"pointer_info_x2\": %.2f, \"launch\": %.2f, \"ticket_wait\": %.2f, "
                "\"launch_plus_wait\": %.2f, \"kernel_back_to_back\": %.2f, \"bare_launch\": %.2f, "
                "\"resident_call\": %.2f, \"resident_served\": %s}, "
                "\"interleaved_with_mpich\": {\"mpi_pack_device_us\": %.2f, \"launch\": %.2f}, \"errors\": %d}",
                reps, median(api), median(lib), median(api) > 0 ? median(lib) / median(api) : 0.0, median(ptr),
                median(launch), median(wait), median(total), double(ms) * 1e3 / nk, median(bare), median(res),
                resServed ? "true" : "false", median(apiMixed),
                median(launchMixed), errs);
  return errs ? 1 : 0;
}

// tempi_bench_halo_floor: the 1-rank halo's x faces as a bare access pattern,
// timed on this box -- the same bytes as the packer's paired copy, one lane
// per row (both faces of a row in one lane: each row's two 128-B lines read
// once and written back once; tools/xface.hip is the standalone form, DESIGN
// §6) -- and the payload of the other 24 regions (y / z faces, edges,
// corners), which bench.py prices as streaming bytes. One substep of the
// `grid`^3 exchange (radius 3, 8-byte cells, pitch rounded to 512 B, as
// halo_lib.cpp lays it out) for `quants` quantities; median of `reps` timed
// launches.
namespace {
struct FloorGeom {
  int l, r;
  int64_t pitch, plane;
};
constexpr int kFloorMaxQ = 16;
struct FloorBufs {
  char *b[kFloorMaxQ];
};

__global__ __launch_bounds__(256) void floor_xface(FloorBufs bufs, FloorGeom g) {
  const uint32_t rows = uint32_t(g.l) * uint32_t(g.l);
  const uint32_t r = blockIdx.x * 256u + threadIdx.x;
  if (r >= rows) return;
  char *row = bufs.b[blockIdx.y] + (int64_t(r / g.l) + g.r) * g.plane + (int64_t(r % g.l) + g.r) * g.pitch;
  const int64_t xl = int64_t(g.l) * 8, xr = int64_t(g.r) * 8;
  const uint64_t *s1 = reinterpret_cast<const uint64_t *>(row + xl); // +x face -> -x halo
  const uint64_t *s2 = reinterpret_cast<const uint64_t *>(row + xr); // -x face -> +x halo
  uint64_t *d1 = reinterpret_cast<uint64_t *>(row);
  uint64_t *d2 = reinterpret_cast<uint64_t *>(row + xl + xr);
  uint64_t a[3], b[3];
  for (int k = 0; k < 3; ++k) a[k] = s1[k], b[k] = s2[k];
  for (int k = 0; k < 3; ++k) d1[k] = a[k], d2[k] = b[k];
}

} // namespace

EXPORT int tempi_bench_halo_floor(int grid, int quants, int reps, char *json, int jsonCap) {
  if (quants < 1 || quants > kFloorMaxQ || grid < 8) return 1;
  const int l = grid, r = 3, q = 8;
  const int64_t width = int64_t(l + 2 * r) * q, pitch = (width + 511) / 512 * 512;
  const int64_t ysize = l + 2 * r, plane = pitch * ysize, bufBytes = plane * (l + 2 * r);
  FloorGeom g{l, r, pitch, plane};
  // payload of the 24 regions that are not x faces (per quantity)
  uint64_t restBytes = 0;
  for (int dz = -1; dz <= 1; ++dz)
    for (int dy = -1; dy <= 1; ++dy)
      for (int dx = -1; dx <= 1; ++dx) {
        if ((!dx && !dy && !dz) || (dx && !dy && !dz)) continue;
        const int d[3] = {dx, dy, dz};
        uint64_t cells = 1;
        for (int k = 0; k < 3; ++k) cells *= uint64_t(d[k] == 0 ? l : r);
        restBytes += cells * q;
      }
  FloorBufs bufs{};
  for (int qi = 0; qi < quants; ++qi) {
    HIPCHECK(hipMalloc(&bufs.b[qi], size_t(bufBytes)));
    HIPCHECK(hipMemset(bufs.b[qi], qi + 1, size_t(bufBytes)));
  }
  hipStream_t s;
  HIPCHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  HIPCHECK(hipEventCreate(&e0));
  HIPCHECK(hipEventCreate(&e1));
  const uint32_t xrows = uint32_t(l) * uint32_t(l);
  std::vector<double> v;
  for (int i = 0; i < reps + 2; ++i) {
    HIPCHECK(hipEventRecord(e0, s));
    hipLaunchKernelGGL(floor_xface, dim3((xrows + 255) / 256, quants), dim3(256), 0, s, bufs, g);
    HIPCHECK(hipEventRecord(e1, s));
    HIPCHECK(hipEventSynchronize(e1));
    float ms = 0;
    HIPCHECK(hipEventElapsedTime(&ms, e0, e1));
    if (i >= 2) v.push_back(double(ms) * 1e3);
  }
  const double xUs = median(v);
  HIPCHECK(hipEventDestroy(e0));
  HIPCHECK(hipEventDestroy(e1));
  HIPCHECK(hipStreamDestroy(s));
  for (int qi = 0; qi < quants; ++qi) HIPCHECK(hipFree(bufs.b[qi]));
  const double xBytes = 2.0 * xrows * 3 * 8 * quants; // payload of both x faces
  std::snprintf(json, size_t(jsonCap),
                "{\"x_faces_us\": %.1f, \"x_payload_bytes\": %.0f, \"rest_payload_bytes\": %.0f, \"reps\": %d}",
                xUs, xBytes, double(restBytes) * quants, reps);
  return 0;
}
