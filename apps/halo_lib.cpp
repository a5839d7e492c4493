// apps/halo_exchange.cpp -- 3D halo exchange through MPI_Isend / MPI_Irecv /
// MPI_Wait on device buffers with subarray datatypes (config 4).
//
// Workload of the reference's bench_isir (/root/reference/bin/
// bench_halo_exchange.cpp:666-949): a global X*Y*Z grid of nQuants 8-byte
// quantities, radius 3, 26 neighbours, periodic, decomposed by recursive
// bisection over the prime factors of the rank count (:679-704), pitched
// allocations (pitch = bytes rounded up to 512, :727-733), one interior and
// one exterior MPI_Type_create_subarray per direction (:87-168), 3 substeps
// per iteration, time = max over ranks per iteration, trimean over iterations.
//
// Two deliberate differences: (1) a receive for the exterior halo on side d
// is matched with the neighbour's send of ITS interior toward -d (tag =
// direction code of the sender's send + 26 * quantity); the reference matches
// by list position, which guarantees only equal sizes. (2) --check verifies
// every halo byte against the value the owning rank wrote.
//
// --reorder: the ranks are first placed by MPI_Dist_graph_create_adjacent
// (reorder = 1, bytes per edge as weights), and every rank plays the rank it
// is given on that communicator (Isend/Irecv, or --neighbor on the graph).
//
// --neighbor: the same exchange as one MPI_Neighbor_alltoallw per quantity
// on an MPI_Dist_graph_create_adjacent communicator (26 out-edges toward each
// direction d, 26 in-edges from the neighbour at -d; repeated edges between
// the same pair match in edge order, which this ordering makes exact).
//
// Library form: tempi_bench_halo() (libtempi_apps.so), called by bench.py
// inside the driver's torch.distributed launch; the CLI wrapper is
// apps/halo_exchange_main.cpp:
//   halo_exchange ITERS X [Y Z] [--quants N] [--radius R] [--check] [--neighbor] [--reorder]
// Result: one JSON object (rank 0).
#include <hip/hip_runtime.h>
#include <mpi.h>

#include "tempi_ext.h"

#include <algorithm>
#include <cmath>
#include <cstdint>
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

struct I3 {
  int x, y, z;
};

static std::vector<int> prime_factors(int n) {
  std::vector<int> r;
  while (n % 2 == 0) {
    r.push_back(2);
    n /= 2;
  }
  for (int i = 3; i * i <= n; i += 2)
    while (n % i == 0) {
      r.push_back(i);
      n /= i;
    }
  if (n > 2) r.push_back(n);
  std::sort(r.begin(), r.end(), [](int a, int b) { return b < a; });
  return r;
}

static int dir_code(int dx, int dy, int dz) { // 0..26, 13 = centre
  return (dz + 1) * 9 + (dy + 1) * 3 + (dx + 1);
}

// the 8-byte value a rank writes for global cell (x, y, z) of quantity q
__host__ __device__ static inline uint64_t cell_value(int64_t x, int64_t y, int64_t z, int q) {
  uint64_t h = uint64_t(x) * 0x9E3779B97F4A7C15ull ^ uint64_t(y) * 0xC2B2AE3D27D4EB4Full ^
               uint64_t(z) * 0x165667B19E3779F9ull ^ uint64_t(q + 1) * 0x27D4EB2F165667C5ull;
  h ^= h >> 29;
  return h * 0xBF58476D1CE4E5B9ull;
}

__global__ void fill_kernel(uint64_t *buf, size_t pitchWords, int ysize, I3 lcr, I3 origin, I3 global, int r,
                            int q) {
  // interior only; the halo starts as a sentinel
  const int64_t n = int64_t(lcr.x) * lcr.y * lcr.z;
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    const int x = int(i % lcr.x), y = int((i / lcr.x) % lcr.y), z = int(i / (int64_t(lcr.x) * lcr.y));
    const int64_t gx = origin.x + x, gy = origin.y + y, gz = origin.z + z;
    buf[(size_t(z + r) * ysize + size_t(y + r)) * pitchWords + size_t(x + r)] = cell_value(gx, gy, gz, q);
  }
}

// --check on the GPU: every cell of the padded block (interior and all 26 halo
// regions, with periodic wrap) against the owner's value; one mismatch count
// per workgroup, summed on the host
constexpr int kCheckBlock = 256, kCheckGrid = 2048;
__global__ void __launch_bounds__(kCheckBlock) check_kernel(const uint64_t *buf, size_t pitchWords, int ysize,
                                                            int zsize, int xsize, I3 origin, I3 global, int r, int q,
                                                            unsigned long long *blockErrors) {
  const int64_t n = int64_t(xsize) * ysize * zsize;
  unsigned long long bad = 0;
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    const int x = int(i % xsize), y = int((i / xsize) % ysize), z = int(i / (int64_t(xsize) * ysize));
    const int64_t gx = (origin.x + x - r + global.x) % global.x;
    const int64_t gy = (origin.y + y - r + global.y) % global.y;
    const int64_t gz = (origin.z + z - r + global.z) % global.z;
    bad += buf[(size_t(z) * ysize + size_t(y)) * pitchWords + size_t(x)] != cell_value(gx, gy, gz, q);
  }
  __shared__ unsigned long long part[kCheckBlock];
  part[threadIdx.x] = bad;
  __syncthreads();
  for (int s = kCheckBlock / 2; s > 0; s >>= 1) {
    if (int(threadIdx.x) < s) part[threadIdx.x] += part[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) blockErrors[blockIdx.x] = part[0];
}

// TEMPI_BENCH_HOST=1: the same exchange on pageable host memory -- the
// library path the reference takes for host buffers. With TEMPI_DISABLE=1 it
// is the host MPI's own strided Isend / Irecv: bench.py's CPU baseline.
static bool host_buffers() {
  const char *e = std::getenv("TEMPI_BENCH_HOST");
  return e && *e && *e != '0';
}

// TEMPI's own entry points, when the interposer is linked (weak: the app runs
// unchanged on a plain MPI)
extern "C" __attribute__((weak)) void tempi_reset_counters(void);
extern "C" __attribute__((weak)) void tempi_get_counters(tempi_counters_t *out);

static double trimean(std::vector<double> v) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  auto pct = [&](double p) {
    const double idx = p * double(v.size() - 1);
    const size_t lo = size_t(std::floor(idx)), hi = size_t(std::ceil(idx));
    return v[lo] + (v[hi] - v[lo]) * (idx - double(lo));
  };
  return (pct(0.25) + 2 * pct(0.5) + pct(0.75)) / 4;
}

extern "C" __attribute__((visibility("default"))) int
tempi_bench_halo(int nIters, int gx, int gy, int gz, int nQuants, int radius, int check, int neighbor,
                 int setDevice, char *json, int jsonCap) {
  int rank, size;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &size);
  const int worldRank = rank; // (--reorder may give this process another rank)
  I3 global{gx, gy, gz};

  // one GPU per rank on the node (ranks beyond the GPU count share)
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0; // (host buffers need no GPU)
  if (setDevice && ndev > 0) {
    MPI_Comm node;
    MPI_Comm_split_type(MPI_COMM_WORLD, MPI_COMM_TYPE_SHARED, rank, MPI_INFO_NULL, &node);
    int lr;
    MPI_Comm_rank(node, &lr);
    HIPCHECK(hipSetDevice(lr % ndev));
    MPI_Comm_free(&node);
  }

  // recursive bisection (/root/reference/bin/bench_halo_exchange.cpp:679-704)
  I3 lcr = global, dims{1, 1, 1};
  for (int f : prime_factors(size)) {
    if (lcr.z >= lcr.y && lcr.z >= lcr.x) {
      lcr.z /= f;
      dims.z *= f;
    } else if (lcr.y >= lcr.x) {
      lcr.y /= f;
      dims.y *= f;
    } else {
      lcr.x /= f;
      dims.x *= f;
    }
  }
  auto coords = [&](int r) { return I3{r % dims.x, (r / dims.x) % dims.y, r / (dims.x * dims.y)}; };
  auto nbr_of = [&](I3 m, int dx, int dy, int dz) {
    const I3 n{(m.x + dx + dims.x) % dims.x, (m.y + dy + dims.y) % dims.y, (m.z + dz + dims.z) % dims.z};
    return n.x + n.y * dims.x + n.z * dims.x * dims.y;
  };

  // --reorder (neighbor & 2): the graph is created first, with reorder = 1
  // and each edge's bytes as its weight, and this process then plays the
  // rank it is given, as the reference's bench does
  // (bench_halo_exchange.cpp:343-360); with TEMPI_PLACEMENT_* and several
  // nodes TEMPI's placement chooses that rank
  const bool reorder = (neighbor & 2) != 0;
  MPI_Comm comm = MPI_COMM_WORLD, graph = MPI_COMM_NULL;
  if (reorder) {
    const I3 w = coords(rank);
    std::vector<int> in, out, inW, outW;
    for (int dz = -1; dz <= 1; ++dz)
      for (int dy = -1; dy <= 1; ++dy)
        for (int dx = -1; dx <= 1; ++dx) {
          if (!dx && !dy && !dz) continue;
          const int bytes = (dx ? radius : lcr.x) * (dy ? radius : lcr.y) * (dz ? radius : lcr.z) * 8 * nQuants;
          out.push_back(nbr_of(w, dx, dy, dz));
          in.push_back(nbr_of(w, -dx, -dy, -dz));
          outW.push_back(bytes);
          inW.push_back(bytes);
        }
    MPI_Dist_graph_create_adjacent(MPI_COMM_WORLD, int(in.size()), in.data(), inW.data(), int(out.size()),
                                   out.data(), outW.data(), MPI_INFO_NULL, 1, &graph);
    MPI_Comm_rank(graph, &rank);
    comm = graph;
  }
  const I3 me = coords(rank);
  const I3 origin{me.x * lcr.x, me.y * lcr.y, me.z * lcr.z};
  const int q = 8; // bytes per quantity
  const size_t width = size_t(lcr.x + 2 * radius) * q;
  const size_t pitch = (width + 511) / 512 * 512;
  const int ysize = lcr.y + 2 * radius, zsize = lcr.z + 2 * radius;
  const size_t bufBytes = pitch * size_t(ysize) * size_t(zsize);

  std::vector<char *> bufs(static_cast<size_t>(nQuants));
  const bool onHost = host_buffers();
  for (int qi = 0; qi < nQuants; ++qi) {
    if (onHost) {
      bufs[size_t(qi)] = static_cast<char *>(std::aligned_alloc(4096, (bufBytes + 4095) / 4096 * 4096));
      std::memset(bufs[size_t(qi)], 0xEE, bufBytes);
      uint64_t *b = reinterpret_cast<uint64_t *>(bufs[size_t(qi)]);
      for (int z = 0; z < lcr.z; ++z)
        for (int y = 0; y < lcr.y; ++y)
          for (int x = 0; x < lcr.x; ++x)
            b[(size_t(z + radius) * ysize + size_t(y + radius)) * (pitch / 8) + size_t(x + radius)] =
                cell_value(origin.x + x, origin.y + y, origin.z + z, qi);
      continue;
    }
    HIPCHECK(hipMalloc(&bufs[size_t(qi)], bufBytes));
    HIPCHECK(hipMemset(bufs[size_t(qi)], 0xEE, bufBytes));
    hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, 0, reinterpret_cast<uint64_t *>(bufs[size_t(qi)]),
                       pitch / 8, ysize, lcr, origin, global, radius, qi);
  }
  if (!onHost) HIPCHECK(hipDeviceSynchronize());

  struct Dir {
    int dx, dy, dz, nbr;
    MPI_Datatype interior, exterior;
    int bytes;
  };
  std::vector<Dir> dirs;
  auto halo_type = [&](int dx, int dy, int dz, bool exterior) {
    const int d[3] = {dx, dy, dz};
    const int l[3] = {lcr.x, lcr.y, lcr.z};
    int p[3], e[3];
    for (int k = 0; k < 3; ++k) {
      if (d[k] == -1)
        p[k] = exterior ? 0 : radius;
      else if (d[k] == 1)
        p[k] = l[k] + (exterior ? radius : 0);
      else
        p[k] = radius;
      e[k] = d[k] == 0 ? l[k] : radius;
    }
    int sizes[3] = {p[2] + e[2], ysize, int(pitch)};
    int subs[3] = {e[2], e[1], e[0] * q};
    int starts[3] = {p[2], p[1], p[0] * q};
    MPI_Datatype t;
    MPI_Type_create_subarray(3, sizes, subs, starts, MPI_ORDER_C, MPI_BYTE, &t);
    MPI_Type_commit(&t);
    return t;
  };
  for (int dz = -1; dz <= 1; ++dz)
    for (int dy = -1; dy <= 1; ++dy)
      for (int dx = -1; dx <= 1; ++dx) {
        if (!dx && !dy && !dz) continue;
        Dir D{dx, dy, dz, nbr_of(me, dx, dy, dz), halo_type(dx, dy, dz, false), halo_type(dx, dy, dz, true), 0};
        MPI_Type_size(D.interior, &D.bytes);
        dirs.push_back(D);
      }

  // per-peer traffic for the xGMI roofline
  std::vector<double> peerBytes(size_t(size), 0);
  double bytesPerIter = 0;
  for (const Dir &D : dirs) {
    bytesPerIter += double(D.bytes) * nQuants * 3;
    if (D.nbr != rank) peerBytes[size_t(D.nbr)] += double(D.bytes) * nQuants * 3;
  }
  const double maxLink = *std::max_element(peerBytes.begin(), peerBytes.end());

  // neighbourhood form: out-edge i toward dirs[i], in-edge i from the
  // neighbour at -dirs[i] (whose send toward dirs[i] fills exterior(-dirs[i]))
  std::vector<int> nbrIn, nbrOut, ncount(dirs.size(), 1);
  long long graphErrors = 0; // the placed graph's neighbours against this rank's own
  std::vector<MPI_Aint> ndispl(dirs.size(), 0);
  std::vector<MPI_Datatype> nsend, nrecv;
  if (neighbor & 1) {
    for (const Dir &D : dirs) {
      nbrOut.push_back(D.nbr);
      nsend.push_back(D.interior);
      for (const Dir &E : dirs)
        if (E.dx == -D.dx && E.dy == -D.dy && E.dz == -D.dz) {
          nbrIn.push_back(E.nbr);
          nrecv.push_back(E.exterior);
        }
    }
    if (!reorder)
      MPI_Dist_graph_create_adjacent(MPI_COMM_WORLD, int(nbrIn.size()), nbrIn.data(), MPI_UNWEIGHTED,
                                     int(nbrOut.size()), nbrOut.data(), MPI_UNWEIGHTED, MPI_INFO_NULL, 0, &graph);
  }
  if (reorder) {
    std::vector<int> gin(dirs.size()), gout(dirs.size()), gw(dirs.size());
    MPI_Dist_graph_neighbors(graph, int(dirs.size()), gin.data(), gw.data(), int(dirs.size()), gout.data(),
                             gw.data());
    for (size_t i = 0; i < dirs.size(); ++i) {
      graphErrors += gout[i] != dirs[i].nbr;
      graphErrors += gin[i] != nbr_of(me, -dirs[i].dx, -dirs[i].dy, -dirs[i].dz);
    }
  }

  std::vector<double> times;
  std::vector<MPI_Request> reqs(dirs.size() * 2 * size_t(nQuants));
  const int warm = 1;
  double tIsend = 0, tIrecv = 0, tWait = 0;
  for (int it = 0; it < nIters + warm; ++it) {
    if (it == warm) {
      if (tempi_reset_counters) tempi_reset_counters();
      tIsend = tIrecv = tWait = 0;
    }
    double exch = 0;
    for (int sub = 0; sub < 3; ++sub) {
      MPI_Barrier(MPI_COMM_WORLD);
      const double t0 = MPI_Wtime();
      if (neighbor & 1) {
        for (int qi = 0; qi < nQuants; ++qi)
          MPI_Neighbor_alltoallw(bufs[size_t(qi)], ncount.data(), ndispl.data(), nsend.data(), bufs[size_t(qi)],
                                 ncount.data(), ndispl.data(), nrecv.data(), graph);
        const double t3 = MPI_Wtime();
        tWait += t3 - t0;
        exch += t3 - t0;
        continue;
      }
      size_t ri = 0;
      for (int qi = 0; qi < nQuants; ++qi)
        for (const Dir &D : dirs)
          MPI_Isend(bufs[size_t(qi)], 1, D.interior, D.nbr, dir_code(D.dx, D.dy, D.dz) + 27 * qi, comm, &reqs[ri++]);
      const double t1 = MPI_Wtime();
      for (int qi = 0; qi < nQuants; ++qi)
        for (const Dir &D : dirs)
          MPI_Irecv(bufs[size_t(qi)], 1, D.exterior, D.nbr, dir_code(-D.dx, -D.dy, -D.dz) + 27 * qi, comm,
                    &reqs[ri++]);
      const double t2 = MPI_Wtime();
      for (MPI_Request &r : reqs) MPI_Wait(&r, MPI_STATUS_IGNORE);
      const double t3 = MPI_Wtime();
      tIsend += t1 - t0;
      tIrecv += t2 - t1;
      tWait += t3 - t2;
      exch += t3 - t0;
    }
    MPI_Allreduce(MPI_IN_PLACE, &exch, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
    if (it >= warm) times.push_back(exch);
  }

  long long errors = graphErrors;
  if (check) {
    // check == 2: a negative control -- one planted wrong cell (rank 0,
    // quantity 0, the halo corner at (0, 0, 0)) must be counted
    if (check == 2 && rank == 0) {
      if (onHost)
        std::memset(bufs[0], 0x5A, 8);
      else
        HIPCHECK(hipMemset(bufs[0], 0x5A, 8));
    }
    if (onHost) {
      const int xsize = lcr.x + 2 * radius;
      for (int qi = 0; qi < nQuants; ++qi) {
        const uint64_t *b = reinterpret_cast<const uint64_t *>(bufs[size_t(qi)]);
        for (int z = 0; z < zsize; ++z)
          for (int y = 0; y < ysize; ++y)
            for (int x = 0; x < xsize; ++x) {
              const int64_t gx = (origin.x + x - radius + global.x) % global.x;
              const int64_t gy = (origin.y + y - radius + global.y) % global.y;
              const int64_t gz = (origin.z + z - radius + global.z) % global.z;
              errors += b[(size_t(z) * ysize + size_t(y)) * (pitch / 8) + size_t(x)] != cell_value(gx, gy, gz, qi);
            }
      }
    } else {
      unsigned long long *dErr = nullptr;
      HIPCHECK(hipMalloc(&dErr, sizeof(unsigned long long) * kCheckGrid));
      std::vector<unsigned long long> hErr(kCheckGrid);
      for (int qi = 0; qi < nQuants; ++qi) {
        hipLaunchKernelGGL(check_kernel, dim3(kCheckGrid), dim3(kCheckBlock), 0, 0,
                           reinterpret_cast<const uint64_t *>(bufs[size_t(qi)]), pitch / 8, ysize, zsize,
                           lcr.x + 2 * radius, origin, global, radius, qi, dErr);
        HIPCHECK(hipMemcpy(hErr.data(), dErr, sizeof(unsigned long long) * kCheckGrid, hipMemcpyDeviceToHost));
        for (unsigned long long e : hErr) errors += (long long)e;
      }
      HIPCHECK(hipFree(dErr));
    }
  }
  MPI_Allreduce(MPI_IN_PLACE, &errors, 1, MPI_LONG_LONG, MPI_SUM, MPI_COMM_WORLD);

  double maxLinkAll = maxLink;
  MPI_Allreduce(MPI_IN_PLACE, &maxLinkAll, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
  double totalBytes = bytesPerIter;
  MPI_Allreduce(MPI_IN_PLACE, &totalBytes, 1, MPI_DOUBLE, MPI_SUM, MPI_COMM_WORLD);
  // the SURVEY 8(d) aggregate-xGMI form: bytes that leave a rank, over the
  // directed (sender, receiver) GPU pairs that carry any
  double remote[2] = {0, 0}; // bytes to other ranks, directed links used
  for (double b : peerBytes)
    if (b > 0) {
      remote[0] += b;
      remote[1] += 1;
    }
  MPI_Allreduce(MPI_IN_PLACE, remote, 2, MPI_DOUBLE, MPI_SUM, MPI_COMM_WORLD);
  const double tIter = trimean(times);
  // the GPU's busy time by TEMPI's own account (a transport batch in flight),
  // so that the line splits an iteration into GPU work and host-only time
  double inflightUs = -1;
  if (tempi_get_counters) {
    tempi_counters_t c{};
    tempi_get_counters(&c);
    inflightUs = double(c.gpu_inflight_ns) * 1e-3 / nIters;
  }
  if (worldRank == 0 && json && jsonCap > 0) {
    std::snprintf(json, size_t(jsonCap), "{\"ranks\": %d, \"global\": [%d, %d, %d], \"dims\": [%d, %d, %d], \"lcr\": [%d, %d, %d], "
                "\"quants\": %d, \"radius\": %d, \"iters\": %d, \"us_per_iter\": %.2f, \"us_min\": %.2f, "
                "\"payload_bytes_per_iter_per_rank0\": %.0f, \"total_bytes_per_iter\": %.0f, "
                "\"max_peer_bytes_per_iter\": %.0f, \"aggregate_GBps\": %.2f, \"busiest_link_GBps\": %.2f, "
                "\"remote_bytes_per_iter\": %.0f, \"links_used\": %.0f, "
                "\"checked\": %s, \"errors\": %lld, \"api\": \"%s\", \"reorder\": %s, \"buffers\": \"%s\", "
                "\"rank0_us_per_iter\": {\"isend\": %.1f, "
                "\"irecv\": %.1f, \"wait\": %.1f, \"gpu_inflight\": %.1f}}\n",
                size, global.x, global.y, global.z, dims.x, dims.y, dims.z, lcr.x, lcr.y, lcr.z, nQuants, radius,
                nIters, tIter * 1e6, *std::min_element(times.begin(), times.end()) * 1e6, bytesPerIter, totalBytes,
                maxLinkAll, totalBytes / tIter / 1e9, maxLinkAll / tIter / 1e9, remote[0], remote[1],
                check ? "true" : "false", errors,
                (neighbor & 1) ? "MPI_Neighbor_alltoallw" : "MPI_Isend/MPI_Irecv/MPI_Wait", reorder ? "true" : "false",
                onHost ? "host" : "device",
                tIsend / nIters * 1e6, tIrecv / nIters * 1e6, tWait / nIters * 1e6, inflightUs);
  }
  if (graph != MPI_COMM_NULL) MPI_Comm_free(&graph);
  for (Dir &D : dirs) {
    MPI_Type_free(&D.interior);
    MPI_Type_free(&D.exterior);
  }
  for (char *b : bufs) {
    if (onHost)
      std::free(b);
    else
      HIPCHECK(hipFree(b));
  }
  return errors ? 3 : 0;
}
