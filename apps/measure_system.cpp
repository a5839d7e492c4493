// apps/measure_system.cpp -- measure this node and write TEMPI_CACHE_DIR/
// perf.json (or --out FILE), the model AUTO method selection interpolates.
//
// Same curves and schema as the reference's measure-system
// (/root/reference/src/internal/measure_system.cu:377-606,
// /root/reference/bin/measure_system.cpp:22-32), measured the MI355X way:
//   cudaKernelLaunch          empty-kernel launch + stream sync (HIP)
//   d2h / h2d                 hipMemcpy between device and pinned host, 2^0..2^23 B
//   intraNodeCpuCpuPingpong   host-buffer MPI_Send/Recv ping-pong, one way
//   intraNodeGpuGpuPingpong   device-buffer ping-pong through TEMPI's IPC
//                             transport (the DEVICE path of this build)
//   packDevice/unpackDevice   MPI_Pack / MPI_Unpack device <-> device
//   packHost/unpackHost       MPI_Pack / MPI_Unpack device <-> pinned host
//                             (the GPU kernel writes / reads host memory)
// 2-D tables: row i = 2^(2i+6) bytes (64 B .. 4 MiB), column j = 2^j-byte
// blocks (1 .. 512 B) at stride 512. inter-node curves are measured only when
// ranks 0 and 1 are on different hosts. Each point is repeated until its
// samples pass the SP 800-90B permutation test (tempi_sp800_90b_iid) or 3
// trials elapse; the stored time is the trimean.
//
// With no GPU visible only the host curves (intraNodeCpuCpuPingpong or
// interNodeCpuCpuPingpong) are measured; the GPU curves stay empty, which the
// model reads as "unknown" (+inf), so AUTO then prices only what was measured.
//
// usage: mpiexec -n 2 measure_system [--out FILE] [--quick]
#include <hip/hip_runtime.h>
#include <mpi.h>

#include "tempi_ext.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
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

__global__ void empty_kernel() {}

struct Point {
  double time;
  bool iid;
};

static bool quick = false;

static double trimean(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  auto pct = [&](double p) {
    const double idx = p * double(v.size() - 1);
    const size_t lo = size_t(std::floor(idx)), hi = size_t(std::ceil(idx));
    return v[lo] + (v[hi] - v[lo]) * (idx - double(lo));
  };
  return (pct(0.25) + 2 * pct(0.5) + pct(0.75)) / 4;
}

// collective when `comm` is set: every rank runs the same number of samples
static Point measure(const std::function<double()> &sample, MPI_Comm comm = MPI_COMM_NULL) {
  const int minS = quick ? 5 : 10, maxS = quick ? 20 : 60, trials = quick ? 1 : 3;
  Point p{0, false};
  for (int t = 0; t < trials; ++t) {
    std::vector<double> s;
    sample(); // warm
    const double t0 = MPI_Wtime();
    while (int(s.size()) < minS || (int(s.size()) < maxS && MPI_Wtime() - t0 < 0.05)) {
      s.push_back(sample());
      if (comm != MPI_COMM_NULL) {
        int more = int(s.size()) < maxS && MPI_Wtime() - t0 < 0.05;
        if (int(s.size()) < minS) more = 1;
        MPI_Bcast(&more, 1, MPI_INT, 0, comm);
        if (!more) break;
      }
    }
    p.time = trimean(s);
    p.iid = tempi_sp800_90b_iid(s.data(), int(s.size()), 1000, 17 + uint64_t(t)) != 0;
    if (comm != MPI_COMM_NULL) {
      int ok = p.iid;
      MPI_Bcast(&ok, 1, MPI_INT, 0, comm);
      p.iid = ok;
    }
    if (p.iid) break;
  }
  return p;
}

static std::string curve_json(const std::vector<Point> &c) {
  std::string s = "[";
  char buf[96];
  for (size_t i = 0; i < c.size(); ++i) {
    std::snprintf(buf, sizeof buf, "%s{\"iid\": %s, \"time\": %.9g}", i ? ", " : "", c[i].iid ? "true" : "false",
                  c[i].time);
    s += buf;
  }
  return s + "]";
}

static std::string table_json(const std::vector<std::vector<Point>> &t) {
  std::string s = "[";
  for (size_t i = 0; i < t.size(); ++i) s += (i ? ",\n    " : "\n    ") + curve_json(t[i]);
  return s + "\n  ]";
}

int main(int argc, char **argv) {
  MPI_Init(&argc, &argv);
  int rank, size;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &size);
  std::string out;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--out")) out = argv[++i];
    if (!std::strcmp(argv[i], "--quick")) quick = true;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0;
  const bool gpu = ndev > 0;
  if (gpu) HIPCHECK(hipSetDevice(rank % ndev));
  const int maxLog = quick ? 20 : 23;

  // node placement of ranks 0 and 1
  char name[MPI_MAX_PROCESSOR_NAME] = {0}, other[MPI_MAX_PROCESSOR_NAME] = {0};
  int len;
  MPI_Get_processor_name(name, &len);
  bool colocated = true;
  if (size >= 2) {
    if (rank == 0) MPI_Recv(other, MPI_MAX_PROCESSOR_NAME, MPI_CHAR, 1, 0, MPI_COMM_WORLD, MPI_STATUS_IGNORE);
    if (rank == 1) MPI_Send(name, MPI_MAX_PROCESSOR_NAME, MPI_CHAR, 0, 0, MPI_COMM_WORLD);
    int co = rank == 0 ? !std::strcmp(name, other) : 0;
    MPI_Bcast(&co, 1, MPI_INT, 0, MPI_COMM_WORLD);
    colocated = co != 0;
  }

  std::vector<Point> d2h, h2d, cpuPP, gpuPP;
  std::vector<std::vector<Point>> packD, unpackD, packH, unpackH;
  double launch = 0;
  const size_t maxBytes = size_t(1) << maxLog;
  // the 2-D tables' strided side: vector(bytes/bl, bl, 512) spans
  // (bytes/bl - 1) * 512 + bl bytes, 2 GiB for the 4 MiB row at bl = 1
  const int maxTableLog = quick ? 18 : 22;
  const size_t tableExtent = ((size_t(1) << maxTableLog) - 1) * 512 + 1;
  const size_t devBytes = std::max(4 * maxBytes, tableExtent);
  char *dev = nullptr, *dev2 = nullptr, *host = nullptr;
  if (gpu) {
    HIPCHECK(hipMalloc(&dev, devBytes));
    HIPCHECK(hipMalloc(&dev2, 4 * maxBytes));
    HIPCHECK(hipMemset(dev, 0, devBytes));
    HIPCHECK(hipHostMalloc(reinterpret_cast<void **>(&host), 4 * maxBytes, hipHostMallocMapped));
  }
  std::vector<char> pageable(maxBytes);

  if (rank == 0 && gpu) {
    launch = measure([&] {
      const double t0 = MPI_Wtime();
      hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(1), 0, 0);
      HIPCHECK(hipDeviceSynchronize());
      return MPI_Wtime() - t0;
    }).time;
    for (int i = 0; i <= maxLog; ++i) {
      const size_t n = size_t(1) << i;
      d2h.push_back(measure([&] {
        const double t0 = MPI_Wtime();
        HIPCHECK(hipMemcpy(host, dev, n, hipMemcpyDeviceToHost));
        return MPI_Wtime() - t0;
      }));
      h2d.push_back(measure([&] {
        const double t0 = MPI_Wtime();
        HIPCHECK(hipMemcpy(dev, host, n, hipMemcpyHostToDevice));
        return MPI_Wtime() - t0;
      }));
    }
    // 2-D pack tables (device only, rank 0)
    for (int i = 0; 2 * i + 6 <= maxTableLog; ++i) {
      const int64_t bytes = int64_t(1) << (2 * i + 6);
      std::vector<Point> pd, ud, ph, uh;
      for (int j = 0; j <= 9; ++j) {
        const int bl = std::min<int64_t>(int64_t(1) << j, bytes);
        MPI_Datatype t;
        MPI_Type_vector(int(bytes / bl), bl, 512, MPI_BYTE, &t);
        MPI_Type_commit(&t);
        MPI_Aint tlb, text;
        MPI_Type_get_true_extent(t, &tlb, &text);
        if (tlb < 0 || size_t(tlb + text) > devBytes || size_t(bytes) > 4 * maxBytes) {
          std::fprintf(stderr, "internal error: table point %lld B / %d B exceeds the buffers\n", (long long)bytes, bl);
          MPI_Abort(MPI_COMM_WORLD, 3);
        }
        auto pk = [&](char *dst) {
          return [&, dst] {
            int pos = 0;
            const double t0 = MPI_Wtime();
            MPI_Pack(dev, 1, t, dst, int(bytes), &pos, MPI_COMM_SELF);
            return MPI_Wtime() - t0;
          };
        };
        auto upk = [&](char *src) {
          return [&, src] {
            int pos = 0;
            const double t0 = MPI_Wtime();
            MPI_Unpack(src, int(bytes), &pos, dev, 1, t, MPI_COMM_SELF);
            return MPI_Wtime() - t0;
          };
        };
        pd.push_back(measure(pk(dev2)));
        ud.push_back(measure(upk(dev2)));
        ph.push_back(measure(pk(host)));
        uh.push_back(measure(upk(host)));
        MPI_Type_free(&t);
      }
      packD.push_back(pd);
      unpackD.push_back(ud);
      packH.push_back(ph);
      unpackH.push_back(uh);
    }
  }

  // ping-pongs between ranks 0 and 1 (rank 0 drives the sample count)
  if (size >= 2) {
    MPI_Comm pair;
    MPI_Comm_split(MPI_COMM_WORLD, rank < 2 ? 0 : MPI_UNDEFINED, rank, &pair);
    if (rank < 2) {
      for (int onGpu = 0; onGpu < (gpu ? 2 : 1); ++onGpu) {
        if (onGpu) tempi_set_datatype_method(4); // IPC: this build's DEVICE path
        for (int i = 0; i <= maxLog; ++i) {
          const int n = 1 << i;
          char *buf = onGpu ? dev : pageable.data();
          Point p = measure(
              [&] {
                MPI_Barrier(pair);
                const double t0 = MPI_Wtime();
                if (rank == 0) {
                  MPI_Send(buf, n, MPI_BYTE, 1, 0, pair);
                  MPI_Recv(buf, n, MPI_BYTE, 1, 0, pair, MPI_STATUS_IGNORE);
                } else {
                  MPI_Recv(buf, n, MPI_BYTE, 0, 0, pair, MPI_STATUS_IGNORE);
                  MPI_Send(buf, n, MPI_BYTE, 0, 0, pair);
                }
                return (MPI_Wtime() - t0) / 2;
              },
              pair);
          (onGpu ? gpuPP : cpuPP).push_back(p);
        }
        tempi_set_datatype_method(0);
      }
      MPI_Comm_free(&pair);
    }
  }

  if (rank == 0) {
    char launchText[32]; // %.9g: std::to_string keeps 6 decimals, 0.00001 for a 10.4 us launch
    std::snprintf(launchText, sizeof launchText, "%.9g", launch);
    std::string doc = "{\n  \"cudaKernelLaunch\": " + std::string(launchText);
    doc += ",\n  \"d2h\": " + curve_json(d2h) + ",\n  \"h2d\": " + curve_json(h2d);
    doc += ",\n  \"intraNodeCpuCpuPingpong\": " + curve_json(colocated ? cpuPP : std::vector<Point>());
    doc += ",\n  \"intraNodeGpuGpuPingpong\": " + curve_json(colocated ? gpuPP : std::vector<Point>());
    doc += ",\n  \"interNodeCpuCpuPingpong\": " + curve_json(colocated ? std::vector<Point>() : cpuPP);
    doc += ",\n  \"interNodeGpuGpuPingpong\": " + curve_json(colocated ? std::vector<Point>() : gpuPP);
    doc += ",\n  \"packDevice\": " + table_json(packD) + ",\n  \"unpackDevice\": " + table_json(unpackD);
    doc += ",\n  \"packHost\": " + table_json(packH) + ",\n  \"unpackHost\": " + table_json(unpackH);
    doc += "\n}\n";
    std::vector<char> check(doc.size() * 2 + 1024);
    if (tempi_perf_roundtrip(doc.c_str(), check.data(), int(check.size())) != 0) {
      std::fprintf(stderr, "internal error: perf.json does not round-trip\n");
      MPI_Abort(MPI_COMM_WORLD, 2);
    }
    if (out.empty()) {
      const char *cd = std::getenv("TEMPI_CACHE_DIR");
      std::string dir = cd ? cd : (std::string(std::getenv("HOME") ? std::getenv("HOME") : "/tmp") + "/.tempi");
      std::string cmd = "mkdir -p '" + dir + "'";
      if (std::system(cmd.c_str()) != 0) std::fprintf(stderr, "cannot create %s\n", dir.c_str());
      out = dir + "/perf.json";
    }
    FILE *f = std::fopen(out.c_str(), "w");
    if (!f) {
      std::fprintf(stderr, "cannot write %s\n", out.c_str());
      MPI_Abort(MPI_COMM_WORLD, 2);
    }
    std::fputs(doc.c_str(), f);
    std::fclose(f);
    std::printf("{\"perf_json\": \"%s\", \"colocated\": %s, \"gpu\": %s, \"launch_us\": %.3f}\n", out.c_str(),
                colocated ? "true" : "false", gpu ? "true" : "false", launch * 1e6);
  }
  if (gpu) {
    HIPCHECK(hipFree(dev));
    HIPCHECK(hipFree(dev2));
    HIPCHECK(hipHostFree(host));
  }
  MPI_Finalize();
  return 0;
}
