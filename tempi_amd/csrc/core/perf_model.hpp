// tempi_amd/csrc/core/perf_model.hpp -- the measured system model that drives
// AUTO method selection, stored as perf.json in TEMPI_CACHE_DIR.
//
// Same schema and interpolation rules as the reference
// (/root/reference/include/measure_system.hpp:20-103,
//  /root/reference/src/internal/measure_system.cpp:31-56 keys,
//  :184-205 interp_time_opt, :217-293 interp_2d_opt), so a perf.json is
// interchangeable; the key "cudaKernelLaunch" keeps its name (on MI355X it is
// the HIP launch latency). Differences:
//  * interp_2d_opt never reads past the table (the reference indexes a[yi2]
//    before checking yi2 < a.size(): SURVEY F11); results for in-table and
//    beyond-table queries are otherwise identical (tests/test_perf_model.py
//    replays the reference's known-answer values);
//  * the model adds the MI355X IPC method: pack on device + a descriptor
//    message + unpack reading the peer over xGMI, priced with the
//    intra-node GPU-GPU ping-pong curve that tools/measure_system measures
//    through TEMPI's own IPC path.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace tempi {

struct IidTime {
  double time = 0; // seconds
  bool iid = false;
};

struct SystemPerformance {
  double cudaKernelLaunch = 0;
  // vec[i]: 2^i bytes
  std::vector<IidTime> intraNodeCpuCpuPingpong, intraNodeGpuGpuPingpong;
  std::vector<IidTime> interNodeCpuCpuPingpong, interNodeGpuGpuPingpong;
  std::vector<IidTime> d2h, h2d;
  // vec[i][j]: 2^(2i+6) bytes in blocks of 2^j bytes (stride 512)
  std::vector<std::vector<IidTime>> packDevice, unpackDevice, packHost, unpackHost;

  bool empty() const;
};

// value or "unknown"
struct Opt {
  bool ok = false;
  double v = 0;
  static Opt none() { return Opt(); }
  static Opt of(double x) {
    Opt o;
    o.ok = true;
    o.v = x;
    return o;
  }
};

Opt interp_time_opt(const std::vector<IidTime> &a, int64_t bytes);
double interp_time(const std::vector<IidTime> &a, int64_t bytes); // +inf when unknown
Opt interp_2d_opt(const std::vector<std::vector<IidTime>> &a, int64_t bytes, int64_t blockLength);
double interp_2d(const std::vector<std::vector<IidTime>> &a, int64_t bytes, int64_t blockLength);

// end-to-end models of one strided message (seconds); unknown when a curve
// is missing
Opt model_oneshot(const SystemPerformance &sp, bool colocated, int64_t bytes, int64_t blockLength);
Opt model_device(const SystemPerformance &sp, bool colocated, int64_t bytes, int64_t blockLength,
                 bool viaTempi = false);
Opt model_staged(const SystemPerformance &sp, bool colocated, int64_t bytes, int64_t blockLength);

// the smallest message size from which IPC beats ONESHOT for non-blocking
// sends of blocks of `blockLength` bytes, priced per batch (perf_model.cpp);
// INT64_MAX: never, -1: unknown (a curve missing)
int64_t batch_ipc_threshold(const SystemPerformance &sp, int64_t blockLength);

std::string to_json(const SystemPerformance &sp);
bool from_json(const std::string &text, SystemPerformance *sp, std::string *err);

// TEMPI_CACHE_DIR/perf.json
bool import_system_performance(SystemPerformance *sp);
bool export_system_performance(const SystemPerformance &sp);

extern SystemPerformance systemPerformance;
extern bool systemPerformanceLoaded;
extern std::string systemPerformanceSource; // the file AUTO's model came from ("" = built-in policy)
extern bool systemPerformanceNode;          // ... and it is this node's own TEMPI_CACHE_DIR/perf.json

} // namespace tempi
