// tempi_amd/csrc/core/gpu.cpp -- see gpu.hpp
#include "gpu.hpp"

#include "log.hpp"

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <link.h>
#include <mutex>
#include <set>
#include <string>
#include <unistd.h>
#include <vector>

namespace tempi {
namespace gpu {

namespace {
int nDevices = 0;
std::mutex mtx;
std::vector<void *> streams; // [device * kMaxLanes + lane]
int nLanes = 3;
// TEMPI_TEST_HOST_ONLY (CPU tests): with no GPU visible, TEMPI still takes the
// host-side paths it takes beside a GPU (descriptor-aware host receives, the
// probe family, send gates), so they can be exercised on a machine without
// one. Device pointers never occur there, so nothing reaches HIP.
bool hostOnlyTest = false;
} // namespace

int lanes() { return nLanes; }

void choose_lanes(int ranksOnNode) {
  nLanes = ranksOnNode > nDevices ? 1 : 3;
  if (const char *e = std::getenv("TEMPI_STREAMS")) nLanes = std::min(kMaxLanes, std::max(1, std::atoi(e)));
  LOG_DEBUG("stream lanes: " << nLanes);
  // The resident packer's kernel keeps a hardware queue busy while it waits
  // for calls. With more than two processes on one GPU, those queues
  // oversubscribe the scheduler, which then time-slices every process's
  // queues: the 8-rank halo on one GPU went from 4.3 to 53.6 ms/iter
  // (profiles/r06/h8_resident_s29.txt). So it is off there unless
  // TEMPI_RESIDENT asks for it.
  if (nDevices > 0 && ranksOnNode > 2 * nDevices && !std::getenv("TEMPI_RESIDENT")) {
    tempi_hip_resident_enable(0);
    LOG_DEBUG("resident packer off: " << ranksOnNode << " ranks on " << nDevices << " GPU(s)");
  }
}

bool available() { return nDevices > 0 || hostOnlyTest; }

std::vector<std::string> hip_runtimes() {
  std::set<std::string> found;
  dl_iterate_phdr(
      [](dl_phdr_info *info, size_t, void *data) -> int {
        const char *name = info->dlpi_name;
        if (name && std::strstr(name, "libamdhip64")) {
          char real[PATH_MAX];
          static_cast<std::set<std::string> *>(data)->insert(realpath(name, real) ? real : name);
        }
        return 0;
      },
      &found);
  return std::vector<std::string>(found.begin(), found.end());
}

void init() {
  int n = 0;
  if (tempi_hip_device_count(&n) != 0) n = 0;
  nDevices = n;
  hostOnlyTest = n == 0 && std::getenv("TEMPI_TEST_HOST_ONLY") != nullptr;
  {
    std::lock_guard<std::mutex> g(mtx);
    streams.assign(size_t(n) * kMaxLanes, nullptr);
    nLanes = 1; // until choose_lanes()
  }
  LOG_DEBUG("visible GPUs: " << n);
  // Two HIP runtimes in one process (a PyTorch wheel bundles its own beside
  // the ROCm one libtempi_hip.so links): each has its own
  // streams, so work the other runtime queued is not ordered with TEMPI's
  // stream, and each sees the other's pinned host allocations as device
  // memory (tools/diag_ptrattr.py, profiles/r06/diag_hostmalloc_s1.jsonl).
  // Said once, on rank 0.
  const std::vector<std::string> rt = hip_runtimes();
  if (n > 0 && rt.size() > 1 && logRank == 0) {
    std::string names;
    for (const std::string &r : rt) names += (names.empty() ? "" : ", ") + r;
    LOG_WARN(rt.size() << " HIP runtimes in this process (" << names
                       << "); TEMPI uses the one libtempi_hip.so links. Work queued through another runtime must be "
                          "complete (that runtime's synchronize) before an MPI call reads or writes its buffers "
                          "(INTEGRATION.md, 'Two HIP runtimes')");
  }
}

void finalize() {
  tempi_hip_resident_stop(); // (before the streams go: nothing may outlive MPI_Finalize)
  std::lock_guard<std::mutex> g(mtx);
  for (void *s : streams)
    if (s) tempi_hip_stream_destroy(s);
  streams.clear();
}

uint32_t identity(int device) {
  static std::vector<uint32_t> ids;
  std::lock_guard<std::mutex> g(mtx);
  if (device < 0 || device >= nDevices) return 0;
  if (ids.size() < size_t(nDevices)) ids.assign(size_t(nDevices), 0);
  if (!ids[size_t(device)]) {
    unsigned char u[16] = {0};
    tempi_hip_device_uuid(device, u);
    uint32_t h = 2166136261u;
    for (unsigned char c : u) h = (h ^ c) * 16777619u;
    // TEMPI_FAKE_FOREIGN_GPU (tests): every process sees its GPU under an
    // identity of its own, so peers sharing this box's GPU take the
    // cross-GPU paths (system-scope loads, the first-contact canary)
    static const bool fakeForeign = std::getenv("TEMPI_FAKE_FOREIGN_GPU") != nullptr;
    if (fakeForeign) h = (h ^ uint32_t(getpid())) * 16777619u;
    ids[size_t(device)] = h ? h : 1;
  }
  return ids[size_t(device)];
}

Ptr classify(const void *p) {
  Ptr r;
  if (!nDevices || !p) return r;
  tempi_hip_ptrinfo info;
  if (tempi_hip_pointer_info(p, &info) != 0) return r;
  if (info.kind == TEMPI_HIP_MEM_HOST || !info.device_ptr) return r;
  r.device_accessible = true;
  r.host_accessible = info.kind != TEMPI_HIP_MEM_DEVICE;
  r.device = info.device < 0 ? 0 : info.device;
  r.dptr = info.device_ptr;
  return r;
}

void *stream(int device, int lane) {
  if (device < 0 || device >= nDevices || lane < 0 || lane >= kMaxLanes) return nullptr;
  const size_t i = size_t(device) * kMaxLanes + size_t(lane);
  std::lock_guard<std::mutex> g(mtx);
  if (!streams[i]) {
    int cur = 0;
    tempi_hip_get_device(&cur);
    if (cur != device) tempi_hip_set_device(device);
    void *s = nullptr;
    // with several lanes, lane 0 (gathers whose packed bytes a peer is
    // waiting for) outranks the scatter lanes
    check(tempi_hip_stream_create_priority(&s, nLanes > 1 && lane == 0), "stream create");
    if (cur != device) tempi_hip_set_device(cur);
    streams[i] = s;
  }
  return streams[i];
}

void check(int status, const char *what) {
  if (status != 0) LOG_FATAL("HIP error in " << what << ": " << tempi_hip_error_string(status));
}

} // namespace gpu
} // namespace tempi
