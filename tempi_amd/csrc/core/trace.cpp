// tempi_amd/csrc/core/trace.cpp -- see trace.hpp
#include "trace.hpp"

#include "log.hpp"

#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <dlfcn.h>
#include <string>
#include <vector>

extern char **environ;

namespace tempi {
namespace trace {

int (*rangePush)(const char *) = nullptr;
int (*rangePop)() = nullptr;
bool timelineOn = false;

namespace {
struct Mark {
  int64_t ns;
  const char *name;
  int phase;
};
std::vector<Mark> marks;
std::string timelinePrefix;
uint64_t dropped = 0;
constexpr size_t kMaxMarks = size_t(1) << 20;
} // namespace

void mark(const char *name, int phase) {
  if (marks.size() >= kMaxMarks) {
    ++dropped;
    return;
  }
  timespec ts;
  clock_gettime(CLOCK_BOOTTIME, &ts);
  marks.push_back({int64_t(ts.tv_sec) * 1000000000 + ts.tv_nsec, name, phase});
}

void finalize(int rank) {
  if (!timelineOn) return;
  timelineOn = false;
  const std::string path = timelinePrefix + ".r" + std::to_string(rank) + ".csv";
  FILE *f = std::fopen(path.c_str(), "w");
  if (!f) {
    LOG_WARN("cannot write the timeline " << path);
  } else {
    std::fprintf(f, "ns,phase,name\n");
    for (const Mark &m : marks) std::fprintf(f, "%lld,%d,%s\n", (long long)m.ns, m.phase, m.name);
    std::fclose(f);
    if (dropped) LOG_WARN("timeline: " << dropped << " marks dropped (more than " << kMaxMarks << ")");
  }
  std::vector<Mark>().swap(marks);
}

static bool under_profiler() {
  for (char **e = environ; e && *e; ++e)
    if (!std::strncmp(*e, "ROCPROF", 7)) return true;
  return false;
}

void init() {
  if (const char *tl = std::getenv("TEMPI_TIMELINE")) {
    if (*tl) {
      timelinePrefix = tl;
      marks.reserve(kMaxMarks);
      timelineOn = true;
    }
  }
  const char *want = std::getenv("TEMPI_ROCTX");
  if (want ? std::strcmp(want, "0") == 0 : !under_profiler()) return;
  for (const char *lib : {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4"}) {
    void *h = dlopen(lib, RTLD_NOW | RTLD_GLOBAL);
    if (!h) continue;
    auto push = reinterpret_cast<int (*)(const char *)>(dlsym(h, "roctxRangePushA"));
    auto pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
    if (push && pop) {
      rangePush = push;
      rangePop = pop;
      LOG_DEBUG("roctx ranges on (" << lib << ")");
      return;
    }
  }
  LOG_DEBUG("roctx library not found: no ranges");
}

} // namespace trace
} // namespace tempi
