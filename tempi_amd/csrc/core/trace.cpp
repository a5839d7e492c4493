// tempi_amd/csrc/core/trace.cpp -- see trace.hpp
#include "trace.hpp"

#include "log.hpp"

#include <cstdlib>
#include <cstring>
#include <dlfcn.h>

extern char **environ;

namespace tempi {
namespace trace {

int (*rangePush)(const char *) = nullptr;
int (*rangePop)() = nullptr;

static bool under_profiler() {
  for (char **e = environ; e && *e; ++e)
    if (!std::strncmp(*e, "ROCPROF", 7)) return true;
  return false;
}

void init() {
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
