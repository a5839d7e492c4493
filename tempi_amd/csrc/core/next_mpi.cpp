// tempi_amd/csrc/core/next_mpi.cpp -- see next_mpi.hpp
#include "next_mpi.hpp"
#include "log.hpp"

#include <cstdlib>
#include <cstring>
#include <dlfcn.h>
#include <mutex>

namespace tempi {

NextMPI next;

static void self_marker() {}

static const char *own_object() {
  static const char *name = [] {
    Dl_info info;
    if (dladdr(reinterpret_cast<void *>(&self_marker), &info) && info.dli_fname)
      return info.dli_fname;
    return "";
  }();
  return name;
}

static bool is_ours(void *p) {
  Dl_info info;
  if (!p || !dladdr(p, &info) || !info.dli_fname) return false;
  return std::strcmp(info.dli_fname, own_object()) == 0;
}

static void *fallback_handle() {
  static void *h = [] {
    const char *name = std::getenv("TEMPI_MPI_LIBRARY");
    if (!name) name = "libmpi.so.12";
    void *hh = dlopen(name, RTLD_NOLOAD | RTLD_LAZY | RTLD_GLOBAL);
    if (!hh) hh = dlopen(name, RTLD_LAZY | RTLD_GLOBAL);
    return hh;
  }();
  return h;
}

static void *find(const char *sym) {
  void *p = dlsym(RTLD_NEXT, sym);
  if (p && !is_ours(p)) return p;
  if (void *h = fallback_handle()) {
    p = dlsym(h, sym);
    if (p && !is_ours(p)) return p;
  }
  LOG_FATAL("unable to resolve the underlying " << sym);
}

void resolve_next() {
  static std::once_flag once;
  std::call_once(once, [] {
#define TEMPI_X(f) next.f = reinterpret_cast<decltype(next.f)>(find(#f));
    TEMPI_NEXT_FUNCS(TEMPI_X)
#undef TEMPI_X
  });
}

} // namespace tempi
