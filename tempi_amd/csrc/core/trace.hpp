// tempi_amd/csrc/core/trace.hpp -- roctx ranges around TEMPI's operations, the
// counterpart of the reference's NVTX ranges (/root/reference/src/pack.cpp:37,
// unpack.cpp:29, internal/alltoallv_impl.cpp:202-239, async_operation.cpp,
// allocators.cpp, events.cpp, streams.cpp). rocprofv3 --marker-trace shows
// them next to the kernels. The roctx library is loaded at MPI_Init only when
// TEMPI_ROCTX=1 or a rocprofv3 session is detected; otherwise a range costs
// one pointer test.
#pragma once

namespace tempi {
namespace trace {

extern int (*rangePush)(const char *);
extern int (*rangePop)();

void init();

struct Range {
  bool on;
  explicit Range(const char *name) : on(rangePush != nullptr) {
    if (on) rangePush(name);
  }
  ~Range() {
    if (on) rangePop();
  }
  Range(const Range &) = delete;
  Range &operator=(const Range &) = delete;
};

} // namespace trace
} // namespace tempi

#define TEMPI_RANGE_CAT2(a, b) a##b
#define TEMPI_RANGE_CAT(a, b) TEMPI_RANGE_CAT2(a, b)
#define TEMPI_RANGE(name) ::tempi::trace::Range TEMPI_RANGE_CAT(tempiRange_, __LINE__)(name)
