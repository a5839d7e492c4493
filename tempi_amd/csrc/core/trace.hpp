// tempi_amd/csrc/core/trace.hpp -- roctx ranges around TEMPI's operations, the
// counterpart of the reference's NVTX ranges (/root/reference/src/pack.cpp:37,
// unpack.cpp:29, internal/alltoallv_impl.cpp:202-239, async_operation.cpp,
// allocators.cpp, events.cpp, streams.cpp). rocprofv3 --marker-trace shows
// them next to the kernels. The roctx library is loaded at MPI_Init only when
// TEMPI_ROCTX=1 or a rocprofv3 session is detected; otherwise a range costs
// one pointer test.
//
// TEMPI_TIMELINE=PREFIX records the same ranges, plus instants such as a
// batch observed complete, as CLOCK_BOOTTIME nanoseconds (the clock of
// rocprofv3's kernel trace) into memory and writes PREFIX.r<rank>.csv at
// MPI_Finalize: a host timeline cheap enough (a clock read per mark, no HIP
// API tracing) that laying it beside a --kernel-trace leaves the timing
// nearly as it is untraced (tools/halo_timeline.py).
#pragma once

namespace tempi {
namespace trace {

extern int (*rangePush)(const char *);
extern int (*rangePop)();
extern bool timelineOn;

void init();
void finalize(int rank);
// phase: 0 begin, 1 end, 2 instant
void mark(const char *name, int phase);

struct Range {
  bool on;
  const char *name;
  explicit Range(const char *n) : on(rangePush != nullptr), name(n) {
    if (timelineOn) mark(n, 0);
    if (on) rangePush(n);
  }
  ~Range() {
    if (on) rangePop();
    if (timelineOn) mark(name, 1);
  }
  Range(const Range &) = delete;
  Range &operator=(const Range &) = delete;
};

} // namespace trace
} // namespace tempi

#define TEMPI_RANGE_CAT2(a, b) a##b
#define TEMPI_RANGE_CAT(a, b) TEMPI_RANGE_CAT2(a, b)
#define TEMPI_RANGE(name) ::tempi::trace::Range TEMPI_RANGE_CAT(tempiRange_, __LINE__)(name)
