// tempi_amd/csrc/core/gpu.hpp -- the GPU as the interposer sees it, through
// the C ABI of include/tempi_hip.h only.
//
// Streams: one non-blocking stream per device, created lazily on the device
// that owns the memory being packed (the reference creates kernStream /
// commStream once at MPI_Init on whatever device is current:
// /root/reference/src/internal/streams.cpp:19-28; a rank that selects its GPU
// after MPI_Init would then pack on the wrong device).
#pragma once

#include "tempi_hip.h"

#include <cstdint>

namespace tempi {
namespace gpu {

// true when at least one GPU is visible (decided at MPI_Init)
bool available();
void init();
void finalize();

struct Ptr {
  bool device_accessible = false;
  bool host_accessible = true; // false for hipMalloc memory
  int device = -1;
  void *dptr = nullptr; // GPU-visible address
};
Ptr classify(const void *p);

// the TEMPI stream of a device (created on first use); nullptr on failure
void *stream(int device);

// a timing event pair owned by TEMPI for `device` (created on first use)
void profiling_events(int device, void **start, void **stop);

// abort with a message on a tempi_hip_* failure
void check(int status, const char *what);

} // namespace gpu
} // namespace tempi
