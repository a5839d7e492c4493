// tempi_amd/csrc/core/gpu.hpp -- the GPU as the interposer sees it, through
// the C ABI of include/tempi_hip.h only.
//
// Streams: one non-blocking stream per device, created lazily on the device
// that owns the memory being packed (the reference creates kernStream /
// commStream once at MPI_Init on whatever device is current:
// /root/reference/src/internal/streams.cpp:19-28; a rank that selects its GPU
// after MPI_Init would then pack on the wrong device).
#pragma once

#include <string>
#include <vector>

#include "tempi_hip.h"

#include <cstdint>

namespace tempi {
namespace gpu {

// true when at least one GPU is visible (decided at MPI_Init)
bool available();
// the distinct libamdhip64 objects mapped into this process (realpath'd)
std::vector<std::string> hip_runtimes();
void init();
void finalize();

struct Ptr {
  bool device_accessible = false;
  bool host_accessible = true; // false for hipMalloc memory
  int device = -1;
  void *dptr = nullptr; // GPU-visible address
};
Ptr classify(const void *p);

// the TEMPI stream of a device (created on first use); nullptr on failure.
// lane 0 carries every synchronous operation and the batched gathers; the
// transport spreads batched scatters / copies over lanes 1 .. lanes()-1 so
// that one batch's tail overlaps the next batch's start.
constexpr int kMaxLanes = 4;
void *stream(int device, int lane = 0);
// lanes in use: TEMPI_STREAMS (1 .. kMaxLanes) if set, else 3 -- or 1 when
// the node runs more ranks than it has visible GPUs, i.e. ranks share a GPU
// (concurrent kernels from several processes' lanes measured 15-50 % slower
// than one stream each; alone on its GPU, 3 lanes are 12 % faster: DESIGN §6)
int lanes();
void choose_lanes(int ranksOnNode); // at MPI_Init, after topology::init


// 32-bit identity of a device's physical GPU, equal in every process that
// sees it (FNV-1a of its UUID); used to tell a peer on the same GPU from a
// peer on another one
uint32_t identity(int device);

// abort with a message on a tempi_hip_* failure
void check(int status, const char *what);

} // namespace gpu
} // namespace tempi
