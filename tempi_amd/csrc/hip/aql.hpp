// tempi_amd/csrc/hip/aql.hpp -- kernel dispatch packets written straight into
// an HSA queue of TEMPI's own, for synchronous MPI_Pack / MPI_Unpack
// (TEMPI_AQL=1). Internal to libtempi_hip.so.
//
// A synchronous small call is launch + completion. The completion is already
// a ticket the kernel stores (ticket.hpp); the launch is hipLaunchKernelGGL,
// ~2.8 us of host time per call on MI355X / ROCm 7.2 (tools/syncbench.cpp,
// profiles/r03/sync2_s7.jsonl) before the doorbell rings. Here the packet is
// written by TEMPI: the kernel object comes from the code object HIP already
// loaded (its name from hipKernelNameRefByPtr, the symbol from the HSA loader),
// the explicit arguments are copied into a kernarg slot and the implicit ones
// (grid / workgroup sizes) are filled as code object v5 lays them out.
//
// Launches on the queue are not ordered with any HIP stream, so a call that
// dispatches here completes on a ticket of the queue's own (its own flag and
// workgroup counters), and its wait never takes an idle stream for done.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace tempi_aql {

struct Queue;

// the queue for synchronous work of the device `s` runs on; nullptr when
// TEMPI_AQL is unset, HSA is unavailable, or the queue could not be made
Queue *for_stream(hipStream_t s);

// dispatch `kernel` (the __global__ function's host-side address) over
// `blocks` workgroups of `wg` lanes with explicit arguments [args, args +
// bytes); false: nothing was dispatched (the kernel object is not found yet,
// its argument layout is not the one expected, or the queue failed), and the
// caller launches through HIP instead
bool dispatch(Queue *q, const void *kernel, hipStream_t s, uint32_t blocks, uint32_t wg, const void *args,
              size_t bytes);

// a TEMPI queue reported an error: waits on its tickets end
bool failed();

struct Stats {
  uint64_t dispatched = 0, refused = 0;
};
Stats stats();

} // namespace tempi_aql
