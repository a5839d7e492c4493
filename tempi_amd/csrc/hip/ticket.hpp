// tempi_amd/csrc/hip/ticket.hpp -- completion tickets of synchronous calls,
// shared by runtime.hip (the tickets, the wait) and pack_kernels.hip (work
// kernels that store the ticket themselves). Internal to libtempi_hip.so.
//
// A synchronous MPI_Pack / MPI_Unpack (/root/reference/src/internal/
// packer_2d.cu:101-118 waits with cudaStreamSynchronize) waits here for a
// ticket in pinned, coherent host memory instead: HIP's completion path costs
// ~5 us more than a flag the GPU stores (tools/flagbench.hip,
// profiles/r02/completion_flag_bench_s13.jsonl). Two ways to store it:
//  * a one-lane kernel queued behind the work (any work, any size);
//  * FOLDED into a small work kernel: every workgroup, once its stores are
//    done, makes them visible device-wide (agent-scope release) and counts
//    itself on a per-stream device counter; the workgroup that completes the
//    count stores the ticket with a system-scope release. That saves the
//    second kernel's dispatch behind the first.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <mutex>

// grids up to this many workgroups store their ticket themselves: each one
// adds a system-scope release (an L2 write-back) and an atomic to its end.
// Measured on MI355X (tools/syncbench.cpp, profiles/r03/sync3_s4.jsonl,
// per synchronous pack): folded 6.5 / 8.0 / 8.6 / 9.5 / 11.5 us at 1 / 8 /
// 64 / 128 / 256 workgroups against 8.4 / 9.8 / 9.8 / 9.9 / 9.9 us with
// the ticket kernel queued behind: the fold wins up to 128
#ifndef TEMPI_FOLD_MAX_BLOCKS
#define TEMPI_FOLD_MAX_BLOCKS 128
#endif
// gathers write their packed chunks, and scatters of 16-byte words their
// words, write-through (sc0 sc1 stores leave L2 as they are written), so only
// the workgroups holding the object's partial first / last chunk write back L2
// before counting themselves; the fold then costs each workgroup one atomic
// on its shard (MI355X_MICROARCH.md "publish-large": write-through + a drained
// flag beats a release per workgroup). Measured: 7.9 us at 256 workgroups
// against 9.7 us with the ticket kernel (profiles/r03/sync3_s7.jsonl)
#ifndef TEMPI_FOLD_MAX_BLOCKS_WT
#define TEMPI_FOLD_MAX_BLOCKS_WT 2048
#endif

namespace tempi_ticket {

// The workgroup count is sharded: workgroup b counts itself on shard b % 8,
// the workgroup completing a shard counts the shard on the top counter, and
// the one completing the top stores the ticket. One counter took every
// workgroup's system-scope atomic in turn (256 of them added ~2.2 us to a
// 256-workgroup call, profiles/r03/sync3_s6.jsonl); eight take them at once.
// Each counter has a 128-byte line of its own.
constexpr int kShards = 8;
constexpr int kCounterStride = 32; // uint32 words between counters (128 B)
constexpr int kCounterWords = (kShards + 1) * kCounterStride;

struct Ticket {
  uint32_t *host = nullptr, *dev = nullptr; // the flag (pinned, coherent)
  uint32_t next = 0;                        // last ticket issued
  uint32_t *counter = nullptr;              // device: kShards shard counters + the top counter
  uint32_t counted[kShards + 1] = {};       // the host's running totals of the same (mod 2^32)
  bool broken = false;                      // a folded launch failed: counters and totals disagree
};

// tickets stored by work kernels / by the ticket kernel, all streams
struct Stats {
  uint64_t folded = 0, queued = 0;
};
Stats &stats(); // (caller holds mutex())

// A fold offered to the next single launch of this thread (set by the
// *_ticket entry points around their launch): the launch takes it only when
// its grid is at most max_blocks workgroups.
struct Fold {
  Ticket *t = nullptr;
  uint32_t ticket = 0;
  uint32_t max_blocks = 0;    // launches whose stores go through L2 write-back
  uint32_t max_blocks_wt = 0; // launches that store write-through (gathers)
  bool taken = false;
};

// the kernel-side view, passed as a kernel argument (flag == nullptr: none)
struct Sig {
  uint32_t *counter;
  uint32_t *flag;
  uint32_t target[kShards]; // each shard's count once this launch's workgroups of that shard have counted
  uint32_t top;             // the top counter's value once this launch's last shard completes
  uint32_t ticket;
};

std::mutex &mutex();
// the stream's ticket state, flag and counter allocated on first use
// (caller holds mutex()); nullptr when allocation failed
Ticket *of(hipStream_t s);
// queue the one-lane ticket kernel storing `ticket` (caller holds mutex())
hipError_t queue_kernel(Ticket &t, hipStream_t s, uint32_t ticket);
// spin until the flag reaches `ticket`; the stream is queried every ~20 us,
// so a faulted stream ends the wait with its error
int wait(hipStream_t s, const uint32_t *flag, uint32_t ticket);
// largest grid a work kernel takes a fold for (TEMPI_FOLD_MAX_BLOCKS, 0 = never)
uint32_t fold_max_blocks();
// the same for launches whose work is stored write-through (TEMPI_FOLD_MAX_BLOCKS_WT)
uint32_t fold_max_blocks_wt();

} // namespace tempi_ticket
