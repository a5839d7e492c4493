// tempi_amd/csrc/core/p2p_board.cpp -- acks between the ranks of one node
// (p2p_internal.hpp)
#include "p2p_internal.hpp"

#include "alloc.hpp"
#include "counters.hpp"
#include "env.hpp"
#include "gpu.hpp"
#include "log.hpp"
#include "next_mpi.hpp"
#include "packer.hpp"
#include "perf_model.hpp"
#include "state.hpp"
#include "topology.hpp"
#include "trace.hpp"
#include "type_cache.hpp"

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <unistd.h>

namespace tempi {
namespace p2p {
namespace detail {

// Acks between the ranks of one node go through shared memory: each rank
// exposes `slots` 32-bit slots (MPI_Win_allocate_shared over its
// MPI_COMM_TYPE_SHARED communicator). A sender takes a free slot of its own
// board for each message whose ack it waits for (IPC slab, IPC COPY) and names
// it as the descriptor's ackTag; the receiver stores code + 1 into that slot
// (release) and the sender polls its outstanding slots on each progress pass
// (acquire). No library message per ack, and no library request in the
// sender's MPI_Testsome for it. Tags below `slots` are board slots; acks that
// travel as library messages (a peer outside the node communicator, no free
// slot) keep tags at or above it.
AckBoard board;

// a free slot of this rank's board for a message to world rank `peer`, or -1
int board_take(int peer) {
  if (!board.slots || peer < 0 || size_t(peer) >= board.of.size() || !board.of[size_t(peer)] ||
      board.freeSlots.empty())
    return -1;
  const int s = board.freeSlots.back();
  board.freeSlots.pop_back();
  return s;
}

// a slot taken for a message that was never sent
void board_give(int slot) { board.freeSlots.push_back(slot); }

// the ack code in this rank's slot (and the slot freed), or -1 until it arrives
int board_poll(int slot) {
  uint32_t *p = board.of[size_t(state.worldRank)] + slot;
  const uint32_t v = __atomic_load_n(p, __ATOMIC_ACQUIRE);
  if (!v) return -1;
  __atomic_store_n(p, 0u, __ATOMIC_RELAXED);
  board.freeSlots.push_back(slot);
  return int(v) - 1;
}

void board_init() {
  board = AckBoard();
  const int half = std::max(1, tagUb / 2);
  const int slots = std::min(16384, half / 2); // (library-message ack tags stay above)
  if (slots < 64) return;
  MPI_Comm_split_type(MPI_COMM_WORLD, MPI_COMM_TYPE_SHARED, state.worldRank, MPI_INFO_NULL, &board.node);
  MPI_Comm_set_errhandler(board.node, MPI_ERRORS_RETURN); // no shared window: library acks, not an abort
  uint32_t *mine = nullptr;
  if (MPI_Win_allocate_shared(MPI_Aint(slots) * MPI_Aint(sizeof(uint32_t)), int(sizeof(uint32_t)), MPI_INFO_NULL,
                              board.node, &mine, &board.win) != MPI_SUCCESS) {
    next.MPI_Comm_free(&board.node);
    return;
  }
  std::memset(mine, 0, size_t(slots) * sizeof(uint32_t));
  int n = 0;
  MPI_Comm_size(board.node, &n);
  MPI_Group g, wg;
  MPI_Comm_group(board.node, &g);
  MPI_Comm_group(MPI_COMM_WORLD, &wg);
  std::vector<int> local(static_cast<size_t>(n)), world(static_cast<size_t>(n));
  for (int i = 0; i < n; ++i) local[size_t(i)] = i;
  MPI_Group_translate_ranks(g, n, local.data(), wg, world.data());
  MPI_Group_free(&g);
  MPI_Group_free(&wg);
  board.of.assign(size_t(state.worldSize), nullptr);
  for (int i = 0; i < n; ++i) {
    MPI_Aint size = 0;
    int unit = 0;
    uint32_t *base = nullptr;
    MPI_Win_shared_query(board.win, i, &size, &unit, &base);
    if (world[size_t(i)] >= 0) board.of[size_t(world[size_t(i)])] = base;
  }
  board.freeSlots.reserve(size_t(slots));
  for (int i = slots - 1; i >= 0; --i) board.freeSlots.push_back(i);
  board.slots = slots;
  MPI_Barrier(board.node); // every board is zeroed before any rank writes to one
}

void board_finalize() {
  if (board.win != MPI_WIN_NULL) MPI_Win_free(&board.win);
  if (board.node != MPI_COMM_NULL) next.MPI_Comm_free(&board.node);
  board = AckBoard();
}

std::vector<std::unique_ptr<PendingAck>> pendingAcks;

int ackCodes[3] = {0, 1, 2};

void send_ack(int world, int tag, int code) {
  if (tag < board.slots && world >= 0 && size_t(world) < board.of.size() && board.of[size_t(world)]) {
    __atomic_store_n(board.of[size_t(world)] + tag, uint32_t(code + 1), __ATOMIC_RELEASE);
    return;
  }
  MPI_Request r;
  next.MPI_Isend(&ackCodes[code], 1, MPI_INT, world, tag, ctrlComm, &r);
  next.MPI_Request_free(&r);
}
void send_ack(const IpcDesc &d, int code) { send_ack(d.senderWorld, d.ackTag, code); }

} // namespace detail
} // namespace p2p
} // namespace tempi
