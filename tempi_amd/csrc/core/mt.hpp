// tempi_amd/csrc/core/mt.hpp -- MPI_THREAD_MULTIPLE: one process-wide lock
// around TEMPI's state.
//
// The transport's state (pending launch lists, the board of operations
// awaiting acks, the library requests it watches, the request table, the self
// channels, send gates: core/p2p_internal.hpp) is unsynchronised. An
// application that asks for MPI_THREAD_MULTIPLE (and gets it from the
// library) therefore runs every interposed call under one lock (`Entry`,
// re-entrant per thread: TEMPI's own calls of interposed functions nest). A
// thread never keeps it while it waits on anything another thread or process
// may have to do first:
//   - wait loops give it up between progress passes (`yield`), so another
//     thread can post the message the loop is waiting for;
//   - blocking library calls run without it (`Unlocked`): MPICH is
//     thread-safe at MULTIPLE on its own, and a blocked MPI_Recv must not keep
//     another thread of this process from sending what the peer waits for.
// Neither gives the lock up inside a progress pass (a callback that waits
// runs a nested pass while the outer one is iterating TEMPI's lists).
// Every other level costs one branch per call: `on` stays false and TEMPI
// reports MPI_THREAD_SERIALIZED at most (interpose_core.cpp).
// (The reference only logs the level: /root/reference/src/init.cpp:36-46.)
#pragma once

namespace tempi {
namespace mt {

extern bool on; // MPI_THREAD_MULTIPLE granted: the lock is in use

void lock();
void unlock();
int &depth(); // this thread's nesting of Entry

struct Entry {
  const bool held;
  Entry() : held(on) {
    if (held && depth()++ == 0) lock();
  }
  ~Entry() {
    if (held && --depth() == 0) unlock();
  }
  Entry(const Entry &) = delete;
  Entry &operator=(const Entry &) = delete;
};

// true when this thread may give the lock up here: it holds it, and no
// progress pass is on its stack
bool may_release();

struct Unlocked {
  int saved = 0;
  Unlocked() {
    if (on && may_release()) {
      saved = depth();
      depth() = 0;
      unlock();
    }
  }
  ~Unlocked() {
    if (saved) {
      lock();
      depth() = saved;
    }
  }
  Unlocked(const Unlocked &) = delete;
  Unlocked &operator=(const Unlocked &) = delete;
};

// between two progress passes of a wait loop: let another thread in
void yield();

} // namespace mt
} // namespace tempi

#define TEMPI_MT_ENTRY ::tempi::mt::Entry tempiMtEntry_
// a blocking library call, made without TEMPI's lock
#define TEMPI_UNLOCKED(...) ([&] { ::tempi::mt::Unlocked u_; return (__VA_ARGS__); }())
