// tempi_amd/csrc/core/mt.cpp -- see mt.hpp
#include "mt.hpp"

#include "p2p.hpp"

#include <mutex>
#include <sched.h>

namespace tempi {
namespace mt {

bool on = false;

namespace {
std::mutex big;
}

void lock() { big.lock(); }
void unlock() { big.unlock(); }

int &depth() {
  static thread_local int d = 0;
  return d;
}

bool may_release() { return depth() > 0 && p2p::progress_depth() == 0; }

void yield() {
  if (!on || !may_release()) return;
  Unlocked u;
  sched_yield();
}

} // namespace mt
} // namespace tempi
