// tempi_amd/csrc/core/alloc.cpp -- see alloc.hpp
#include "trace.hpp"
#include "alloc.hpp"

#include "gpu.hpp"
#include "log.hpp"
#include "tempi_hip.h"

#include <atomic>
#include <cstring>

namespace tempi {

namespace {
std::atomic<uint32_t> nextId{1};

int size_class(size_t n) {
  int c = 12; // 4 KiB minimum
  while ((size_t(1) << c) < n) ++c;
  return c;
}
} // namespace

SlabPool::~SlabPool() {
  // process teardown: the runtime may already be gone; leak rather than crash
}

Slab *SlabPool::get(size_t n, int device) {
  const int c = size_class(n);
  std::lock_guard<std::mutex> g(mtx_);
  if (size_t(c) < free_.size()) {
    auto &fl = free_[size_t(c)];
    for (size_t i = fl.size(); i-- > 0;) {
      if (kind_ == PINNED || fl[i]->device == device) {
        Slab *s = fl[i];
        fl.erase(fl.begin() + long(i));
        return s;
      }
    }
  }
  TEMPI_RANGE(kind_ == DEVICE ? "tempi::slab alloc (device)" : "tempi::slab alloc (pinned)");
  Slab *s = new Slab();
  s->size = size_t(1) << c;
  s->device = device;
  s->id = nextId++;
  int e;
  if (kind_ == DEVICE) {
    int cur = 0;
    tempi_hip_get_device(&cur);
    if (cur != device) tempi_hip_set_device(device);
    e = tempi_hip_malloc(&s->dev, s->size);
    if (cur != device) tempi_hip_set_device(cur);
  } else {
    e = tempi_hip_host_alloc(&s->host, &s->dev, s->size);
  }
  if (e != 0) {
    LOG_ERROR("slab allocation of " << s->size << " B failed: " << tempi_hip_error_string(e));
    delete s;
    return nullptr;
  }
  all_.push_back(s);
  held_ += s->size;
  return s;
}

void SlabPool::put(Slab *s) {
  if (!s) return;
  const int c = size_class(s->size);
  std::lock_guard<std::mutex> g(mtx_);
  if (free_.size() <= size_t(c)) free_.resize(size_t(c) + 1);
  free_[size_t(c)].push_back(s);
}

void SlabPool::discard(Slab *s, bool free) {
  if (!s) return;
  {
    std::lock_guard<std::mutex> g(mtx_);
    for (size_t i = 0; i < all_.size(); ++i)
      if (all_[i] == s) {
        all_.erase(all_.begin() + long(i));
        break;
      }
    held_ -= s->size;
  }
  if (free) {
    if (kind_ == DEVICE)
      tempi_hip_free(s->dev);
    else
      tempi_hip_host_free(s->host);
  }
  delete s;
}

void SlabPool::release_all() {
  std::lock_guard<std::mutex> g(mtx_);
  for (Slab *s : all_) {
    if (kind_ == DEVICE)
      tempi_hip_free(s->dev);
    else
      tempi_hip_host_free(s->host);
    delete s;
  }
  all_.clear();
  free_.clear();
  held_ = 0;
}

SlabPool &device_pool() {
  static SlabPool *p = new SlabPool(SlabPool::DEVICE);
  return *p;
}

SlabPool &pinned_pool() {
  static SlabPool *p = new SlabPool(SlabPool::PINNED);
  return *p;
}

const unsigned char *slab_ipc_handle(Slab *s) {
  if (!s->ipcReady) {
    gpu::check(tempi_hip_ipc_get_handle(s->ipc, s->dev), "ipc get handle");
    s->ipcReady = true;
  }
  return s->ipc;
}

} // namespace tempi
