// tempi_amd/csrc/core/alloc.hpp -- power-of-two slab pools for intermediate
// packed buffers.
//
// Replaces the reference's SlabAllocator over cudaMalloc / new[] +
// cudaHostRegister(Mapped) (/root/reference/include/allocator_slab.hpp:17-198,
// allocator_device.hpp:35-53, allocator_host.hpp:31-60, globals at
// /root/reference/src/internal/allocators.cpp:10-11). Differences:
//  * each slab is its own allocation (device: hipMalloc, host: hipHostMalloc
//    mapped + portable), so a device slab can be exported whole through an
//    IPC handle, which is cached with the slab;
//  * a slab's size class is log2, min 4 KiB; free slabs are reused LIFO (warm
//    in the MALL), and everything is released at MPI_Finalize;
//  * every slab has a process-unique id (the IPC transport names slabs by it).
#pragma once

#include <cstddef>
#include <cstdint>
#include <mutex>
#include <vector>

namespace tempi {

struct Slab {
  void *host = nullptr; // CPU address (pinned pools) or nullptr
  void *dev = nullptr;  // GPU address
  size_t size = 0;      // capacity
  int device = -1;      // owning device (device pools)
  uint32_t id = 0;      // process-unique
  bool ipcReady = false;
  unsigned char ipc[64]; // IPC handle of `dev` (device pools)
};

class SlabPool {
public:
  enum Kind { DEVICE, PINNED };
  explicit SlabPool(Kind k) : kind_(k) {}
  ~SlabPool();

  // a slab of at least n bytes (nullptr on allocation failure)
  Slab *get(size_t n, int device);
  void put(Slab *s);
  // free a slab now instead of keeping it (an oversized one-off); free =
  // false leaves the memory allocated (a kernel may still be using it) and
  // only forgets it
  void discard(Slab *s, bool free = true);
  void release_all();
  size_t bytes_held() const { return held_; }

private:
  Kind kind_;
  std::mutex mtx_;
  std::vector<std::vector<Slab *>> free_; // by size class
  std::vector<Slab *> all_;
  size_t held_ = 0;
};

SlabPool &device_pool();
SlabPool &pinned_pool();

// IPC handle for a device slab (computed once)
const unsigned char *slab_ipc_handle(Slab *s);

} // namespace tempi
