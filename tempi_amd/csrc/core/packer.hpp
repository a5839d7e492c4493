// tempi_amd/csrc/core/packer.hpp -- pack / unpack of `count` elements of a
// canonical type on a TEMPI stream.
//
// Replaces the reference's Packer hierarchy (/root/reference/include/
// packer.hpp:14-49, packer_1d/2d/3d): one object serves every
// dimensionality, because the element count is folded in as the outermost
// dimension (stride = extent) and the GPU layer handles any rank up to
// TEMPI_HIP_MAX_DIMS; deeper types are issued as several launches.
#pragma once

#include "types.hpp"

#include "tempi_hip.h"

#include <cstdint>
#include <vector>

namespace tempi {

struct PackStats;

class Packer {
public:
  explicit Packer(const StridedBlock &sb) : sb_(sb) {}

  int64_t packed_bytes(int64_t count) const { return sb_.size * count; }

  // enqueue: packed[0..bytes) <- `count` elements at `origin` (GPU-visible
  // addresses). Returns 0 or a tempi_hip status.
  int pack_async(void *packed, const void *origin, int64_t count, void *stream) const;
  int unpack_async(void *origin, const void *packed, int64_t count, void *stream) const;

  // the same plus a completion ticket for a synchronous caller: done->flag
  // reaching done->ticket means the work is complete (tempi_hip_ticket_wait);
  // done->flag stays nullptr when nothing was launched
  struct Completion {
    const uint32_t *flag = nullptr;
    uint32_t ticket = 0;
  };
  int pack_ticket(void *packed, const void *origin, int64_t count, void *stream, Completion *done) const;
  int unpack_ticket(void *origin, const void *packed, int64_t count, void *stream, Completion *done) const;

  // the same work as launch items, appended to `out` (nothing is launched):
  // the transport batches many messages into one kernel launch
  void items(void *packed, const void *origin, int64_t count, std::vector<tempi_hip_batch_item> &out) const;

  // `count` elements as ONE descriptor whose first byte is origin + start
  // (false when it needs more than TEMPI_HIP_MAX_DIMS dimensions)
  bool flat(int64_t count, tempi_hip_desc *out) const;

  const StridedBlock &desc() const { return sb_; }

private:
  int launch(bool pack, char *packed, char *origin, int64_t count, void *stream, Completion *done) const;
  StridedBlock sb_;
};

} // namespace tempi
