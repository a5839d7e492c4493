// tempi_amd/csrc/core/types.hpp -- datatype canonicalisation.
//
// Replaces the reference's Type tree + simplify passes + StridedBlock
// (/root/reference/src/internal/types.cpp:42-705,
//  /root/reference/include/strided_block.hpp:12-67,
//  /root/reference/include/type_cache.hpp:23-30) with an order-preserving
// design:
//  * the decoded type is a list of strided dimensions, OUTERMOST FIRST, over a
//    contiguous block, plus the byte offset of the first byte;
//  * simplification only ever drops unit dimensions, folds a dense innermost
//    dimension into the block, and merges two adjacent dimensions whose
//    strides line up -- all of which keep MPI type-map order. The reference's
//    stride sort (stream_swap) is NOT done, because it changes the packed byte
//    order;
//  * the type's extent is kept, and the element count of a Pack call becomes
//    one more dimension of stride = extent (fixes SURVEY F2);
//  * 64-bit counts/offsets throughout;
//  * anything that is not a strided block (irregular indexed, struct with
//    several types, darray, ...) is marked not-representable and goes to the
//    library (never a null-packer crash: SURVEY F3).
#pragma once

#include <mpi.h>

#include <cstdint>
#include <string>
#include <vector>

namespace tempi {

struct Dim {
  int64_t count;
  int64_t stride; // bytes, may be negative
  bool operator==(const Dim &o) const { return count == o.count && stride == o.stride; }
};

struct StridedBlock {
  bool valid = false; // false: not representable, the library handles it
  int64_t start = 0;  // byte offset of the first byte from the buffer origin
  int64_t block = 0;  // contiguous bytes
  std::vector<Dim> dims; // outermost first
  int64_t size = 0;      // MPI_Type_size
  int64_t lb = 0, extent = 0;

  int64_t rows() const {
    int64_t r = 1;
    for (const Dim &d : dims) r *= d.count;
    return r;
  }
  std::string str() const;
};

// decode + simplify an MPI datatype (may call MPI_Type_get_envelope /
// _contents / _get_extent / _size; frees any derived handles it obtains)
StridedBlock canonicalise(MPI_Datatype t);

// order-preserving simplification (exposed for tests of the rules)
void simplify(StridedBlock &sb);

} // namespace tempi
