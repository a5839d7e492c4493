// tempi_amd/csrc/core/type_cache.hpp -- committed-type records, keyed by
// handle (the reference's typeCache: /root/reference/include/
// type_cache.hpp:23-30, filled at /root/reference/src/type_commit.cpp:16-114,
// dropped at /root/reference/src/type_free.cpp:14-27).
#pragma once

#include "packer.hpp"
#include "types.hpp"

#include <mpi.h>

#include <memory>

namespace tempi {

struct TypeRecord;
// in-flight operations hold their type's record: MPI_Type_free may come
// before the operation completes
typedef std::shared_ptr<const TypeRecord> RecordRef;

struct TypeRecord : std::enable_shared_from_this<TypeRecord> {
  StridedBlock desc;
  std::unique_ptr<Packer> packer; // null when !desc.valid (library handles it)
  tempi_hip_desc flat1{};         // one element as a single descriptor
  bool flat1ok = false;

  RecordRef ref() const { return shared_from_this(); }
  // `count` elements as one descriptor (Packer::flat; cached for count 1)
  bool flat(int64_t count, tempi_hip_desc *out) const {
    if (count == 1) {
      *out = flat1;
      return flat1ok;
    }
    return packer && packer->flat(count, out);
  }
};

// analyse + cache (no-op when already cached); returns the record
const TypeRecord *type_commit(MPI_Datatype t);
// nullptr when unknown
const TypeRecord *type_lookup(MPI_Datatype t);
void type_release(MPI_Datatype t);
// bumped whenever a record is added or dropped: plans that captured type
// records by handle (neighbourhood-collective plans) are stale once it moves
uint64_t type_generation();
// records for the predefined dense types
void types_init();
void types_finalize();

} // namespace tempi
