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

struct TypeRecord {
  StridedBlock desc;
  std::unique_ptr<Packer> packer; // null when !desc.valid (library handles it)
};

// analyse + cache (no-op when already cached); returns the record
const TypeRecord *type_commit(MPI_Datatype t);
// nullptr when unknown
const TypeRecord *type_lookup(MPI_Datatype t);
void type_release(MPI_Datatype t);
// records for the predefined dense types
void types_init();
void types_finalize();

} // namespace tempi
