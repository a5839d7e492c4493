// tempi_amd/csrc/core/type_cache.cpp -- see type_cache.hpp
#include "type_cache.hpp"

#include "log.hpp"

#include <mutex>
#include <unordered_map>

namespace tempi {

namespace {
std::mutex mtx;
std::unordered_map<MPI_Datatype, std::shared_ptr<TypeRecord>> cache;
uint64_t generation = 1;
} // namespace

uint64_t type_generation() {
  std::lock_guard<std::mutex> g(mtx);
  return generation;
}

const TypeRecord *type_commit(MPI_Datatype t) {
  {
    std::lock_guard<std::mutex> g(mtx);
    auto it = cache.find(t);
    if (it != cache.end()) return it->second.get();
  }
  auto rec = std::make_shared<TypeRecord>();
  rec->desc = canonicalise(t);
  if (rec->desc.valid) {
    rec->packer = std::make_unique<Packer>(rec->desc);
    rec->flat1ok = rec->packer->flat(1, &rec->flat1);
    LOG_SPEW("type " << t << " -> " << rec->desc.str());
  } else {
    LOG_DEBUG("type " << t << " is not a strided block; library handles it");
  }
  std::lock_guard<std::mutex> g(mtx);
  auto &slot = cache[t];
  if (!slot) {
    slot = std::move(rec);
    generation++;
  }
  return slot.get();
}

// every MPI_Isend / MPI_Irecv / MPI_Pack looks its type up: no lock here.
// Lookups run inside interposed calls, which never overlap at the levels TEMPI
// reports (SERIALIZED, or MULTIPLE under TEMPI's own lock, mt.hpp), so they
// cannot race with the commit or free that changes the cache.
const TypeRecord *type_lookup(MPI_Datatype t) {
  auto it = cache.find(t);
  return it == cache.end() ? nullptr : it->second.get();
}

void type_release(MPI_Datatype t) {
  std::lock_guard<std::mutex> g(mtx);
  if (cache.erase(t)) generation++;
}

void types_init() {
  for (MPI_Datatype t : {MPI_BYTE, MPI_CHAR, MPI_SIGNED_CHAR, MPI_UNSIGNED_CHAR, MPI_SHORT,
                         MPI_UNSIGNED_SHORT, MPI_INT, MPI_UNSIGNED, MPI_LONG, MPI_UNSIGNED_LONG,
                         MPI_LONG_LONG, MPI_UNSIGNED_LONG_LONG, MPI_FLOAT, MPI_DOUBLE, MPI_INT8_T,
                         MPI_INT16_T, MPI_INT32_T, MPI_INT64_T, MPI_UINT8_T, MPI_UINT16_T,
                         MPI_UINT32_T, MPI_UINT64_T, MPI_C_BOOL, MPI_WCHAR})
    type_commit(t);
}

void types_finalize() {
  std::lock_guard<std::mutex> g(mtx);
  cache.clear();
  generation++;
}

} // namespace tempi
