// tempi_amd/csrc/core/env.hpp -- presence-only environment switches, same
// names and defaults as the reference (/root/reference/src/internal/
// env.cpp:23-107, /root/reference/include/env.hpp:10-37), plus:
//   TEMPI_DATATYPE_STAGED  (the reference has the enum value but no variable)
//   TEMPI_DATATYPE_IPC     (MI355X intra-node device-to-device transport)
//   TEMPI_LOG_LEVEL=<level>
// TEMPI_PLACEMENT_KAHIP and TEMPI_PLACEMENT_METIS both select TEMPI's own
// partitioner (core/placement.hpp): neither library is in this image.
#pragma once

#include <string>

namespace tempi {

enum class DatatypeMethod { AUTO, ONESHOT, DEVICE, STAGED, IPC };
enum class ContiguousMethod { NONE, AUTO, STAGED };
enum class AlltoallvMethod { NONE, AUTO, REMOTE_FIRST, STAGED, ISIR_STAGED, ISIR_REMOTE_STAGED };
enum class PlacementMethod { NONE, RANDOM, PARTITION };

struct Environment {
  bool noTempi = false;      // TEMPI_DISABLE
  bool noPack = false;       // TEMPI_NO_PACK
  bool noTypeCommit = false; // TEMPI_NO_TYPE_COMMIT
  bool faultPack = false;    // TEMPI_FAULT_PACK (tests): every MPI_Pack / MPI_Unpack kernel launch "fails"
  DatatypeMethod datatype = DatatypeMethod::AUTO;
  ContiguousMethod contiguous = ContiguousMethod::NONE;
  AlltoallvMethod alltoallv = AlltoallvMethod::AUTO;
  PlacementMethod placement = PlacementMethod::NONE; // TEMPI_PLACEMENT_{KAHIP,METIS,RANDOM}
  std::string cacheDir;
};

extern Environment env;

void read_environment();

} // namespace tempi
