// tempi_amd/csrc/core/state.hpp -- process-wide TEMPI state shared by the
// interposed entry points.
#pragma once

#include <mpi.h>

namespace tempi {

struct State {
  bool active = false; // MPI initialised through TEMPI and TEMPI not disabled
  int worldRank = 0;
  int worldSize = 1;
};

extern State state;

// raise `code` on the communicator's error handler (as the library would)
// and return it
int raise_error(MPI_Comm comm, int code);

// bring up / tear down everything after the library's MPI_Init / before its
// MPI_Finalize
void init_after_mpi();
void finalize_before_mpi();

} // namespace tempi
