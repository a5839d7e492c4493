// tempi_amd/csrc/core/state.hpp -- process-wide TEMPI state shared by the
// interposed entry points.
#pragma once

#include <mpi.h>

#include <cstdint>

namespace tempi {

struct State {
  bool active = false; // MPI initialised through TEMPI and TEMPI not disabled
  int worldRank = 0;
  int worldSize = 1;
  int32_t pid = 0; // getpid() at MPI_Init (glibc no longer caches it: a syscall per call)
};

extern State state;

// raise `code` on the communicator's error handler (as the library would)
// and return it
int raise_error(MPI_Comm comm, int code);

// bring up / tear down everything after the library's MPI_Init / before its
// MPI_Finalize
void init_after_mpi();
void finalize_before_mpi();

// TEMPI's MPI_Pack / MPI_Unpack (GPU kernels, or the library with host
// staging for types that are not strided blocks)
int pack(const void *inbuf, int incount, MPI_Datatype datatype, void *outbuf, int outsize, int *position,
         MPI_Comm comm);
int unpack(const void *inbuf, int insize, int *position, void *outbuf, int outcount, MPI_Datatype datatype,
           MPI_Comm comm);

} // namespace tempi
