// tempi_amd/csrc/core/next_mpi.hpp -- the MPI library underneath TEMPI.
//
// Every MPI symbol TEMPI exports is resolved to the NEXT definition in the
// dynamic-link search order with dlsym(RTLD_NEXT, ...), as the reference does
// (/root/reference/src/internal/symbols.cpp:14-51) -- not through PMPI, so
// TEMPI chains with PMPI tools. When RTLD_NEXT finds nothing (libtempi was
// dlopen'ed after the MPI library, e.g. from Python), the MPI library named by
// TEMPI_MPI_LIBRARY (default libmpi.so.12) is searched directly. A definition
// that lives in libtempi itself is never accepted (no self-recursion).
#pragma once

#include <mpi.h>

#define TEMPI_NEXT_FUNCS(X)                                                    \
  X(MPI_Init)                                                                  \
  X(MPI_Init_thread)                                                           \
  X(MPI_Query_thread)                                                          \
  X(MPI_Finalize)                                                              \
  X(MPI_Type_commit)                                                           \
  X(MPI_Type_free)                                                             \
  X(MPI_Pack)                                                                  \
  X(MPI_Unpack)                                                                \
  X(MPI_Send)                                                                  \
  X(MPI_Recv)                                                                  \
  X(MPI_Isend)                                                                 \
  X(MPI_Irecv)                                                                 \
  X(MPI_Wait)                                                                  \
  X(MPI_Waitall)                                                               \
  X(MPI_Test)                                                                  \
  X(MPI_Testsome)                                                              \
  X(MPI_Testall)                                                               \
  X(MPI_Testany)                                                               \
  X(MPI_Waitany)                                                               \
  X(MPI_Waitsome)                                                              \
  X(MPI_Request_free)                                                          \
  X(MPI_Request_get_status)                                                    \
  X(MPI_Cancel)                                                                \
  X(MPI_Sendrecv)                                                              \
  X(MPI_Probe)                                                                 \
  X(MPI_Iprobe)                                                                \
  X(MPI_Mprobe)                                                                \
  X(MPI_Improbe)                                                               \
  X(MPI_Mrecv)                                                                 \
  X(MPI_Imrecv)                                                                \
  X(MPI_Barrier)                                                               \
  X(MPI_Ssend)                                                                 \
  X(MPI_Bsend)                                                                 \
  X(MPI_Rsend)                                                                 \
  X(MPI_Issend)                                                                \
  X(MPI_Ibsend)                                                                \
  X(MPI_Irsend)                                                                \
  X(MPI_Send_init)                                                             \
  X(MPI_Ssend_init)                                                            \
  X(MPI_Bsend_init)                                                            \
  X(MPI_Rsend_init)                                                            \
  X(MPI_Recv_init)                                                             \
  X(MPI_Start)                                                                 \
  X(MPI_Startall)                                                              \
  X(MPI_Sendrecv_replace)                                                      \
  X(MPI_Buffer_detach)                                                         \
  X(MPI_Alltoallv)                                                             \
  X(MPI_Neighbor_alltoallv)                                                    \
  X(MPI_Neighbor_alltoallw)                                                    \
  X(MPI_Dist_graph_create_adjacent)                                            \
  X(MPI_Dist_graph_neighbors)                                                  \
  X(MPI_Comm_rank)                                                             \
  X(MPI_Comm_free)

namespace tempi {

struct NextMPI {
#define TEMPI_X(f) decltype(&::f) f = nullptr;
  TEMPI_NEXT_FUNCS(TEMPI_X)
#undef TEMPI_X
};

extern NextMPI next;

// idempotent; aborts if a symbol cannot be found anywhere
void resolve_next();

} // namespace tempi
