// tempi_amd/csrc/core/topology.hpp -- which ranks share this node.
//
// The reference allgathers MPI_Get_processor_name at init and per cached
// communicator (/root/reference/src/internal/topology.cpp:34-90) and answers
// is_colocated (:191-196). Here: one allgather of host names over
// MPI_COMM_WORLD at MPI_Init; other communicators are mapped to world ranks
// with MPI_Group_translate_ranks once, cached per handle and dropped by the
// interposed MPI_Comm_free before the library frees (and may reuse) the
// handle (/root/reference/src/comm_free.cpp:13-19 does the same). Rank
// placement (core/placement.hpp) needs no app/library rank translation here:
// its communicator is created with the application's rank order.
#pragma once

#include <mpi.h>

namespace tempi {
namespace topology {

void init();
void finalize();
int world_rank(MPI_Comm comm, int rank); // MPI_UNDEFINED if not in world
void uncache(MPI_Comm comm);              // the handle is about to be freed
bool colocated(MPI_Comm comm, int rank);
bool colocated_world(int worldRank);
int node_of_world(int worldRank); // index of the node (host name), numbered by first world rank on it
int node_local_rank(); // this rank's index among the ranks on its node
int ranks_on_node();

} // namespace topology
} // namespace tempi
