// tempi_amd/csrc/core/placement.hpp -- rank placement for
// MPI_Dist_graph_create_adjacent(..., reorder = 1, ...).
//
// Reference: /root/reference/src/dist_graph_create_adjacent.cpp:55-470 with
// partition.cpp:27-50, partition_{kahip,metis}.cpp and make_placement
// (topology.cpp:97-144). When the communicator spans more than one node with
// more than one rank per node (the guard at :98; on one node nothing moves,
// SURVEY F12), the communication graph is gathered to rank 0, partitioned
// into one part per node (part sizes = the nodes' rank counts), and
// application rank q is given to the process that make_placement picks on
// q's node. Process p then presents old rank q's edges as its own, as the
// reference does (:371-431).
//
// What differs:
//   - the partitioner is TEMPI's own (TEMPI_PLACEMENT_KAHIP and
//     TEMPI_PLACEMENT_METIS both select it; neither library is in this image,
//     SURVEY 8(c)): graph growing from several seeds, then balance-preserving
//     pairwise-swap (Kernighan-Lin) refinement of the edge cut; exact part
//     sizes, so nodes with unequal rank counts work too;
//   - TEMPI_PLACEMENT_RANDOM is the reference's rule (partition.cpp:27-34:
//     i * nodes / ranks, shuffled by a default_random_engine seeded 0 and
//     shared by every call);
//   - the new communicator is created by the library on a split of comm_old
//     keyed by application rank, with reorder = 0, so its rank numbers ARE the
//     application's: MPI_Comm_rank, MPI_Dist_graph_neighbors, every
//     point-to-point call, status MPI_SOURCE and every collective are right
//     without translation (the reference translates ranks in Comm_rank,
//     Dist_graph_neighbors and its device send/receive paths only, so a
//     library collective on its reordered communicator sees library order);
//   - its traffic (edge gather, partition broadcast, edge exchange) runs on a
//     private duplicate of comm_old, never on the application's tags.
// TEMPI_FAKE_NODE_SIZE=k (tests) groups the ranks into nodes of k consecutive
// world ranks for placement only; the transport's co-location is unchanged.
#pragma once

#include "env.hpp"

#include <mpi.h>

#include <cstdint>
#include <vector>

namespace tempi {
namespace placement {

// undirected weighted graph in CSR form, no self loops, one entry per
// neighbour (weights of both directions and repeated edges summed)
struct Graph {
  int n = 0;
  std::vector<int> xadj, adj;
  std::vector<int64_t> w;
};

struct Edge {
  int u, v;
  int64_t w;
};

Graph make_graph(int n, const std::vector<Edge> &edges);

// sum of the weights of edges whose ends are in different parts
int64_t edge_cut(const Graph &g, const std::vector<int> &part);

// part[v] in [0, sizes.size()), exactly sizes[k] vertices in part k
std::vector<int> partition(const Graph &g, const std::vector<int> &sizes);

// the reference's random placement (partition.cpp:27-34) with part sizes
// `sizes` (equal sizes give its exact sequence); advances one generator
std::vector<int> random_parts(const std::vector<int> &sizes);

// MPI_Dist_graph_create_adjacent with TEMPI's placement. Returns false (and
// does nothing) when no placement applies: env.placement NONE, reorder == 0, one
// node, or one rank per node; the caller then makes the library call.
bool create(MPI_Comm comm_old, int indegree, const int sources[], const int sourceweights[], int outdegree,
            const int destinations[], const int destweights[], MPI_Info info, int reorder,
            MPI_Comm *comm_dist_graph, int *rc);

// the last placement this process took part in
struct Info {
  int placed = 0;  // 1 after a placement
  int nodes = 0;   // parts
  int method = 0;  // PlacementMethod
  int appRank = -1; // this process's rank in the new communicator
  int64_t cutIdentity = 0, cutPlaced = 0; // edge cut of the library's order / of the placement (rank 0's graph)
};
Info last();

} // namespace placement
} // namespace tempi
