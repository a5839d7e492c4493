// tempi_amd/csrc/core/topology.cpp -- see topology.hpp
#include "topology.hpp"

#include "log.hpp"
#include "state.hpp"

#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

namespace tempi {
namespace topology {

namespace {
std::vector<int> nodeOf; // world rank -> node index
int myNode = 0, localRank = 0, nodeRanks = 1;
// communicator -> world rank of each of its ranks (remote group for an
// intercommunicator); dropped by MPI_Comm_free (uncache)
std::unordered_map<MPI_Comm, std::vector<int>> worldOf;
} // namespace

void init() {
  const int n = state.worldSize;
  std::vector<char> names(size_t(n) * MPI_MAX_PROCESSOR_NAME, 0);
  char mine[MPI_MAX_PROCESSOR_NAME] = {0};
  int len = 0;
  MPI_Get_processor_name(mine, &len);
  MPI_Allgather(mine, MPI_MAX_PROCESSOR_NAME, MPI_CHAR, names.data(), MPI_MAX_PROCESSOR_NAME, MPI_CHAR,
                MPI_COMM_WORLD);
  std::vector<std::string> uniq;
  nodeOf.assign(size_t(n), 0);
  for (int r = 0; r < n; ++r) {
    std::string s(&names[size_t(r) * MPI_MAX_PROCESSOR_NAME]);
    size_t k = 0;
    while (k < uniq.size() && uniq[k] != s) ++k;
    if (k == uniq.size()) uniq.push_back(s);
    nodeOf[size_t(r)] = int(k);
  }
  myNode = nodeOf[size_t(state.worldRank)];
  localRank = 0;
  nodeRanks = 0;
  for (int r = 0; r < n; ++r) {
    if (nodeOf[size_t(r)] != myNode) continue;
    if (r < state.worldRank) ++localRank;
    ++nodeRanks;
  }
  LOG_DEBUG("topology: " << uniq.size() << " node(s), " << nodeRanks << " rank(s) on mine");
}

void finalize() {
  nodeOf.clear();
  worldOf.clear();
}

int world_rank(MPI_Comm comm, int rank) {
  if (comm == MPI_COMM_WORLD) return rank;
  if (rank < 0) return MPI_UNDEFINED;
  auto it = worldOf.find(comm);
  if (it == worldOf.end()) {
    MPI_Group g, wg;
    int inter = 0;
    MPI_Comm_test_inter(comm, &inter);
    if (inter)
      MPI_Comm_remote_group(comm, &g);
    else
      MPI_Comm_group(comm, &g);
    MPI_Comm_group(MPI_COMM_WORLD, &wg);
    int n = 0;
    MPI_Group_size(g, &n);
    std::vector<int> mine(static_cast<size_t>(n)), world(static_cast<size_t>(n), MPI_UNDEFINED);
    for (int i = 0; i < n; ++i) mine[size_t(i)] = i;
    MPI_Group_translate_ranks(g, n, mine.data(), wg, world.data());
    MPI_Group_free(&g);
    MPI_Group_free(&wg);
    it = worldOf.emplace(comm, std::move(world)).first;
  }
  return size_t(rank) < it->second.size() ? it->second[size_t(rank)] : MPI_UNDEFINED;
}

void uncache(MPI_Comm comm) { worldOf.erase(comm); }

bool colocated_world(int w) {
  if (w < 0 || size_t(w) >= nodeOf.size()) return false;
  return nodeOf[size_t(w)] == myNode;
}

int node_of_world(int w) { return w >= 0 && size_t(w) < nodeOf.size() ? nodeOf[size_t(w)] : -1; }

bool colocated(MPI_Comm comm, int rank) { return colocated_world(world_rank(comm, rank)); }

int node_local_rank() { return localRank; }
int ranks_on_node() { return nodeRanks; }

} // namespace topology
} // namespace tempi
