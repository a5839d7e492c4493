// apps/alltoallv_sparse.cpp -- CLI for config 5: MPI_Alltoallv of device
// buffers with the reference's random sparse byte-count matrices
// (tempi_bench_alltoallv in apps/bench_lib.cpp, after
// /root/reference/bin/bench_alltoallv_random_sparse.cpp:160-222).
//
// --neighbor: the same matrices as the distributed graph of the reference's
// bench_nbr_alltoallv_random_sparse (MPI_Dist_graph_create_adjacent with
// reorder = 1, then MPI_Neighbor_alltoallv: tempi_bench_nbr_alltoallv);
// --no-reorder creates the graph with reorder = 0.
//
// usage: mpiexec -n N alltoallv_sparse ITERS [--scale S] [--density D] [--seed K] [--check]
//                                           [--neighbor [--no-reorder]]
//        mpiexec -n N alltoallv_sparse ITERS --sweep   (the reference's scales x densities)
// One JSON object per point (rank 0).
#include <mpi.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <set>
#include <vector>

extern "C" int tempi_bench_alltoallv(int iters, int scale, double density, int seed, int check, int setDevice,
                                     char *json, int jsonCap);
extern "C" int tempi_bench_nbr_alltoallv(int iters, int scale, double density, int seed, int reorder, int check,
                                         int setDevice, char *json, int jsonCap);

int main(int argc, char **argv) {
  MPI_Init(&argc, &argv);
  int rank, size;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &size);
  int iters = argc > 1 ? std::atoi(argv[1]) : 30, scale = 1000, seed = 101, check = 0, sweep = 0, neighbor = 0,
      reorder = 1;
  double density = 1.0;
  for (int i = 2; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--scale") && i + 1 < argc) scale = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--density") && i + 1 < argc) density = std::atof(argv[++i]);
    else if (!std::strcmp(argv[i], "--seed") && i + 1 < argc) seed = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--check")) check = 1;
    else if (!std::strcmp(argv[i], "--sweep")) sweep = 1;
    else if (!std::strcmp(argv[i], "--neighbor")) neighbor = 1;
    else if (!std::strcmp(argv[i], "--no-reorder")) reorder = 0;
  }
  std::vector<int> scales{scale};
  std::set<double> densities{density};
  if (sweep) { // /root/reference/bin/bench_alltoallv_random_sparse.cpp:176-189 (and
               // bench_nbr_alltoallv_random_sparse.cpp:344-355)
    scales = {1, 10, 100, 1000, 10000, 100000, 1000000};
    densities = {1.0, 0.5, 0.1, 0.05};
    for (int nnz : {1, 2, 4, 8, 16})
      if (double(nnz) / size <= 1) densities.insert(double(nnz) / size);
  }
  int rc = 0;
  std::vector<char> json(1024, 0);
  for (int s : scales)
    for (double d : densities) {
      rc |= neighbor ? tempi_bench_nbr_alltoallv(iters, s, d, seed, reorder, check, 1, json.data(), int(json.size()))
                     : tempi_bench_alltoallv(iters, s, d, seed, check, 1, json.data(), int(json.size()));
      if (rank == 0) std::printf("%s\n", json.data());
      std::fflush(stdout);
    }
  MPI_Finalize();
  return rc;
}
