// apps/halo_exchange_main.cpp -- CLI for the 3D halo exchange of
// apps/halo_lib.cpp (config 4):
//   mpiexec -n N halo_exchange ITERS X [Y Z] [--quants N] [--radius R] [--check] [--neighbor] [--reorder]
#include <mpi.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

extern "C" int tempi_bench_halo(int nIters, int gx, int gy, int gz, int nQuants, int radius, int check,
                                int neighbor, int setDevice, char *json, int jsonCap);

int main(int argc, char **argv) {
  MPI_Init(&argc, &argv);
  int rank;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  int nQuants = 8, radius = 3, check = 0, neighbor = 0;
  std::vector<int> pos;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--check"))
      check = 1;
    else if (!std::strcmp(argv[i], "--check-control")) // a planted error the check must find
      check = 2;
    else if (!std::strcmp(argv[i], "--neighbor"))
      neighbor |= 1;
    else if (!std::strcmp(argv[i], "--reorder")) // placed ranks (TEMPI_PLACEMENT_*)
      neighbor |= 2;
    else if (!std::strcmp(argv[i], "--quants") && i + 1 < argc)
      nQuants = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--radius") && i + 1 < argc)
      radius = std::atoi(argv[++i]);
    else
      pos.push_back(std::atoi(argv[i]));
  }
  if (pos.size() != 2 && pos.size() != 4) {
    if (!rank) std::fprintf(stderr, "usage: %s ITERS X [Y Z] [--quants N] [--radius R] [--check] [--neighbor] [--reorder]\n", argv[0]);
    MPI_Abort(MPI_COMM_WORLD, 1);
  }
  std::vector<char> json(4096, 0);
  const int rc = tempi_bench_halo(pos[0], pos[1], pos.size() == 4 ? pos[2] : pos[1],
                                  pos.size() == 4 ? pos[3] : pos[1], nQuants, radius, check, neighbor, 1, json.data(),
                                  int(json.size()));
  if (rank == 0) std::printf("%s\n", json.data());
  MPI_Finalize();
  return rc;
}
