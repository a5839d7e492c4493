// apps/pingpong_nd.cpp -- CLI for the strided MPI_Send / MPI_Recv ping-pong of
// device buffers between ranks 0 and 1 (config 3; the workload and checks are
// tempi_bench_pingpong in apps/bench_lib.cpp, after /root/reference/bin/
// bench_mpi_pingpong_nd.cpp:146-197). The method comes from the environment
// (TEMPI_DATATYPE_*).
//
// usage: mpiexec -n 2 pingpong_nd ITERS TOTAL_BYTES BLOCK [STRIDE] [--check]
#include <mpi.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

extern "C" int tempi_bench_pingpong(int iters, long total, long bl, long stride, int check, int setDevice,
                                    char *json, int jsonCap);

int main(int argc, char **argv) {
  MPI_Init(&argc, &argv);
  int rank, size;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &size);
  int check = 0;
  std::vector<long> pos;
  for (int i = 1; i < argc; ++i) {
    if (std::string(argv[i]) == "--check")
      check = 1;
    else
      pos.push_back(std::atol(argv[i]));
  }
  if (size < 2 || pos.size() < 3) {
    if (!rank) std::fprintf(stderr, "usage: %s ITERS TOTAL BLOCK [STRIDE] [--check] (2+ ranks)\n", argv[0]);
    MPI_Abort(MPI_COMM_WORLD, 1);
  }
  std::vector<char> json(1024, 0);
  const int rc = tempi_bench_pingpong(int(pos[0]), pos[1], pos[2], pos.size() > 3 ? pos[3] : 512, check, 1,
                                      json.data(), int(json.size()));
  if (rank == 0) std::printf("%s\n", json.data());
  MPI_Finalize();
  return rc;
}
