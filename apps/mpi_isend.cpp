// apps/mpi_isend.cpp -- CLI for the reference's bench_mpi_isend
// (/root/reference/bin/bench_mpi_isend.cpp): ranks 0 and 1 ping-pong 10
// overlapping contiguous MPI_BYTE messages per size over device buffers
// (tempi_bench_isend in apps/bench_lib.cpp); the reference's sizes,
// 1 B .. 1 MiB, when none are given.
//
// usage: mpiexec -n 2 mpi_isend ITERS [BYTES...] [--tags N] [--check]   one JSON object per size
#include <mpi.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

extern "C" int tempi_bench_isend(int iters, long bytes, int tags, int check, char *json, int jsonCap);

int main(int argc, char **argv) {
  MPI_Init(&argc, &argv);
  int rank, size;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &size);
  int check = 0, tags = 10;
  std::vector<long> pos;
  for (int i = 1; i < argc; ++i) {
    if (std::string(argv[i]) == "--check")
      check = 1;
    else if (std::string(argv[i]) == "--tags" && i + 1 < argc)
      tags = std::atoi(argv[++i]);
    else
      pos.push_back(std::atol(argv[i]));
  }
  if (size < 2 || pos.empty()) {
    if (!rank) std::fprintf(stderr, "usage: %s ITERS [BYTES...] [--tags N] [--check] (2+ ranks)\n", argv[0]);
    MPI_Abort(MPI_COMM_WORLD, 1);
  }
  if (pos.size() == 1) // the reference's sizes (bench_mpi_isend.cpp:104-107)
    for (long n : {1L, 2L, 4L, 8L, 16L, 32L, 64L, 128L, 256L, 512L, 1024L, 1L << 11, 4096L, 1L << 13, 16384L,
                   1L << 15, 65536L, 1L << 17, 1L << 20})
      pos.push_back(n);
  int rc = 0;
  std::vector<char> json(1024, 0);
  for (size_t k = 1; k < pos.size(); ++k) {
    rc |= tempi_bench_isend(int(pos[0]), pos[k], tags, check, json.data(), int(json.size()));
    if (rank == 0) std::printf("%s\n", json.data());
    std::fflush(stdout);
  }
  MPI_Finalize();
  return rc;
}
