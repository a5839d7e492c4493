// apps/pingpong_1d.cpp -- CLI for the contiguous ping-pong of the reference's
// bench_mpi_pingpong_1d (MPI_BYTE count = TOTAL, device buffers, ranks r and
// r + size/2 paired, all pairs at once; tempi_bench_pingpong_1d in
// apps/bench_lib.cpp). TEMPI_CONTIGUOUS_* / TEMPI_DATATYPE_* pick the method.
//
// usage: mpiexec -n 2k pingpong_1d ITERS TOTAL_BYTES... [--check]   one JSON object per size
#include <mpi.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

extern "C" int tempi_bench_pingpong_1d(int iters, long total, int check, int setDevice, char *json, int jsonCap);

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
  if (size < 2 || pos.size() < 1) {
    if (!rank) std::fprintf(stderr, "usage: %s ITERS [TOTAL...] [--check] (2+ ranks)\n", argv[0]);
    MPI_Abort(MPI_COMM_WORLD, 1);
  }
  if (pos.size() == 1) { // the reference's sizes (bench_mpi_pingpong_1d.cpp:135)
    pos.push_back(1L << 21);
    pos.push_back(1L << 24);
  }
  int rc = 0;
  std::vector<char> json(1024, 0);
  for (size_t k = 1; k < pos.size(); ++k) {
    rc |= tempi_bench_pingpong_1d(int(pos[0]), pos[k], check, 1, json.data(), int(json.size()));
    if (rank == 0) std::printf("%s\n", json.data());
    std::fflush(stdout);
  }
  MPI_Finalize();
  return rc;
}
