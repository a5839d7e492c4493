// tools/postbench.cpp -- host cost of posting through libtempi: a burst of
// MPI_Isend to this same rank (the self channel), then the matching MPI_Irecv
// burst, then MPI_Waitall, as the halo's substep does, with small strided
// device objects so the GPU work stays negligible. Prints per-call µs of each
// phase (median over ROUNDS bursts).
// build (one command):
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 -Iinclude -I/opt/conda/include -o tempi_amd/lib/postbench
//     tools/postbench.cpp -Ltempi_amd/lib -ltempi -L/opt/conda/lib -lmpi -Wl,-rpath,'$ORIGIN'
//     -Wl,-rpath,/opt/conda/lib
//   mpiexec -n 1 tempi_amd/lib/postbench ROUNDS BURST
#include <hip/hip_runtime.h>
#include <mpi.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

int main(int argc, char **argv) {
  MPI_Init(&argc, &argv);
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 200;
  const int burst = argc > 2 ? std::atoi(argv[2]) : 208;
  char *buf = nullptr;
  if (hipMalloc(&buf, 1 << 22) != hipSuccess) MPI_Abort(MPI_COMM_WORLD, 1);
  MPI_Datatype t;
  MPI_Type_vector(16, 24, 4608, MPI_BYTE, &t); // a sliver of a halo x face
  MPI_Type_commit(&t);
  std::vector<MPI_Request> reqs(2 * size_t(burst));
  std::vector<double> ts, tr, tw;
  for (int r = 0; r < rounds + 5; ++r) {
    const double t0 = MPI_Wtime();
    for (int i = 0; i < burst; ++i) MPI_Isend(buf + (i % 64) * 24, 1, t, 0, i, MPI_COMM_WORLD, &reqs[size_t(i)]);
    const double t1 = MPI_Wtime();
    for (int i = 0; i < burst; ++i)
      MPI_Irecv(buf + (1 << 21) + (i % 64) * 24, 1, t, 0, i, MPI_COMM_WORLD, &reqs[size_t(burst + i)]);
    const double t2 = MPI_Wtime();
    MPI_Waitall(2 * burst, reqs.data(), MPI_STATUSES_IGNORE);
    const double t3 = MPI_Wtime();
    if (r >= 5) {
      ts.push_back((t1 - t0) / burst);
      tr.push_back((t2 - t1) / burst);
      tw.push_back(t3 - t2);
    }
  }
  auto med = [](std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  std::printf("{\"burst\": %d, \"rounds\": %d, \"isend_us\": %.4f, \"irecv_us\": %.4f, \"waitall_us\": %.2f}\n", burst,
              rounds, med(ts) * 1e6, med(tr) * 1e6, med(tw) * 1e6);
  MPI_Type_free(&t);
  hipFree(buf);
  MPI_Finalize();
  return 0;
}
