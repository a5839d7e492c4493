// tools/hostcost.cpp -- host cost per interposed call on the halo's path:
// hipPointerGetAttributes alone, then rounds of 208 MPI_Isend to this rank
// followed by 208 MPI_Irecv and one MPI_Waitall (the 1-rank halo's posting
// pattern, 26 directions x 8 quantities) with small strided device types, so
// the host side dominates. One JSON line: microseconds per call.
//   mpiexec -n 1 tools/hostcost [ROUNDS]
// Build: make tools/hostcost (see the Makefile rule for tools).
#include <hip/hip_runtime.h>
#include <mpi.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
  MPI_Init(&argc, &argv);
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 200;
  const int kMsgs = 208;
  char *buf = nullptr;
  if (hipMalloc(&buf, 64 << 20) != hipSuccess) return 2;

  // 1. the pointer query TEMPI makes per call
  hipPointerAttribute_t a;
  const int nq = 200000;
  double t0 = now();
  for (int i = 0; i < nq; ++i) (void)hipPointerGetAttributes(&a, buf + (i % 4096) * 64);
  const double ptrUs = (now() - t0) / nq * 1e6;

  // 2. a small 3D subarray (3 x 4 x 24 B rows of a 16 x 16 x 512 B block)
  int sizes[3] = {16, 16, 512}, subs[3] = {3, 4, 24}, starts[3] = {2, 3, 64};
  MPI_Datatype t;
  MPI_Type_create_subarray(3, sizes, subs, starts, MPI_ORDER_C, MPI_BYTE, &t);
  MPI_Type_commit(&t);
  const size_t stride = 16 * 16 * 512;
  std::vector<MPI_Request> reqs(2 * kMsgs);
  double tSend = 0, tRecv = 0, tWait = 0;
  for (int r = 0; r < rounds + 5; ++r) {
    const double a0 = now();
    for (int i = 0; i < kMsgs; ++i)
      MPI_Isend(buf + size_t(i % 64) * stride, 1, t, 0, i, MPI_COMM_WORLD, &reqs[size_t(i)]);
    const double a1 = now();
    for (int i = 0; i < kMsgs; ++i)
      MPI_Irecv(buf + size_t(64 + i % 64) * stride, 1, t, 0, i, MPI_COMM_WORLD, &reqs[size_t(kMsgs + i)]);
    const double a2 = now();
    MPI_Waitall(2 * kMsgs, reqs.data(), MPI_STATUSES_IGNORE);
    const double a3 = now();
    if (r >= 5) {
      tSend += a1 - a0;
      tRecv += a2 - a1;
      tWait += a3 - a2;
    }
  }
  std::printf("{\"pointer_query_us\": %.3f, \"isend_us\": %.3f, \"irecv_us\": %.3f, \"waitall_us_per_round\": %.1f, "
              "\"rounds\": %d, \"messages_per_round\": %d}\n",
              ptrUs, tSend / rounds / kMsgs * 1e6, tRecv / rounds / kMsgs * 1e6, tWait / rounds * 1e6, rounds, kMsgs);
  MPI_Type_free(&t);
  (void)hipFree(buf);
  MPI_Finalize();
  return 0;
}
