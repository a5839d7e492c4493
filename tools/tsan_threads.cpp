// tools/tsan_threads.cpp -- MPI_THREAD_MULTIPLE through libtempi under
// ThreadSanitizer (host code only; tools/cpu_tsan.sh builds and runs it).
// THREADS threads, no application lock: each sends a strided host object to
// the next rank with its own tag, receives the one the previous rank's next
// thread sent (so its wait depends on another thread), blocks in MPI_Wait,
// then in a host MPI_Recv for a message another thread sent; every byte
// checked. Run with TEMPI_TEST_HOST_ONLY=1 so TEMPI's host-side paths (its
// request table, descriptor-aware receives, the probe loop, progress) are
// the ones the threads share.
// usage: mpiexec -n 1|2 tsan_threads [THREADS ITERS]
#include <mpi.h>

#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

static unsigned char byte_of(int rank, int thread, int it, int i) {
  return (unsigned char)(rank * 131 + thread * 31 + it * 7 + i);
}

int main(int argc, char **argv) {
  int provided = 0;
  MPI_Init_thread(&argc, &argv, MPI_THREAD_MULTIPLE, &provided);
  int rank, size;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &size);
  const int nth = argc > 1 ? std::atoi(argv[1]) : 3;
  const int iters = argc > 2 ? std::atoi(argv[2]) : 100;
  const int peer = (rank + 1) % size, src = (rank + size - 1) % size;
  MPI_Datatype t; // 64 rows of 24 bytes at stride 96
  MPI_Type_vector(64, 24, 96, MPI_BYTE, &t);
  MPI_Type_commit(&t);
  const int ext = 63 * 96 + 24;
  std::vector<long> errors(size_t(nth), 0);
  auto worker = [&](int w) {
    const int partner = (w + 1) % nth;
    std::vector<unsigned char> sb(static_cast<size_t>(ext)), rb(static_cast<size_t>(ext)), hs(256), hr(256);
    for (int it = 0; it < iters; ++it) {
      for (int i = 0; i < ext; ++i) sb[size_t(i)] = byte_of(rank, w, it, i);
      for (int i = 0; i < 256; ++i) hs[size_t(i)] = byte_of(rank, w, it, i + 5);
      std::fill(rb.begin(), rb.end(), 0);
      MPI_Request sq, hq, rq;
      MPI_Isend(sb.data(), 1, t, peer, 100 + w, MPI_COMM_WORLD, &sq);
      MPI_Isend(hs.data(), 256, MPI_BYTE, peer, 300 + w, MPI_COMM_WORLD, &hq);
      MPI_Irecv(rb.data(), 1, t, src, 100 + partner, MPI_COMM_WORLD, &rq);
      MPI_Wait(&rq, MPI_STATUS_IGNORE);
      MPI_Recv(hr.data(), 256, MPI_BYTE, src, 300 + partner, MPI_COMM_WORLD, MPI_STATUS_IGNORE);
      MPI_Wait(&sq, MPI_STATUS_IGNORE);
      MPI_Wait(&hq, MPI_STATUS_IGNORE);
      for (int r = 0; r < 64; ++r)
        for (int i = 0; i < 24; ++i) {
          const int at = r * 96 + i;
          errors[size_t(w)] += rb[size_t(at)] != byte_of(src, partner, it, at);
        }
      for (int i = 0; i < 256; ++i) errors[size_t(w)] += hr[size_t(i)] != byte_of(src, partner, it, i + 5);
    }
  };
  std::vector<std::thread> ths;
  for (int w = 0; w < nth; ++w) ths.emplace_back(worker, w);
  for (auto &th : ths) th.join();
  long e = 0;
  for (long x : errors) e += x;
  MPI_Type_free(&t);
  MPI_Finalize();
  std::printf("RESULT errors=%ld provided=%d\n", e, provided);
  return e ? 1 : 0;
}
