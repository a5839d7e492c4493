// tools/hostbench.cpp -- host-side cost of the primitives the transport uses
// per message, on the GPU box (singleton MPI, the library directly -- not
// through libtempi): hipPointerGetAttributes, event record / query, a
// batched launch, MPI_Isend to self + MPI_Request_free, MPI_Irecv matching an
// unexpected self message, MPI_Test, MPI_Pack_size.
//   hostbench N
#include "tempi_hip.h"

#include <mpi.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define T(name, body)                                                                              \
  do {                                                                                             \
    const double t0_ = now_us();                                                                   \
    for (int i = 0; i < n; ++i) {                                                                  \
      body;                                                                                        \
    }                                                                                              \
    std::printf("{\"op\": \"%s\", \"us\": %.3f}\n", name, (now_us() - t0_) / n);                     \
  } while (0)

int main(int argc, char **argv) {
  MPI_Init(&argc, &argv);
  const int n = argc > 1 ? std::atoi(argv[1]) : 2000;
  void *dev = nullptr, *s = nullptr;
  tempi_hip_malloc(&dev, 1 << 24);
  tempi_hip_stream_create(&s);
  tempi_hip_ptrinfo info;
  T("hipPointerGetAttributes", tempi_hip_pointer_info(static_cast<char *>(dev) + i, &info));
  std::vector<void *> ev(static_cast<size_t>(n), nullptr);
  for (auto &e : ev) tempi_hip_event_create(&e, 0);
  T("hipEventRecord", tempi_hip_event_record(ev[size_t(i)], s));
  T("hipEventQuery", tempi_hip_event_query(ev[size_t(i)]));
  tempi_hip_copy_item it{};
  it.dst_first = dev;
  it.src_first = static_cast<char *>(dev) + (1 << 23);
  it.dst.block = it.src.block = 4096;
  it.dst.ndims = it.src.ndims = 1;
  it.dst.counts[0] = it.src.counts[0] = 2;
  it.dst.strides[0] = it.src.strides[0] = 8192;
  std::vector<tempi_hip_copy_item> items(16, it);
  T("copy_batch(1 item) launch", tempi_hip_copy_batch(items.data(), 1, s));
  tempi_hip_stream_synchronize(s);
  T("copy_batch(16 items) launch", tempi_hip_copy_batch(items.data(), 16, s));
  tempi_hip_stream_synchronize(s);
  char desc[160] = {0};
  std::vector<char> rbuf(160 * static_cast<size_t>(n));
  T("MPI_Isend self + Request_free", {
    MPI_Request r;
    MPI_Isend(desc, 160, MPI_PACKED, 0, i % 300, MPI_COMM_WORLD, &r);
    MPI_Request_free(&r);
  });
  std::vector<MPI_Request> rr(static_cast<size_t>(n));
  T("MPI_Irecv (unexpected queue, in order)",
    MPI_Irecv(&rbuf[size_t(i) * 160], 160, MPI_PACKED, 0, i % 300, MPI_COMM_WORLD, &rr[size_t(i)]));
  T("MPI_Test (complete)", {
    int f;
    MPI_Test(&rr[size_t(i)], &f, MPI_STATUS_IGNORE);
  });
  int ps;
  T("MPI_Pack_size", MPI_Pack_size(i + 1, MPI_BYTE, MPI_COMM_WORLD, &ps));
  MPI_Finalize();
  return 0;
}
