// tools/batchlaunch.hip -- host time of one batched launch, by kernarg size
// and stream state (the halo's batched launches take
// 4.7-5.2 us of host time against 2.35 us for a bare launch). Median of REPS
// calls of:
//   empty_<B>        hipLaunchKernelGGL of an empty kernel whose argument is
//                    B bytes (64, 184, 1024, 3584)
//   copy_batch_<n>   tempi_hip_copy_batch of n small items (x-face rows of
//                    the 1-rank halo, 64 rows each: the kernarg block is the
//                    full CBatchArgs whatever n)
// each on an idle stream (after hipStreamSynchronize) and back-to-back
// (stream still busy with the previous launches: queued, not synchronised).
// usage: batchlaunch [REPS]   (HIP_FORCE_DEV_KERNARG=0|1 to compare HIP's
// kernarg placement)
//   hipcc --offload-arch=gfx950 -O2 -Iinclude -o tools/_variants/batchlaunch tools/batchlaunch.hip
//         -Ltempi_amd/lib -ltempi_hip -Wl,-rpath,'$ORIGIN/../../tempi_amd/lib'
#include <hip/hip_runtime.h>

#include "tempi_hip.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

template <int B> struct Arg {
  unsigned char b[B];
};
template <int B> __global__ void empty_kernel(Arg<B> a) {
  if (a.b[0] == 0xEE && threadIdx.x == 1000) a.b[1] = 0; // never true; keeps the argument
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static double med(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 1000;
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking)) return 3;
  // a 64 x 518 x 518-cell grid of 8-byte cells, pitch 4608 B: x-face rows
  const int64_t pitch = 4608, plane = pitch * 518;
  char *grid = nullptr;
  if (hipMalloc(&grid, size_t(plane) * 70)) return 3;
  std::vector<tempi_hip_copy_item> items(64);
  for (int i = 0; i < 64; ++i) {
    tempi_hip_copy_item &c = items[size_t(i)];
    c = tempi_hip_copy_item{};
    char *base = grid + int64_t(i % 60 + 3) * plane;
    c.src_first = base + 3 * pitch + 512 * 8; // interior x face, 64 rows
    c.dst_first = base + 3 * pitch;           // exterior x face
    for (tempi_hip_desc *d : {&c.src, &c.dst}) {
      d->block = 24;
      d->ndims = 1;
      d->counts[0] = 64;
      d->strides[0] = pitch;
    }
  }
  auto time = [&](const char *name, const std::function<int()> &launch) {
    std::vector<double> idle, busy;
    for (int i = 0; i < reps + 20; ++i) {
      if (hipStreamSynchronize(s)) return 4;
      double t0 = now_us();
      if (launch()) return 5;
      double t1 = now_us();
      if (launch()) return 5; // queued behind the first
      double t2 = now_us();
      if (i >= 20) {
        idle.push_back(t1 - t0);
        busy.push_back(t2 - t1);
      }
    }
    std::printf("{\"bench\": \"batchlaunch\", \"what\": \"%s\", \"idle_us\": %.2f, \"busy_us\": %.2f, \"dev_kernarg\": \"%s\"}\n",
                name, med(idle), med(busy), std::getenv("HIP_FORCE_DEV_KERNARG") ? std::getenv("HIP_FORCE_DEV_KERNARG") : "");
    return 0;
  };
  int e = 0;
  e |= time("empty_64", [&] { hipLaunchKernelGGL(empty_kernel<64>, dim3(256), dim3(128), 0, s, Arg<64>{}); return int(hipGetLastError()); });
  e |= time("empty_184", [&] { hipLaunchKernelGGL(empty_kernel<184>, dim3(256), dim3(128), 0, s, Arg<184>{}); return int(hipGetLastError()); });
  e |= time("empty_1024", [&] { hipLaunchKernelGGL(empty_kernel<1024>, dim3(256), dim3(128), 0, s, Arg<1024>{}); return int(hipGetLastError()); });
  e |= time("empty_3584", [&] { hipLaunchKernelGGL(empty_kernel<3584>, dim3(256), dim3(128), 0, s, Arg<3584>{}); return int(hipGetLastError()); });
  for (int n : {1, 2, 8, 16, 32}) {
    char name[32];
    std::snprintf(name, sizeof name, "copy_batch_%d", n);
    e |= time(name, [&] { return tempi_hip_copy_batch(items.data(), n, s); });
  }
  hipStreamSynchronize(s);
  hipFree(grid);
  return e;
}
