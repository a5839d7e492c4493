// tools/latbench.hip -- host-observed latency floor of one small kernel on
// MI355X: launch + hipEventRecord + poll hipEventQuery until complete, and
// launch + hipStreamSynchronize. Sets the floor for the small-message
// ping-pong (two such round trips per one-way message).
#include <hip/hip_runtime.h>
#pragma clang diagnostic ignored "-Wunused-value"
#pragma clang diagnostic ignored "-Wunused-result"
#include <chrono>
#include <cstdio>

__global__ void tiny(unsigned *p) {
  if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1u;
}

struct Big {
  unsigned n;
  unsigned pad[895]; // 3584 bytes: the batched kernels' argument size
};
__global__ void tiny_big(unsigned *p, Big b) {
  if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += b.n + b.pad[b.n & 7];
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  unsigned *d;
  hipMalloc(&d, 4096);
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipEvent_t ev;
  hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  const int n = 2000;
  Big big{};
  big.n = 1;
  const char *names[] = {"launch+event poll", "launch+stream sync", "memcpyAsync 1KiB D2D+event poll",
                         "launch 3.5 KiB kernarg+event poll"};
  for (int mode = 0; mode < 4; ++mode) {
    double best = 1e30, sum = 0, host = 0;
    for (int i = 0; i < n + 100; ++i) {
      const double t0 = now_us();
      if (mode == 2) {
        hipMemcpyAsync(d + 512, d, 1024, hipMemcpyDeviceToDevice, s);
      } else if (mode == 3) {
        hipLaunchKernelGGL(tiny_big, dim3(1), dim3(64), 0, s, d, big);
      } else {
        hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d);
      }
      const double tl = now_us() - t0;
      if (mode == 1) {
        hipStreamSynchronize(s);
      } else {
        hipEventRecord(ev, s);
        while (hipEventQuery(ev) == hipErrorNotReady) {
        }
      }
      const double t = now_us() - t0;
      if (i >= 100) {
        sum += t;
        host += tl;
        if (t < best) best = t;
      }
    }
    std::printf("{\"mode\": \"%s\", \"mean_us\": %.2f, \"min_us\": %.2f, \"launch_call_us\": %.2f}\n",
                names[mode], sum / n, best, host / n);
  }
  return 0;
}
