// tools/queue_probe.hip -- does a kernel that stays running on one stream hold
// up kernels of the process's other streams? HIP maps streams onto at most
// GPU_MAX_HW_QUEUES hardware queues (4 on the pool); two streams on one queue
// run in one order, so a resident kernel would block its queue-mate until it
// leaves. TEMPI's streams are mimicked (lane 0 at high priority, lanes 1-2,
// the null stream), then the "server" stream is made one way or another, a
// kernel spins 20 ms on it, and a trivial kernel + synchronise is timed on
// every other stream. One JSON line per way of making the server stream.
// usage: queue_probe
//   hipcc --offload-arch=gfx950 -O2 -o tools/bin/queue_probe tools/queue_probe.hip
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
__global__ void spin(uint64_t ticks, uint32_t *flag) {
  const uint64_t t0 = wall_clock64();
  while (int64_t(wall_clock64() - t0) < int64_t(ticks)) __builtin_amdgcn_s_sleep(10);
  if (threadIdx.x == 0 && blockIdx.x == 0) __hip_atomic_store(flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void nop() {}

int main() {
  int least = 0, greatest = 0;
  hipDeviceGetStreamPriorityRange(&least, &greatest);
  uint32_t *flag;
  hipHostMalloc(reinterpret_cast<void **>(&flag), 64, hipHostMallocMapped | hipHostMallocCoherent);
  const char *ways[] = {"normal", "high", "low", "cumask_all", "first_created"};
  for (const char *way : ways) {
    std::vector<hipStream_t> others;
    hipStream_t server = nullptr;
    auto make_server = [&]() {
      if (!std::strcmp(way, "high"))
        hipStreamCreateWithPriority(&server, hipStreamNonBlocking, greatest);
      else if (!std::strcmp(way, "low"))
        hipStreamCreateWithPriority(&server, hipStreamNonBlocking, least);
      else if (!std::strcmp(way, "cumask_all")) {
        uint32_t mask[8];
        for (auto &m : mask) m = 0xffffffffu;
        hipExtStreamCreateWithCUMask(&server, 8, mask);
      } else
        hipStreamCreateWithFlags(&server, hipStreamNonBlocking);
    };
    if (!std::strcmp(way, "first_created")) make_server();
    hipStream_t s;
    hipStreamCreateWithPriority(&s, hipStreamNonBlocking, greatest); // lane 0
    others.push_back(s);
    for (int i = 0; i < 2; ++i) {
      hipStreamCreateWithPriority(&s, hipStreamNonBlocking, least); // lanes 1, 2
      others.push_back(s);
    }
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking); // torch-like stream
    others.push_back(s);
    if (std::strcmp(way, "first_created")) make_server();
    *flag = 0;
    hipLaunchKernelGGL(spin, dim3(97), dim3(128), 0, server, uint64_t(2000000), flag); // 20 ms
    while (!__atomic_load_n(flag, __ATOMIC_ACQUIRE) && false) {}
    std::string res;
    for (size_t i = 0; i <= others.size(); ++i) {
      hipStream_t t = i < others.size() ? others[i] : nullptr; // last: the null stream
      const double t0 = now_us();
      hipLaunchKernelGGL(nop, dim3(1), dim3(64), 0, t);
      hipStreamSynchronize(t);
      char b[64];
      std::snprintf(b, sizeof b, "%s%.0f", i ? ", " : "", now_us() - t0);
      res += b;
    }
    hipStreamSynchronize(server);
    std::printf("{\"probe\": \"queue_sharing\", \"server_stream\": \"%s\", \"nop_us_on_lane0_lane1_lane2_other_null\": [%s]}\n",
                way, res.c_str());
    std::fflush(stdout);
    for (hipStream_t x : others) hipStreamDestroy(x);
    hipStreamDestroy(server);
  }
  return 0;
}
