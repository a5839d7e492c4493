// tools/flagbench.hip -- host-observed completion of a small kernel on MI355X:
// hipStreamSynchronize, against the host spinning on a flag in pinned memory
// written (system-scope release) by a one-lane kernel queued behind it, or by
// the last workgroup of the kernel itself (each workgroup fencing at system
// scope first); and HIP's own completion polled instead of waited for:
// hipStreamQuery / hipEventQuery in a spin loop, hipEventSynchronize.
// profiles/r02/completion_flag_bench_s11.jsonl, _s13.jsonl; DESIGN §6.
//   hipcc --offload-arch=gfx950 -O2 -o flagbench tools/flagbench.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>
#include <algorithm>
__global__ void work(unsigned *p, int n) { int i = blockIdx.x * blockDim.x + threadIdx.x; if (i < n) p[i] += 1; }
__global__ void work_flag(unsigned *p, int n, unsigned *cnt, volatile unsigned *flag, unsigned ticket) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] += 1;
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();
    unsigned old = atomicAdd(cnt, 1u);
    if (old == gridDim.x - 1) { *cnt = 0; __threadfence_system(); __hip_atomic_store((unsigned*)flag, ticket, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM); }
  }
}
__global__ void signal(volatile unsigned *flag, unsigned ticket) {
  if (threadIdx.x == 0 && blockIdx.x == 0) __hip_atomic_store((unsigned*)flag, ticket, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
static double now_us() { return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
int main() {
  unsigned *d, *cnt; hipMalloc(&d, 1 << 22); hipMalloc(&cnt, 4); hipMemset(cnt, 0, 4);
  unsigned *flag; hipHostMalloc(&flag, 64, hipHostMallocMapped | hipHostMallocCoherent); *flag = 0;
  unsigned *dflag; hipHostGetDevicePointer((void**)&dflag, flag, 0);
  hipStream_t s; hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipEvent_t ev; hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  for (int blocks : {1, 64, 512}) {
    int n = blocks * 256;
    std::vector<double> a, b, c, q, eq, es;
    unsigned ticket = 1;
    for (int it = 0; it < 300; ++it) {
      double t0 = now_us(); hipLaunchKernelGGL(work, dim3(blocks), dim3(256), 0, s, d, n); hipStreamSynchronize(s); a.push_back(now_us() - t0);
      ++ticket; t0 = now_us(); hipLaunchKernelGGL(work, dim3(blocks), dim3(256), 0, s, d, n);
      hipLaunchKernelGGL(signal, dim3(1), dim3(64), 0, s, dflag, ticket);
      while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != ticket) __builtin_ia32_pause(); b.push_back(now_us() - t0);
      hipStreamSynchronize(s);
      ++ticket; t0 = now_us(); hipLaunchKernelGGL(work_flag, dim3(blocks), dim3(256), 0, s, d, n, cnt, dflag, ticket);
      while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != ticket) __builtin_ia32_pause(); c.push_back(now_us() - t0);
      hipStreamSynchronize(s);
      t0 = now_us(); hipLaunchKernelGGL(work, dim3(blocks), dim3(256), 0, s, d, n);
      while (hipStreamQuery(s) == hipErrorNotReady) __builtin_ia32_pause(); q.push_back(now_us() - t0);
      t0 = now_us(); hipLaunchKernelGGL(work, dim3(blocks), dim3(256), 0, s, d, n); hipEventRecord(ev, s);
      while (hipEventQuery(ev) == hipErrorNotReady) __builtin_ia32_pause(); eq.push_back(now_us() - t0);
      t0 = now_us(); hipLaunchKernelGGL(work, dim3(blocks), dim3(256), 0, s, d, n); hipEventRecord(ev, s);
      hipEventSynchronize(ev); es.push_back(now_us() - t0);
    }
    auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
    printf("{\"blocks\": %d, \"sync_us\": %.2f, \"signal_kernel_flag_us\": %.2f, \"last_wg_flag_us\": %.2f, "
           "\"stream_query_poll_us\": %.2f, \"event_query_poll_us\": %.2f, \"event_sync_us\": %.2f}\n",
           blocks, med(a), med(b), med(c), med(q), med(eq), med(es));
  }
  return 0;
}
