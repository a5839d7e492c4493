// tools/smallbatch.hip -- what a small message's batched gather / scatter
// costs, and why (the ONESHOT route of a small device message is one
// gather into pinned host memory and one scatter out of it, each a batch
// kernel of a few microseconds: DESIGN §7). At libtempi_hip's C ABI, one
// item per batch, the ticket folded in, median of REPS calls:
//   call_us   tempi_hip_{pack,unpack}_batch_ticket + tempi_hip_ticket_wait
// for each (direction, packed side, shape):
//   packed side  device memory | pinned host memory (hipHostMalloc, mapped)
//   shape        1 B contiguous | 1 KiB contiguous | 128 rows of 8 B at stride 512
// Run under rocprofv3 --kernel-trace --stats for the kernels' own durations.
// usage: smallbatch [REPS]
//   hipcc --offload-arch=gfx950 -O2 -Iinclude -o tools/_variants/smallbatch tools/smallbatch.hip
//         -Ltempi_amd/lib -ltempi_hip -Wl,-rpath,'$ORIGIN/../../tempi_amd/lib'
#include <hip/hip_runtime.h>

#include "tempi_hip.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static double med(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 2000;
  char *obj = nullptr, *dpk = nullptr;
  void *hpk = nullptr, *hpk_dev = nullptr;
  if (hipMalloc(&obj, 1 << 20) || hipMalloc(&dpk, 1 << 20) || tempi_hip_host_alloc(&hpk, &hpk_dev, 1 << 20)) return 3;
  if (hipMemset(obj, 1, 1 << 20) || hipDeviceSynchronize()) return 3;
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking)) return 3;
  struct Shape {
    const char *name;
    tempi_hip_desc d;
  };
  std::vector<Shape> shapes(3);
  shapes[0].name = "1B";
  shapes[0].d.block = 1;
  shapes[1].name = "1KiB";
  shapes[1].d.block = 1024;
  shapes[2].name = "128x8B_st512";
  shapes[2].d.block = 8;
  shapes[2].d.ndims = 1;
  shapes[2].d.counts[0] = 128;
  shapes[2].d.strides[0] = 512;
  for (int pack = 1; pack >= 0; --pack) {
    for (int host = 0; host < 2; ++host) {
      for (const Shape &sh : shapes) {
        tempi_hip_batch_item it{};
        it.packed = host ? hpk_dev : dpk;
        it.first = obj;
        it.desc = sh.d;
        std::vector<double> t;
        for (int i = 0; i < reps + 50; ++i) {
          const uint32_t *flag = nullptr;
          uint32_t ticket = 0;
          const double t0 = now_us();
          const int e = pack ? tempi_hip_pack_batch_ticket(&it, 1, s, &flag, &ticket)
                             : tempi_hip_unpack_batch_ticket(&it, 1, s, &flag, &ticket);
          if (e) return 4;
          if (flag) {
            if (tempi_hip_ticket_wait(s, flag, ticket)) return 5;
          } else if (hipStreamSynchronize(s)) {
            return 5;
          }
          if (i >= 50) t.push_back(now_us() - t0);
        }
        std::printf("{\"bench\": \"smallbatch\", \"dir\": \"%s\", \"packed\": \"%s\", \"shape\": \"%s\", \"reps\": %d, "
                    "\"call_us\": %.2f}\n",
                    pack ? "pack" : "unpack", host ? "pinned_host" : "device", sh.name, reps, med(t));
        std::fflush(stdout);
      }
    }
  }
  return 0;
}
