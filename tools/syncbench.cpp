// tools/syncbench.cpp -- where a synchronous small MPI_Pack's time goes
// (VERDICT r02 next 5), at the C ABI of libtempi_hip.so (no MPI, no Python):
// per call, median of REPS, for BASELINE config 1 (vector(1024, 512, 1024),
// 512 KiB packed) and a 1 KiB object (vector(2, 512, 1024)):
//   ptrinfo      tempi_hip_pointer_info on a device pointer (the interposer
//                classifies both sides of every call)
//   launch       tempi_hip_pack alone (the host cost of the launch)
//   sync         tempi_hip_pack + hipStreamSynchronize
//   ticket_fold  tempi_hip_pack_ticket + tempi_hip_ticket_wait (the kernel's
//                last workgroup stores the ticket; TEMPI_FOLD_MAX_BLOCKS)
//   ticket_kern  tempi_hip_pack + tempi_hip_stream_ticket (a ticket kernel
//                queued behind) + wait
// usage: syncbench LIB.so [REPS]  -> one JSON line per shape
//   g++ -O2 -std=c++17 -Iinclude -o tools/_variants/syncbench tools/syncbench.cpp -ldl
#include "tempi_hip.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <dlfcn.h>
#include <vector>

#define SYM(name) auto name = reinterpret_cast<decltype(&::name)>(dlsym(h, #name)); \
  if (!name) { std::fprintf(stderr, "missing %s\n", #name); return 2; }
#define CK(x) do { int e_ = (x); if (e_) { std::fprintf(stderr, "%s: error %d\n", #x, e_); return 3; } } while (0)

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char **argv) {
  if (argc < 2) return 1;
  void *h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    std::fprintf(stderr, "dlopen: %s\n", dlerror());
    return 2;
  }
  const int reps = argc > 2 ? std::atoi(argv[2]) : 2000;
  SYM(tempi_hip_pack) SYM(tempi_hip_pack_ticket) SYM(tempi_hip_malloc) SYM(tempi_hip_stream_create)
  SYM(tempi_hip_stream_synchronize) SYM(tempi_hip_stream_ticket) SYM(tempi_hip_ticket_wait)
  SYM(tempi_hip_pointer_info) SYM(tempi_hip_memset_async)
  void *s = nullptr;
  CK(tempi_hip_stream_create(&s));
  void *src = nullptr, *dst = nullptr;
  CK(tempi_hip_malloc(&src, 2 << 20));
  CK(tempi_hip_malloc(&dst, 1 << 20));
  CK(tempi_hip_memset_async(src, 1, 2 << 20, s));
  CK(tempi_hip_stream_synchronize(s));
  for (int n : {2, 8, 32, 64, 128, 256, 512, 1024}) { // 1, 2, 8, 16, 32, 64, 128, 256 workgroups of the packer
    tempi_hip_desc d{};
    d.block = 512;
    d.ndims = 1;
    d.counts[0] = n;
    d.strides[0] = 1024;
    std::vector<double> pi, la, sy, tf, tk;
    for (int r = 0; r < reps + 20; ++r) {
      const bool keep = r >= 20;
      tempi_hip_ptrinfo info;
      double t0 = now_us();
      tempi_hip_pointer_info(src, &info);
      tempi_hip_pointer_info(dst, &info);
      double t1 = now_us();
      CK(tempi_hip_pack(dst, src, &d, s));
      double t2 = now_us();
      CK(tempi_hip_stream_synchronize(s));
      double t3 = now_us();
      CK(tempi_hip_pack(dst, src, &d, s));
      CK(tempi_hip_stream_synchronize(s));
      double t4 = now_us();
      const uint32_t *flag = nullptr;
      uint32_t ticket = 0;
      CK(tempi_hip_pack_ticket(dst, src, &d, s, &flag, &ticket));
      CK(tempi_hip_ticket_wait(s, flag, ticket));
      double t5 = now_us();
      CK(tempi_hip_pack(dst, src, &d, s));
      CK(tempi_hip_stream_ticket(s, &flag, &ticket));
      CK(tempi_hip_ticket_wait(s, flag, ticket));
      double t6 = now_us();
      if (keep) {
        pi.push_back((t1 - t0) / 2);
        la.push_back(t2 - t1);
        sy.push_back(t4 - t3);
        tf.push_back(t5 - t4);
        tk.push_back(t6 - t5);
      }
      (void)t3;
    }
    std::printf("{\"shape\": \"vector(%d, 512, 1024)\", \"packed\": %d, \"reps\": %d, \"ptrinfo_us\": %.2f, "
                "\"launch_us\": %.2f, \"sync_us\": %.2f, \"ticket_fold_us\": %.2f, \"ticket_kern_us\": %.2f, "
                "\"fold_max_blocks\": \"%s\", \"dev_kernarg\": \"%s\"}\n",
                n, n * 512, reps, median(pi), median(la), median(sy), median(tf), median(tk),
                std::getenv("TEMPI_FOLD_MAX_BLOCKS") ? std::getenv("TEMPI_FOLD_MAX_BLOCKS") : "default",
                std::getenv("HIP_FORCE_DEV_KERNARG") ? std::getenv("HIP_FORCE_DEV_KERNARG") : "unset");
    std::fflush(stdout);
  }
  return 0;
}
