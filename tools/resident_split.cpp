// tools/resident_split.cpp -- where a resident-packer call's time goes
// (DESIGN §6.4): config 1's object (vector(1024, 512, 1024), 512 KiB) packed
// through tempi_hip_pack_resident with TEMPI_RESIDENT_STAMPS=1; per call the
// host's time around the call and the GPU clock at five points of it
// (tempi_hip_resident_stamps): leader saw the request -> worker 0 saw the
// hand-off -> its acquire done -> its share done -> the completion stored.
// The host legs (post -> leader, completion -> host) are the call minus the
// GPU span. Then the same calls back to back without reading the stamps.
// Medians of REPS. The library is dlopen'ed (A/B builds: tools/build_ab.sh).
// usage: resident_split [LIB] [REPS] [ROWS BLOCK STRIDE]
//   hipcc --offload-arch=gfx950 -O2 -Iinclude -o tools/bin/resident_split tools/resident_split.cpp -ldl
#include <hip/hip_runtime.h>

#include "tempi_hip.h"

#include <dlfcn.h>

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
  return v.empty() ? -1 : v[v.size() / 2];
}

int main(int argc, char **argv) {
  setenv("TEMPI_RESIDENT_STAMPS", "1", 1);
  const char *lib = argc > 1 ? argv[1] : "tempi_amd/lib/libtempi_hip.so";
  const int reps = argc > 2 ? std::atoi(argv[2]) : 1000;
  const int rows = argc > 5 ? std::atoi(argv[3]) : 1024, block = argc > 5 ? std::atoi(argv[4]) : 512,
            stride = argc > 5 ? std::atoi(argv[5]) : 1024;
  void *h = dlopen(lib, RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    std::fprintf(stderr, "%s\n", dlerror());
    return 2;
  }
#define SYM(n) auto n = reinterpret_cast<decltype(&::n)>(dlsym(h, #n))
  SYM(tempi_hip_pack_resident);
  SYM(tempi_hip_resident_stamps);
  SYM(tempi_hip_resident_stats);
  SYM(tempi_hip_resident_stop);
  SYM(tempi_hip_pack_ticket);
  SYM(tempi_hip_ticket_wait);
  if (!tempi_hip_pack_ticket || !tempi_hip_ticket_wait || !tempi_hip_pack_resident || !tempi_hip_resident_stamps || !tempi_hip_resident_stats || !tempi_hip_resident_stop)
    return 2;
  char *src, *dst;
  if (hipMalloc(&src, size_t(rows) * stride) || hipMalloc(&dst, size_t(rows) * block)) return 3;
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking)) return 3;
  tempi_hip_desc d{};
  d.block = block;
  d.ndims = 1;
  d.counts[0] = rows;
  d.strides[0] = stride;
  std::vector<double> call, gpu, handoff, acquire, body, fold, host, b2b;
  int unserved = 0;
  for (int i = 0; i < reps + 20; ++i) {
    int served = 0;
    const double t0 = now_us();
    if (tempi_hip_pack_resident(dst, src, &d, s, &served)) return 4;
    const double t1 = now_us();
    uint64_t st[5];
    if (tempi_hip_resident_stamps(st)) return 5;
    unserved += !served;
    if (i < 20 || !served) continue;
    auto us = [&](int a, int b) { return double(int64_t(st[b] - st[a])) / 100.0; };
    call.push_back(t1 - t0);
    gpu.push_back(us(0, 4));
    handoff.push_back(us(0, 1));
    acquire.push_back(us(1, 2));
    body.push_back(us(2, 3));
    fold.push_back(us(3, 4));
    host.push_back((t1 - t0) - us(0, 4));
  }
  for (int i = 0; i < reps + 20; ++i) {
    int served = 0;
    const double t0 = now_us();
    if (tempi_hip_pack_resident(dst, src, &d, s, &served)) return 4;
    if (i >= 20) b2b.push_back(now_us() - t0);
    unserved += !served;
  }
  // the launched path on the same object: launch + the folded ticket's wait
  std::vector<double> launched;
  for (int i = 0; i < reps + 20; ++i) {
    const uint32_t *flag = nullptr;
    uint32_t ticket = 0;
    const double t0 = now_us();
    if (tempi_hip_pack_ticket(dst, src, &d, s, &flag, &ticket)) return 4;
    if (flag && tempi_hip_ticket_wait(s, flag, ticket)) return 4;
    if (!flag && hipStreamSynchronize(s)) return 4;
    if (i >= 20) launched.push_back(now_us() - t0);
  }
  uint64_t sv, la, rp;
  tempi_hip_resident_stats(&sv, &la, &rp);
  tempi_hip_resident_stop();
  std::printf("{\"tool\": \"resident_split\", \"rows\": %d, \"block\": %d, \"stride\": %d, \"reps\": %d, "
              "\"unserved\": %d, \"call_us\": %.2f, \"gpu_leader_to_done_us\": %.2f, \"handoff_us\": %.2f, "
              "\"acquire_us\": %.2f, \"worker0_share_us\": %.2f, \"worker0_to_done_us\": %.2f, "
              "\"host_legs_us\": %.2f, \"back_to_back_call_us\": %.2f, \"launched_call_us\": %.2f, \"served\": %lu, "
              "\"launches\": %lu, "
              "\"reposts\": %lu}\n",
              rows, block, stride, reps, unserved, med(call), med(gpu), med(handoff), med(acquire), med(body),
              med(fold), med(host), med(b2b), med(launched), (unsigned long)sv, (unsigned long)la, (unsigned long)rp);
  return unserved ? 6 : 0;
}
