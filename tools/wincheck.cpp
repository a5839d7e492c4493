// tools/wincheck.cpp -- byte-exact check of a libtempi_hip.so variant's
// tempi_hip_pack against a host gather, over narrow-row shapes at every
// strided / packed base offset mod 16 (A/B builds: tools/build_ab.sh).
// usage: wincheck LIB
//   hipcc --offload-arch=gfx950 -O2 -Iinclude -o tools/bin/wincheck tools/wincheck.cpp -ldl
#include <hip/hip_runtime.h>

#include "tempi_hip.h"

#include <dlfcn.h>

#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

int main(int argc, char **argv) {
  if (argc < 2) return 1;
  void *h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    std::fprintf(stderr, "dlopen: %s\n", dlerror());
    return 2;
  }
  auto pack = reinterpret_cast<decltype(&tempi_hip_pack)>(dlsym(h, "tempi_hip_pack"));
  if (!pack) return 2;
  // block, then (count, stride) pairs outermost first
  struct Shape {
    long long b;
    std::vector<long long> cs;
  };
  const std::vector<Shape> shapes = {
      {2, {1 << 20, 18}}, {3, {700000, 19}}, {4, {600000, 20}}, {1, {2000000, 17}}, {8, {300000, 24}},
      {2, {37, 30000 * 18 + 64, 30000, 18}}, {4, {5, 123457 * 20 + 8, 123457, 20}}, {16, {100000, 79}},
      {2, {3000, 11}}, {5, {100001, 33}}};
  std::mt19937_64 rng(7);
  int bad = 0, runs = 0;
  for (const Shape &sh : shapes) {
    tempi_hip_desc d{};
    d.block = sh.b;
    d.ndims = int(sh.cs.size() / 2);
    long long extent = sh.b, payload = sh.b;
    for (int k = 0; k < d.ndims; ++k) {
      d.counts[k] = sh.cs[2 * k];
      d.strides[k] = sh.cs[2 * k + 1];
      payload *= d.counts[k];
    }
    for (int k = 0; k < d.ndims; ++k) extent += (d.counts[k] - 1) * d.strides[k];
    std::vector<unsigned char> src(size_t(extent) + 16);
    for (auto &c : src) c = static_cast<unsigned char>(rng());
    char *ds = nullptr, *dp = nullptr;
    if (hipMalloc(&ds, src.size()) || hipMalloc(&dp, size_t(payload) + 16)) return 3;
    if (hipMemcpy(ds, src.data(), src.size(), hipMemcpyHostToDevice)) return 3;
    std::vector<unsigned char> out(static_cast<size_t>(payload)), exp(static_cast<size_t>(payload));
    for (int so : {0, 1, 2, 3, 7, 8, 12, 15}) {
      // host gather in type-map order from src + so
      size_t q = 0;
      std::vector<long long> idx(size_t(d.ndims), 0);
      for (;;) {
        long long off = so;
        for (int k = 0; k < d.ndims; ++k) off += idx[size_t(k)] * d.strides[k];
        std::memcpy(&exp[q], &src[size_t(off)], size_t(sh.b));
        q += size_t(sh.b);
        int k = d.ndims - 1;
        while (k >= 0 && ++idx[size_t(k)] == d.counts[k]) idx[size_t(k--)] = 0;
        if (k < 0) break;
      }
      for (int po : {0, 4, 9}) {
        if (hipMemset(dp, 0, size_t(payload) + 16)) return 3;
        if (pack(dp + po, ds + so, &d, nullptr)) return 4;
        if (hipDeviceSynchronize()) return 5;
        if (hipMemcpy(out.data(), dp + po, size_t(payload), hipMemcpyDeviceToHost)) return 3;
        ++runs;
        if (std::memcmp(out.data(), exp.data(), size_t(payload)) != 0) {
          size_t i = 0;
          while (out[i] == exp[i]) ++i;
          std::printf("MISMATCH block %lld dims %d strided+%d packed+%d: first at byte %zu of %lld\n", sh.b, d.ndims, so,
                      po, i, payload);
          ++bad;
        }
      }
    }
    (void)hipFree(ds);
    (void)hipFree(dp);
  }
  std::printf("{\"tool\": \"wincheck\", \"lib\": \"%s\", \"runs\": %d, \"mismatches\": %d}\n", argv[1], runs, bad);
  return bad ? 6 : 0;
}
