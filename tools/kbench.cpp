// tools/kbench.cpp -- kernel microbenchmark for libtempi_hip.so variants.
//
// usage: kbench LIB.so REPS SHAPE...   where SHAPE = block:count1:stride1[:count2:stride2]
//   (dims outermost first after the block, e.g. 512:2097152:1024)
// Also times hipMemcpyAsync D2D of the same payload (achievable-copy peak), and
// the strided -> strided copy kernel between two objects of this shape, with
// plain loads and with the source flagged TEMPI_HIP_ITEM_REMOTE (the
// system-scope loads a reader on another GPU uses; here on local memory).
// Prints one JSON line per shape: kernel ms (HIP events, back-to-back
// launches) and algorithmic GB/s (2 x payload per pack, unpack or copy).
// KBENCH_OFFSET=B starts both strided objects B bytes into their allocations
// (the halo's regions start 24 B into 512-B-aligned rows), KBENCH_POFF=B the
// packed buffer.
#include "tempi_hip.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <dlfcn.h>
#include <string>
#include <vector>

#define SYM(name) auto name = reinterpret_cast<decltype(&::name)>(dlsym(h, #name)); \
  if (!name) { std::fprintf(stderr, "missing %s\n", #name); return 2; }
#define CK(x) do { int e_ = (x); if (e_) { std::fprintf(stderr, "%s: error %d\n", #x, e_); return 3; } } while (0)

int main(int argc, char **argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s LIB REPS SHAPE...\n", argv[0]);
    return 1;
  }
  void *h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    std::fprintf(stderr, "dlopen: %s\n", dlerror());
    return 2;
  }
  SYM(tempi_hip_pack) SYM(tempi_hip_unpack) SYM(tempi_hip_malloc) SYM(tempi_hip_free)
  SYM(tempi_hip_stream_create) SYM(tempi_hip_event_create) SYM(tempi_hip_event_record)
  SYM(tempi_hip_event_synchronize) SYM(tempi_hip_event_elapsed_ms) SYM(tempi_hip_memcpy_async)
  SYM(tempi_hip_memset_async) SYM(tempi_hip_stream_synchronize) SYM(tempi_hip_desc_bytes)
  SYM(tempi_hip_copy_batch)
  const int reps = std::atoi(argv[2]);
  void *s, *e0, *e1;
  CK(tempi_hip_stream_create(&s));
  CK(tempi_hip_event_create(&e0, 1));
  CK(tempi_hip_event_create(&e1, 1));
  for (int a = 3; a < argc; ++a) {
    std::vector<long long> v;
    std::string sh = argv[a];
    size_t p = 0;
    while (p <= sh.size()) {
      size_t q = sh.find(':', p);
      if (q == std::string::npos) q = sh.size();
      v.push_back(std::atoll(sh.substr(p, q - p).c_str()));
      p = q + 1;
    }
    tempi_hip_desc d{};
    d.block = v[0];
    d.ndims = int((v.size() - 1) / 2);
    long long extent = d.block;
    for (int k = 0; k < d.ndims; ++k) {
      d.counts[k] = v[1 + 2 * k];
      d.strides[k] = v[2 + 2 * k];
    }
    // extent: outermost count * stride (enough for positive strides)
    extent = d.ndims ? d.counts[0] * d.strides[0] : d.block;
    const long long payload = tempi_hip_desc_bytes(&d);
    void *strided0, *packed0, *other0 = nullptr;
    const long long off = std::getenv("KBENCH_OFFSET") ? std::atoll(std::getenv("KBENCH_OFFSET")) : 0;
    const long long poff = std::getenv("KBENCH_POFF") ? std::atoll(std::getenv("KBENCH_POFF")) : 0;
    CK(tempi_hip_malloc(&strided0, size_t(extent + off)));
    CK(tempi_hip_malloc(&packed0, size_t(payload + poff)));
    CK(tempi_hip_memset_async(strided0, 1, size_t(extent + off), s));
    const bool copies = std::getenv("KBENCH_NO_COPY") == nullptr;
    if (copies) CK(tempi_hip_malloc(&other0, size_t(extent + off)));
    char *strided = static_cast<char *>(strided0) + off, *packed = static_cast<char *>(packed0) + poff;
    char *other = other0 ? static_cast<char *>(other0) + off : nullptr;
    tempi_hip_copy_item ci{};
    ci.dst_first = other;
    ci.src_first = strided;
    ci.dst = d;
    ci.src = d;
    float ms[5] = {0, 0, 0, 0, 0};
    for (int mode = 0; mode < (copies ? 5 : 3); ++mode) {
      ci.flags = mode == 4 ? TEMPI_HIP_ITEM_REMOTE : 0;
      auto run = [&]() -> int {
        if (mode == 0) return tempi_hip_pack(packed, strided, &d, s);
        if (mode == 1) return tempi_hip_unpack(strided, packed, &d, s);
        if (mode == 2) return tempi_hip_memcpy_async(packed, strided, size_t(payload), s);
        return tempi_hip_copy_batch(&ci, 1, s);
      };
      for (int w = 0; w < 2; ++w) CK(run()); // warm-up
      CK(tempi_hip_event_record(e0, s));
      for (int r = 0; r < reps; ++r) CK(run());
      CK(tempi_hip_event_record(e1, s));
      CK(tempi_hip_event_synchronize(e1));
      CK(tempi_hip_event_elapsed_ms(&ms[mode], e0, e1));
      ms[mode] /= float(reps);
    }
    auto gbs = [&](float m) { return 2.0 * double(payload) / (double(m) * 1e-3) / 1e9; };
    std::printf("{\"lib\": \"%s\", \"shape\": \"%s\", \"offset\": %lld, \"poff\": %lld, \"payload\": %lld, \"pack_ms\": %.4f, \"unpack_ms\": %.4f, "
                "\"memcpy_ms\": %.4f, \"pack_gbs\": %.1f, \"unpack_gbs\": %.1f, \"memcpy_gbs\": %.1f, "
                "\"copy_gbs\": %.1f, \"copy_remote_gbs\": %.1f}\n",
                argv[1], argv[a], off, poff, payload, ms[0], ms[1], ms[2], gbs(ms[0]), gbs(ms[1]), gbs(ms[2]),
                copies ? gbs(ms[3]) : 0.0, copies ? gbs(ms[4]) : 0.0);
    std::fflush(stdout);
    tempi_hip_free(strided0);
    tempi_hip_free(packed0);
    if (other0) tempi_hip_free(other0);
  }
  return 0;
}
