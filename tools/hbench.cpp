// tools/hbench.cpp -- halo-region kernel microbenchmark (config 4 shapes).
//
// usage: hbench LIB.so REPS [LCR] [QUANTS]
// One rank's buffers of the 512^3 halo exchange (LCR^3 cells + radius 3, 8-byte
// quantities, pitch rounded to 512 B, /root/reference/bin/bench_halo_exchange.cpp:
// 727-733). For each class of region (x / y / z faces, edges, corners, all 26)
// it times, with HIP events over REPS back-to-back batched launches:
//   pack   interior(d) -> packed slab            (tempi_hip_pack_batch)
//   unpack packed slab  -> exterior(-d)          (tempi_hip_unpack_batch)
//   copy   interior(d)  -> exterior(-d) directly (tempi_hip_copy_batch)
// over QUANTS buffers, and prints one JSON line per class with the kernel time
// and the algorithmic GB/s (2 x payload per launch set), plus the host time of
// one tempi_hip_copy_batch call (planning + launch; copy_host_us).
// Then (HBENCH_CONCURRENT=1) the x faces against the y + z faces: one after
// the other on one stream, and side by side on two streams -- does the
// x faces' isolated-line pattern overlap with the streaming faces?
// HBENCH_SCHEDULE=1: all 26 regions' copies under several launch schedules
// (one call, by class, chunks of HBENCH_CHUNK (32) on 1 / 2 lanes, x faces
// apart) -- what batch composition costs the GPU.
#include "tempi_hip.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <dlfcn.h>
#include <string>
#include <vector>

#define SYM(name)                                                                                  \
  auto name = reinterpret_cast<decltype(&::name)>(dlsym(h, #name));                               \
  if (!name) {                                                                                     \
    std::fprintf(stderr, "missing %s\n", #name);                                                   \
    return 2;                                                                                      \
  }
#define CK(x)                                                                                      \
  do {                                                                                             \
    int e_ = (x);                                                                                  \
    if (e_) {                                                                                      \
      std::fprintf(stderr, "%s: error %d\n", #x, e_);                                              \
      return 3;                                                                                    \
    }                                                                                              \
  } while (0)

struct Region {
  int dx, dy, dz;
  tempi_hip_desc desc;
  long long srcOff, dstOff, bytes;
};

int main(int argc, char **argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s LIB REPS [LCR] [QUANTS]\n", argv[0]);
    return 1;
  }
  void *h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    std::fprintf(stderr, "dlopen: %s\n", dlerror());
    return 2;
  }
  SYM(tempi_hip_pack_batch) SYM(tempi_hip_unpack_batch) SYM(tempi_hip_copy_batch) SYM(tempi_hip_malloc)
  SYM(tempi_hip_stream_create) SYM(tempi_hip_event_create) SYM(tempi_hip_event_record)
  SYM(tempi_hip_event_synchronize) SYM(tempi_hip_event_elapsed_ms) SYM(tempi_hip_memset_async)
  SYM(tempi_hip_stream_synchronize)
  const int reps = std::atoi(argv[2]);
  const int l = argc > 3 ? std::atoi(argv[3]) : 512;
  const int nq = argc > 4 ? std::atoi(argv[4]) : 8;
  const int r = 3, q = 8;
  const long long width = (l + 2LL * r) * q, pitch = (width + 511) / 512 * 512;
  const long long ysize = l + 2 * r, zsize = l + 2 * r;
  const long long plane = pitch * ysize, bufBytes = plane * zsize;

  std::vector<Region> regions;
  for (int dz = -1; dz <= 1; ++dz)
    for (int dy = -1; dy <= 1; ++dy)
      for (int dx = -1; dx <= 1; ++dx) {
        if (!dx && !dy && !dz) continue;
        const int d[3] = {dx, dy, dz};
        long long pin[3], pex[3], e[3];
        for (int k = 0; k < 3; ++k) {
          pin[k] = d[k] == -1 ? r : d[k] == 1 ? l : r;
          // the exterior on the OPPOSITE side receives interior(d)
          pex[k] = -d[k] == -1 ? 0 : -d[k] == 1 ? l + r : r;
          e[k] = d[k] == 0 ? l : r;
        }
        Region R{dx, dy, dz, {}, 0, 0, 0};
        R.desc.block = e[0] * q;
        R.desc.ndims = 2;
        R.desc.counts[0] = e[2];
        R.desc.strides[0] = plane;
        R.desc.counts[1] = e[1];
        R.desc.strides[1] = pitch;
        R.srcOff = pin[2] * plane + pin[1] * pitch + pin[0] * q;
        R.dstOff = pex[2] * plane + pex[1] * pitch + pex[0] * q;
        R.bytes = e[0] * e[1] * e[2] * q;
        regions.push_back(R);
      }

  std::vector<char *> bufs(static_cast<size_t>(nq), nullptr);
  void *s, *e0, *e1;
  CK(tempi_hip_stream_create(&s));
  CK(tempi_hip_event_create(&e0, 1));
  CK(tempi_hip_event_create(&e1, 1));
  for (auto &b : bufs) {
    void *p;
    CK(tempi_hip_malloc(&p, size_t(bufBytes)));
    CK(tempi_hip_memset_async(p, 1, size_t(bufBytes), s));
    b = static_cast<char *>(p);
  }
  long long slabBytes = 0;
  for (const Region &R : regions) slabBytes += (R.bytes + 255) / 256 * 256;
  void *slab;
  CK(tempi_hip_malloc(&slab, size_t(slabBytes * nq)));
  CK(tempi_hip_stream_synchronize(s));


  struct Cls {
    const char *name;
    bool (*pick)(const Region &);
  };
  const Cls classes[] = {
      {"x_faces", [](const Region &R) { return R.dx != 0 && !R.dy && !R.dz; }},
      {"y_faces", [](const Region &R) { return !R.dx && R.dy != 0 && !R.dz; }},
      {"z_faces", [](const Region &R) { return !R.dx && !R.dy && R.dz != 0; }},
      {"edges", [](const Region &R) { return (R.dx != 0) + (R.dy != 0) + (R.dz != 0) == 2; }},
      {"corners", [](const Region &R) { return R.dx != 0 && R.dy != 0 && R.dz != 0; }},
      {"all26", [](const Region &) { return true; }},
  };

  const char *only = std::getenv("HBENCH_ONLY"); // one class (profiling runs)
  for (const Cls &c : classes) {
    if (only && std::strcmp(only, c.name) != 0) continue;
    std::vector<tempi_hip_batch_item> pk, up;
    std::vector<tempi_hip_copy_item> cp;
    long long payload = 0, off = 0;
    for (int qi = 0; qi < nq; ++qi)
      for (const Region &R : regions) {
        if (!c.pick(R)) continue;
        char *packed = static_cast<char *>(slab) + off;
        off += (R.bytes + 255) / 256 * 256;
        payload += R.bytes;
        tempi_hip_batch_item a{}, b{};
        tempi_hip_copy_item cc{};
        a.packed = b.packed = packed;
        a.first = bufs[size_t(qi)] + R.srcOff;
        b.first = bufs[size_t(qi)] + R.dstOff;
        a.desc = b.desc = cc.dst = cc.src = R.desc;
        cc.dst_first = b.first;
        cc.src_first = a.first;
        pk.push_back(a);
        up.push_back(b);
        cp.push_back(cc);
      }
    float ms[3];
    double hostUs = 0;
    for (int mode = 0; mode < 3; ++mode) {
      auto run = [&]() -> int {
        if (mode == 0) return tempi_hip_pack_batch(pk.data(), int(pk.size()), s);
        if (mode == 1) return tempi_hip_unpack_batch(up.data(), int(up.size()), s);
        return tempi_hip_copy_batch(cp.data(), int(cp.size()), s);
      };
      CK(run());
      CK(run());
      CK(tempi_hip_event_record(e0, s));
      const auto h0 = std::chrono::steady_clock::now();
      for (int i = 0; i < reps; ++i) CK(run());
      if (mode == 2)
        hostUs = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - h0).count() / reps;
      CK(tempi_hip_event_record(e1, s));
      CK(tempi_hip_event_synchronize(e1));
      CK(tempi_hip_event_elapsed_ms(&ms[mode], e0, e1));
      ms[mode] /= float(reps);
    }
    auto gbs = [&](float m) { return 2.0 * double(payload) / (double(m) * 1e-3) / 1e9; };
    std::printf("{\"lib\": \"%s\", \"class\": \"%s\", \"items\": %zu, \"payload\": %lld, \"pack_us\": %.1f, "
                "\"unpack_us\": %.1f, \"copy_us\": %.1f, \"pack_gbs\": %.1f, \"unpack_gbs\": %.1f, "
                "\"copy_gbs\": %.1f, \"copy_host_us\": %.2f}\n",
                argv[1], c.name, cp.size(), payload, ms[0] * 1e3, ms[1] * 1e3, ms[2] * 1e3, gbs(ms[0]), gbs(ms[1]),
                gbs(ms[2]), hostUs);
    std::fflush(stdout);
  }
  if (std::getenv("HBENCH_CONCURRENT")) {
    std::vector<tempi_hip_copy_item> xs, yz;
    for (int qi = 0; qi < nq; ++qi)
      for (const Region &R : regions) {
        const bool x = R.dx != 0 && !R.dy && !R.dz, y = !R.dx && R.dy != 0 && !R.dz, z = !R.dx && !R.dy && R.dz != 0;
        if (!x && !y && !z) continue;
        tempi_hip_copy_item cc{};
        cc.dst = cc.src = R.desc;
        cc.src_first = bufs[size_t(qi)] + R.srcOff;
        cc.dst_first = bufs[size_t(qi)] + R.dstOff;
        (x ? xs : yz).push_back(cc);
      }
    void *s2, *f0, *f1;
    CK(tempi_hip_stream_create(&s2));
    CK(tempi_hip_event_create(&f0, 0));
    CK(tempi_hip_event_create(&f1, 0));
    SYM(tempi_hip_stream_wait_event)
    float ms[2];
    for (int mode = 0; mode < 2; ++mode) {
      auto run = [&]() -> int {
        if (mode == 0) {
          if (int e = tempi_hip_copy_batch(xs.data(), int(xs.size()), s)) return e;
          return tempi_hip_copy_batch(yz.data(), int(yz.size()), s);
        }
        // fork s2 off s, run the two classes side by side, join back into s
        if (int e = tempi_hip_event_record(f0, s)) return e;
        if (int e = tempi_hip_stream_wait_event(s2, f0)) return e;
        if (int e = tempi_hip_copy_batch(xs.data(), int(xs.size()), s)) return e;
        if (int e = tempi_hip_copy_batch(yz.data(), int(yz.size()), s2)) return e;
        if (int e = tempi_hip_event_record(f1, s2)) return e;
        return tempi_hip_stream_wait_event(s, f1);
      };
      CK(run());
      CK(run());
      CK(tempi_hip_event_record(e0, s));
      for (int i = 0; i < reps; ++i) CK(run());
      CK(tempi_hip_event_record(e1, s));
      CK(tempi_hip_event_synchronize(e1));
      CK(tempi_hip_event_elapsed_ms(&ms[mode], e0, e1));
      ms[mode] /= float(reps);
    }
    std::printf("{\"lib\": \"%s\", \"class\": \"x_vs_yz\", \"x_items\": %zu, \"yz_items\": %zu, "
                "\"sequential_us\": %.1f, \"concurrent_us\": %.1f}\n",
                argv[1], xs.size(), yz.size(), ms[0] * 1e3, ms[1] * 1e3);
  }
  if (std::getenv("HBENCH_SCHEDULE")) {
    // the 208 copies of one substep (all26, app order) under different
    // launch schedules: how batch composition and chunking move the GPU time
    std::vector<tempi_hip_copy_item> all;
    std::vector<int> cls; // 0 x face, 1 y / z face, 2 edge, 3 corner
    for (int qi = 0; qi < nq; ++qi)
      for (const Region &R : regions) {
        tempi_hip_copy_item cc{};
        cc.dst = cc.src = R.desc;
        cc.src_first = bufs[size_t(qi)] + R.srcOff;
        cc.dst_first = bufs[size_t(qi)] + R.dstOff;
        all.push_back(cc);
        const int nz = (R.dx != 0) + (R.dy != 0) + (R.dz != 0);
        cls.push_back(nz == 1 ? (R.dx ? 0 : 1) : nz == 2 ? 2 : 3);
      }
    const int chunk = std::getenv("HBENCH_CHUNK") ? std::atoi(std::getenv("HBENCH_CHUNK")) : 32;
    std::vector<void *> lanes{s};
    for (int i = 0; i < 2; ++i) {
      void *t;
      CK(tempi_hip_stream_create(&t));
      lanes.push_back(t);
    }
    void *fork, *join[3];
    CK(tempi_hip_event_create(&fork, 0));
    for (auto &j : join) CK(tempi_hip_event_create(&j, 0));
    SYM(tempi_hip_stream_wait_event)
    typedef std::vector<std::vector<tempi_hip_copy_item>> Chunks;
    auto chunked = [&](const std::vector<tempi_hip_copy_item> &v, int n) {
      Chunks c;
      for (size_t i = 0; i < v.size(); i += size_t(n))
        c.emplace_back(v.begin() + long(i), v.begin() + long(std::min(v.size(), i + size_t(n))));
      return c;
    };
    std::vector<tempi_hip_copy_item> byClass, xs, rest;
    for (int k = 0; k < 4; ++k)
      for (size_t i = 0; i < all.size(); ++i)
        if (cls[i] == k) byClass.push_back(all[i]);
    for (size_t i = 0; i < all.size(); ++i) (cls[i] == 0 ? xs : rest).push_back(all[i]);
    struct Sched {
      const char *name;
      Chunks chunks;
      int nl;
    };
    std::vector<Sched> scheds = {
        {"one_call_app_order", {all}, 1},
        {"one_call_by_class", {byClass}, 1},
        {"chunks_app_order_1lane", chunked(all, chunk), 1},
        {"chunks_app_order_2lanes", chunked(all, chunk), 2},
        {"chunks_by_class_2lanes", chunked(byClass, chunk), 2},
        {"x_one_call_then_rest_chunks_1lane", {}, 1},
        {"x_lane_rest_lane", {}, 2},
        {"rest_chunks_2lanes_then_x_joined", {}, 2},
    };
    scheds[5].chunks.push_back(xs);
    for (auto &c : chunked(rest, chunk)) scheds[5].chunks.push_back(c);
    scheds[6].chunks = scheds[5].chunks; // x on lane 0, every rest chunk on lane 1
    scheds[7].chunks = chunked(rest, chunk);
    scheds[7].chunks.push_back(xs); // (issued on s after both lanes joined)
    for (Sched &S : scheds) {
      const bool xlane = std::strcmp(S.name, "x_lane_rest_lane") == 0;
      auto run = [&]() -> int {
        if (S.nl > 1) {
          if (int e = tempi_hip_event_record(fork, s)) return e;
          for (int l = 1; l < S.nl; ++l)
            if (int e = tempi_hip_stream_wait_event(lanes[size_t(l)], fork)) return e;
        }
        const bool xlast = std::strcmp(S.name, "rest_chunks_2lanes_then_x_joined") == 0;
        const size_t nchunks = S.chunks.size() - (xlast ? 1 : 0);
        for (size_t i = 0; i < nchunks; ++i) {
          const size_t lane = xlane ? (i == 0 ? 0 : 1) : i % size_t(S.nl);
          if (int e = tempi_hip_copy_batch(S.chunks[i].data(), int(S.chunks[i].size()), lanes[lane])) return e;
        }
        for (int l = 1; l < S.nl; ++l) {
          if (int e = tempi_hip_event_record(join[l], lanes[size_t(l)])) return e;
          if (int e = tempi_hip_stream_wait_event(s, join[l])) return e;
        }
        if (xlast) return tempi_hip_copy_batch(S.chunks.back().data(), int(S.chunks.back().size()), s);
        return 0;
      };
      CK(run());
      CK(run());
      CK(tempi_hip_event_record(e0, s));
      for (int i = 0; i < reps; ++i) CK(run());
      CK(tempi_hip_event_record(e1, s));
      CK(tempi_hip_event_synchronize(e1));
      float ms = 0;
      CK(tempi_hip_event_elapsed_ms(&ms, e0, e1));
      std::printf("{\"lib\": \"%s\", \"schedule\": \"%s\", \"chunk\": %d, \"launch_calls\": %zu, \"copy_us\": %.1f}\n",
                  argv[1], S.name, chunk, S.chunks.size(), double(ms) * 1e3 / reps);
      std::fflush(stdout);
    }
  }
  return 0;
}
