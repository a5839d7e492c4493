// tempi_amd/csrc/core/perf_model.cpp -- see perf_model.hpp
#include "perf_model.hpp"

#include "env.hpp"
#include "log.hpp"

#include <algorithm>
#include <cctype>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <dlfcn.h>
#include <fstream>
#include <limits>
#include <map>
#include <memory>
#include <sstream>
#include <sys/stat.h>

namespace tempi {

SystemPerformance systemPerformance;
bool systemPerformanceLoaded = false;
std::string systemPerformanceSource;
bool systemPerformanceNode = false;

bool SystemPerformance::empty() const {
  return intraNodeCpuCpuPingpong.empty() && intraNodeGpuGpuPingpong.empty() && d2h.empty() && packDevice.empty();
}

namespace {
int log2_floor(int64_t x) {
  int r = -1;
  while (x) {
    x >>= 1;
    ++r;
  }
  return r;
}
int log2_ceil(int64_t x) {
  const int f = log2_floor(x);
  return (int64_t(1) << f) == x ? f : f + 1;
}
} // namespace

Opt interp_time_opt(const std::vector<IidTime> &a, int64_t bytes) {
  if (a.empty() || bytes <= 0) return Opt::none();
  const int lb = log2_floor(bytes), ub = log2_ceil(bytes);
  if (size_t(ub) >= a.size()) // beyond the table: scale the largest time
    return Opt::of(a.back().time * double(bytes) / double(int64_t(1) << (a.size() - 1)));
  if (lb == ub) return Opt::of(a[size_t(lb)].time);
  const float num = float(bytes - (int64_t(1) << lb));
  const float den = float((int64_t(1) << ub) - (int64_t(1) << lb));
  const float sf = num / den;
  return Opt::of(a[size_t(lb)].time * (1 - sf) + a[size_t(ub)].time * sf);
}

double interp_time(const std::vector<IidTime> &a, int64_t bytes) {
  const Opt o = interp_time_opt(a, bytes);
  return o.ok ? o.v : std::numeric_limits<double>::infinity();
}

Opt interp_2d_opt(const std::vector<std::vector<IidTime>> &a, int64_t bytes, int64_t x) {
  if (a.empty() || bytes <= 0 || x <= 0) return Opt::none();
  if (x > 512) x = 512;
  // rows: 2^(2i+6) bytes; columns: block 2^j
  // below the first row (64 B): use the first row
  const int yi1 = bytes < 64 ? 0 : (log2_floor(bytes) - 6) / 2;
  const int64_t y1 = int64_t(1) << (yi1 * 2 + 6);
  const int yi2 = (y1 == bytes || bytes < 64) ? yi1 : yi1 + 1;
  const int64_t y2 = int64_t(1) << (yi2 * 2 + 6);
  // the row whose width bounds the columns (never past the table: F11)
  const size_t clampRow = std::min<size_t>(size_t(yi2), a.size() - 1);
  int xi1 = log2_floor(x);
  int xi2 = log2_ceil(x);
  if (size_t(xi2) >= a[clampRow].size()) xi2 = int(a[clampRow].size()) - 1;
  xi1 = std::min(xi1, xi2);
  const int64_t x1 = int64_t(1) << log2_floor(x), x2 = int64_t(1) << log2_ceil(x);
  const float sfx = (xi2 == xi1) ? 0.f : float(x - x1) / float(x2 - x1);
  const float sfy = (yi2 == yi1) ? 0.f : float(bytes - y1) / float(y2 - y1);
  if (size_t(yi2) >= a.size()) { // message beyond the table: scale the last row
    const auto &r = a.back();
    const float base = (1 - sfx) * float(r[size_t(xi1)].time) + sfx * float(r[size_t(xi2)].time);
    const float ymax = float(int64_t(1) << ((a.size() - 1) * 2 + 6));
    return Opt::of(double(base / ymax * float(bytes)));
  }
  const auto &r1 = a[size_t(yi1)], &r2 = a[size_t(yi2)];
  const float fy1 = (1 - sfx) * float(r1[size_t(xi1)].time) + sfx * float(r1[size_t(xi2)].time);
  const float fy2 = (1 - sfx) * float(r2[size_t(xi1)].time) + sfx * float(r2[size_t(xi2)].time);
  return Opt::of(double((1 - sfy) * fy1 + sfy * fy2));
}

double interp_2d(const std::vector<std::vector<IidTime>> &a, int64_t bytes, int64_t x) {
  const Opt o = interp_2d_opt(a, bytes, x);
  return o.ok ? o.v : std::numeric_limits<double>::infinity();
}

static Opt sum(std::initializer_list<Opt> parts) {
  double s = 0;
  for (const Opt &p : parts) {
    if (!p.ok) return Opt::none();
    s += p.v;
  }
  return Opt::of(s);
}

// /root/reference/src/internal/measure_system.cpp:100-116
Opt model_oneshot(const SystemPerformance &sp, bool colocated, int64_t bytes, int64_t bl) {
  return sum({interp_2d_opt(sp.packHost, bytes, bl),
              interp_time_opt(colocated ? sp.intraNodeCpuCpuPingpong : sp.interNodeCpuCpuPingpong, bytes),
              interp_2d_opt(sp.unpackHost, bytes, bl)});
}

// /root/reference/src/internal/measure_system.cpp:118-132
// viaTempi: the GPU-GPU ping-pong curve was measured through TEMPI's own IPC
// transport (apps/measure_system.cpp: no GPU-aware library underneath), so it
// already contains a contiguous gather and scatter; those (the 512-byte-block
// column of the tables, i.e. contiguous at stride 512) are taken out before
// the type's own pack and unpack are added, or the model would count the
// kernels twice and under-rate the IPC path
Opt model_device(const SystemPerformance &sp, bool colocated, int64_t bytes, int64_t bl, bool viaTempi) {
  const Opt pp = interp_time_opt(colocated ? sp.intraNodeGpuGpuPingpong : sp.interNodeGpuGpuPingpong, bytes);
  Opt transfer = pp;
  if (viaTempi && pp.ok) {
    const Opt own = sum({interp_2d_opt(sp.packDevice, bytes, 512), interp_2d_opt(sp.unpackDevice, bytes, 512)});
    if (own.ok) transfer = Opt::of(std::max(pp.v - own.v, 0.05 * pp.v));
  }
  return sum({interp_2d_opt(sp.packDevice, bytes, bl), transfer, interp_2d_opt(sp.unpackDevice, bytes, bl)});
}

// /root/reference/src/internal/sender.cpp:239-249
Opt model_staged(const SystemPerformance &sp, bool colocated, int64_t bytes, int64_t bl) {
  return sum({interp_2d_opt(sp.packDevice, bytes, bl), interp_time_opt(sp.d2h, bytes),
              interp_time_opt(colocated ? sp.intraNodeCpuCpuPingpong : sp.interNodeCpuCpuPingpong, bytes),
              interp_time_opt(sp.h2d, bytes), interp_2d_opt(sp.unpackDevice, bytes, bl)});
}

// The IPC / ONESHOT crossover of NON-blocking sends, priced per batch
// (the reference prices each Isend by the model,
// /root/reference/src/internal/async_operation.cpp:334-389). The curves are
// synchronous calls, but a burst of MPI_Isend / MPI_Irecv shares one gather
// launch and one scatter launch and overlaps its library messages, so a
// message adds only the MARGINAL cost of its bytes to each stage: the stage's
// time at its size minus its time at the smallest measured size (launch,
// completion and latency, paid once per batch). Both methods send one
// library message per message (IPC: a 128-byte descriptor; ONESHOT: the
// payload), so the library's per-message cost cancels and ONESHOT keeps the
// marginal cost of moving its payload through the library:
//   IPC(b)     = m(packDevice) + m(transfer over xGMI) + m(unpackDevice)
//   ONESHOT(b) = m(packHost) + m(intra-node CPU ping-pong) + m(unpackHost)
// where the transfer is the GPU-GPU ping-pong less the contiguous gather and
// scatter it contains (model_device's viaTempi correction). The threshold is
// the smallest power of two from which IPC stays cheaper up to 4 MiB; none
// (INT64_MAX) when ONESHOT is cheaper at 4 MiB, -1 when a curve is missing.
namespace {
double marginal2(const std::vector<std::vector<IidTime>> &t, int64_t b, int64_t bl) {
  const Opt x = interp_2d_opt(t, b, bl), z = interp_2d_opt(t, 64, bl);
  return x.ok && z.ok ? std::max(0.0, x.v - z.v) : -1;
}
double marginal1(const std::vector<IidTime> &c, int64_t b) {
  const Opt x = interp_time_opt(c, b), z = interp_time_opt(c, 1);
  return x.ok && z.ok ? std::max(0.0, x.v - z.v) : -1;
}
} // namespace

int64_t batch_ipc_threshold(const SystemPerformance &sp, int64_t bl) {
  constexpr int kLo = 6, kHi = 22;
  int64_t thr = INT64_MAX;
  for (int k = kHi; k >= kLo; --k) {
    const int64_t b = int64_t(1) << k;
    const double pd = marginal2(sp.packDevice, b, bl), ud = marginal2(sp.unpackDevice, b, bl);
    const double pd5 = marginal2(sp.packDevice, b, 512), ud5 = marginal2(sp.unpackDevice, b, 512);
    const double pp = marginal1(sp.intraNodeGpuGpuPingpong, b);
    const double ph = marginal2(sp.packHost, b, bl), uh = marginal2(sp.unpackHost, b, bl);
    const double cc = marginal1(sp.intraNodeCpuCpuPingpong, b);
    if (pd < 0 || ud < 0 || pd5 < 0 || ud5 < 0 || pp < 0 || ph < 0 || uh < 0 || cc < 0) return -1;
    const double ipc = pd + std::max(0.0, pp - pd5 - ud5) + ud;
    const double oneshot = ph + cc + uh;
    if (ipc < oneshot)
      thr = b; // IPC cheaper from here up
    else
      break;
  }
  return thr;
}

// ------------------------------------------------------------------- JSON

namespace {

struct JV { // minimal JSON value
  enum Kind { NUL, NUM, BOOL, STR, ARR, OBJ } k = NUL;
  double num = 0;
  bool b = false;
  std::string s;
  std::vector<JV> arr;
  std::map<std::string, JV> obj;
};

struct Parser {
  const char *p;
  std::string err;
  void ws() {
    while (*p && std::isspace((unsigned char)*p)) ++p;
  }
  bool parse(JV &v) {
    ws();
    if (*p == '{') {
      ++p;
      v.k = JV::OBJ;
      ws();
      if (*p == '}') {
        ++p;
        return true;
      }
      for (;;) {
        JV key;
        if (!parse(key) || key.k != JV::STR) return fail("object key");
        ws();
        if (*p++ != ':') return fail("':'");
        if (!parse(v.obj[key.s])) return false;
        ws();
        if (*p == ',') {
          ++p;
          continue;
        }
        if (*p == '}') {
          ++p;
          return true;
        }
        return fail("',' or '}'");
      }
    }
    if (*p == '[') {
      ++p;
      v.k = JV::ARR;
      ws();
      if (*p == ']') {
        ++p;
        return true;
      }
      for (;;) {
        v.arr.emplace_back();
        if (!parse(v.arr.back())) return false;
        ws();
        if (*p == ',') {
          ++p;
          continue;
        }
        if (*p == ']') {
          ++p;
          return true;
        }
        return fail("',' or ']'");
      }
    }
    if (*p == '"') {
      ++p;
      v.k = JV::STR;
      while (*p && *p != '"') v.s += *p++;
      if (*p++ != '"') return fail("string end");
      return true;
    }
    if (!std::strncmp(p, "true", 4)) {
      p += 4;
      v.k = JV::BOOL;
      v.b = true;
      return true;
    }
    if (!std::strncmp(p, "false", 5)) {
      p += 5;
      v.k = JV::BOOL;
      return true;
    }
    if (!std::strncmp(p, "null", 4)) {
      p += 4;
      return true;
    }
    char *end = nullptr;
    v.num = std::strtod(p, &end);
    if (end == p) return fail("value");
    v.k = JV::NUM;
    p = end;
    return true;
  }
  bool fail(const char *what) {
    err = std::string("expected ") + what + " near '" + std::string(p).substr(0, 20) + "'";
    return false;
  }
};

bool curve(const JV &v, std::vector<IidTime> *out) {
  if (v.k != JV::ARR) return false;
  out->clear();
  for (const JV &e : v.arr) {
    if (e.k != JV::OBJ || !e.obj.count("time")) return false;
    IidTime t;
    t.time = e.obj.at("time").num;
    t.iid = e.obj.count("iid") && e.obj.at("iid").b;
    out->push_back(t);
  }
  return true;
}

bool curve2(const JV &v, std::vector<std::vector<IidTime>> *out) {
  if (v.k != JV::ARR) return false;
  out->clear();
  for (const JV &row : v.arr) {
    out->emplace_back();
    if (!curve(row, &out->back())) return false;
  }
  return true;
}

void put(std::ostringstream &o, const std::vector<IidTime> &c, int indent) {
  o << "[";
  for (size_t i = 0; i < c.size(); ++i) {
    o << (i ? "," : "") << "\n" << std::string(size_t(indent + 2), ' ') << "{\"iid\": " << (c[i].iid ? "true" : "false")
      << ", \"time\": " << c[i].time << "}";
  }
  o << "\n" << std::string(size_t(indent), ' ') << "]";
}
void put2(std::ostringstream &o, const std::vector<std::vector<IidTime>> &c) {
  o << "[";
  for (size_t i = 0; i < c.size(); ++i) {
    o << (i ? "," : "") << "\n    ";
    put(o, c[i], 4);
  }
  o << "\n  ]";
}

} // namespace

std::string to_json(const SystemPerformance &sp) {
  std::ostringstream o;
  o.precision(9);
  o << "{\n  \"cudaKernelLaunch\": " << sp.cudaKernelLaunch;
  auto one = [&](const char *k, const std::vector<IidTime> &c) {
    o << ",\n  \"" << k << "\": ";
    put(o, c, 2);
  };
  auto two = [&](const char *k, const std::vector<std::vector<IidTime>> &c) {
    o << ",\n  \"" << k << "\": ";
    put2(o, c);
  };
  one("d2h", sp.d2h);
  one("h2d", sp.h2d);
  one("interNodeCpuCpuPingpong", sp.interNodeCpuCpuPingpong);
  one("interNodeGpuGpuPingpong", sp.interNodeGpuGpuPingpong);
  one("intraNodeCpuCpuPingpong", sp.intraNodeCpuCpuPingpong);
  one("intraNodeGpuGpuPingpong", sp.intraNodeGpuGpuPingpong);
  two("packDevice", sp.packDevice);
  two("packHost", sp.packHost);
  two("unpackDevice", sp.unpackDevice);
  two("unpackHost", sp.unpackHost);
  o << "\n}\n";
  return o.str();
}

bool from_json(const std::string &text, SystemPerformance *sp, std::string *err) {
  Parser ps{text.c_str(), ""};
  JV root;
  if (!ps.parse(root) || root.k != JV::OBJ) {
    if (err) *err = ps.err.empty() ? "not a JSON object" : ps.err;
    return false;
  }
  SystemPerformance r;
  auto need = [&](const char *k) -> const JV * {
    auto it = root.obj.find(k);
    if (it == root.obj.end()) {
      if (err) *err = std::string("missing key ") + k;
      return nullptr;
    }
    return &it->second;
  };
  const JV *v;
  if (!(v = need("cudaKernelLaunch"))) return false;
  r.cudaKernelLaunch = v->num;
  struct {
    const char *k;
    std::vector<IidTime> *c;
  } ones[] = {{"intraNodeCpuCpuPingpong", &r.intraNodeCpuCpuPingpong},
              {"intraNodeGpuGpuPingpong", &r.intraNodeGpuGpuPingpong},
              {"interNodeCpuCpuPingpong", &r.interNodeCpuCpuPingpong},
              {"interNodeGpuGpuPingpong", &r.interNodeGpuGpuPingpong},
              {"d2h", &r.d2h},
              {"h2d", &r.h2d}};
  for (auto &o : ones)
    if (!(v = need(o.k)) || !curve(*v, o.c)) {
      if (err && v) *err = std::string("bad curve ") + o.k;
      return false;
    }
  struct {
    const char *k;
    std::vector<std::vector<IidTime>> *c;
  } twos[] = {{"packDevice", &r.packDevice},
              {"unpackDevice", &r.unpackDevice},
              {"packHost", &r.packHost},
              {"unpackHost", &r.unpackHost}};
  for (auto &o : twos)
    if (!(v = need(o.k)) || !curve2(*v, o.c)) {
      if (err && v) *err = std::string("bad table ") + o.k;
      return false;
    }
  *sp = r;
  return true;
}

static std::string perf_path() { return env.cacheDir + "/perf.json"; }

// the model shipped with the library: measured on an MI355X node by
// apps/measure_system (tempi_amd/data/perf_mi355x.json, found next to
// lib/libtempi.so as ../data/)
static std::string shipped_path() {
  Dl_info info;
  if (!dladdr(reinterpret_cast<void *>(&shipped_path), &info) || !info.dli_fname) return "";
  std::string lib = info.dli_fname;
  const size_t slash = lib.rfind('/');
  if (slash == std::string::npos) return "";
  return lib.substr(0, slash) + "/../data/perf_mi355x.json";
}

static bool load_file(const std::string &path, SystemPerformance *sp) {
  std::ifstream f(path);
  if (!f) return false;
  std::stringstream ss;
  ss << f.rdbuf();
  std::string err;
  if (!from_json(ss.str(), sp, &err)) {
    LOG_ERROR("ignoring " << path << ": " << err << " (re-run measure_system)");
    return false;
  }
  LOG_DEBUG("loaded " << path);
  return true;
}

bool import_system_performance(SystemPerformance *sp) {
  // this node's own measurement first (TEMPI_CACHE_DIR/perf.json, as in the
  // reference), then the shipped MI355X model; with neither, AUTO uses the
  // built-in policy (the reference stops: F10)
  systemPerformanceSource.clear();
  systemPerformanceNode = false;
  if (load_file(perf_path(), sp)) {
    systemPerformanceSource = perf_path();
    systemPerformanceNode = true;
    return true;
  }
  if (load_file(shipped_path(), sp)) {
    systemPerformanceSource = shipped_path();
    return true;
  }
  LOG_DEBUG("no perf.json: AUTO uses the built-in policy");
  return false;
}

bool export_system_performance(const SystemPerformance &sp) {
  ::mkdir(env.cacheDir.c_str(), 0755);
  std::ofstream f(perf_path());
  if (!f) {
    LOG_ERROR("cannot write " << perf_path());
    return false;
  }
  f << to_json(sp);
  return bool(f);
}

} // namespace tempi
