// tempi_amd/csrc/core/iid.cpp -- is a benchmark's sample set independent and
// identically distributed? The permutation test of NIST SP 800-90B sec. 5.1,
// used by tools/measure_system to decide when a timing curve is trustworthy
// (the reference repeats a measurement until its samples pass:
// /root/reference/src/internal/benchmark.cpp:44-89, sp_800_90B at
// /root/reference/src/internal/iid.cpp:180-245).
//
// Statistics (SP 800-90B 5.1.1-5.1.11 for non-binary data): excursion,
// number and longest length of directional runs, max(increases, decreases),
// number and longest length of runs about the median, average and maximum
// collision distance, periodicity and covariance at lags 1, 2, 8, 16, 32.
// Each is computed on the sequence and on `perms` random shuffles of it;
// IID is rejected when the original ranks in the extreme tails:
// (C0 + C1 <= 5*perms/10000) or (C0 >= 9995*perms/10000), with C0 / C1 the
// shuffles whose statistic is greater than / equal to the original.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <numeric>
#include <random>
#include <vector>

namespace tempi {
namespace {

typedef std::vector<double> Seq;

double median(Seq s) {
  std::sort(s.begin(), s.end());
  const size_t n = s.size();
  return n % 2 ? s[n / 2] : 0.5 * (s[n / 2 - 1] + s[n / 2]);
}

// all statistics of one sequence (median passed in: it is permutation-invariant)
std::vector<double> statistics(const Seq &s, double med) {
  const size_t n = s.size();
  std::vector<double> t;
  const double mean = std::accumulate(s.begin(), s.end(), 0.0) / double(n);
  { // excursion
    double run = 0, mx = 0;
    for (size_t i = 0; i < n; ++i) {
      run += s[i];
      mx = std::max(mx, std::fabs(run - double(i + 1) * mean));
    }
    t.push_back(mx);
  }
  { // directional runs: number, longest, max(inc, dec)
    double runs = n > 1 ? 1 : 0, longest = n > 1 ? 1 : 0, cur = 1, inc = 0, dec = 0;
    for (size_t i = 0; i + 1 < n; ++i) {
      const bool up = s[i] <= s[i + 1];
      (up ? inc : dec) += 1;
      if (i + 2 < n) {
        const bool up2 = s[i + 1] <= s[i + 2];
        if (up2 == up) {
          ++cur;
        } else {
          ++runs;
          cur = 1;
        }
        longest = std::max(longest, cur);
      }
    }
    t.push_back(runs);
    t.push_back(longest);
    t.push_back(std::max(inc, dec));
  }
  { // runs about the median
    double runs = 1, longest = 1, cur = 1;
    for (size_t i = 0; i + 1 < n; ++i) {
      if ((s[i] >= med) == (s[i + 1] >= med)) {
        ++cur;
      } else {
        ++runs;
        cur = 1;
      }
      longest = std::max(longest, cur);
    }
    t.push_back(runs);
    t.push_back(longest);
  }
  { // collisions: distance to the next repeat of a value
    double sum = 0, cnt = 0, mx = 0;
    size_t i = 0;
    while (i < n) {
      size_t j = i + 1;
      for (; j < n; ++j)
        if (s[j] == s[i]) break;
      if (j < n) {
        sum += double(j - i);
        cnt += 1;
        mx = std::max(mx, double(j - i));
      }
      i = j + 1;
    }
    t.push_back(cnt ? sum / cnt : 0);
    t.push_back(mx);
  }
  for (size_t p : {1, 2, 8, 16, 32}) { // periodicity and covariance
    double per = 0, cov = 0;
    for (size_t i = 0; i + p < n; ++i) {
      per += s[i] == s[i + p];
      cov += s[i] * s[i + p];
    }
    t.push_back(per);
    t.push_back(cov);
  }
  return t;
}

} // namespace

bool sp800_90b_iid(const std::vector<double> &s, int perms, uint64_t seed) {
  if (s.size() < 3) return false;
  const double med = median(s);
  const std::vector<double> t0 = statistics(s, med);
  std::vector<int> c0(t0.size(), 0), c1(t0.size(), 0);
  std::mt19937_64 g(seed);
  Seq p = s;
  for (int k = 0; k < perms; ++k) {
    std::shuffle(p.begin(), p.end(), g);
    const std::vector<double> t = statistics(p, med);
    for (size_t i = 0; i < t.size(); ++i) {
      if (t[i] > t0[i])
        ++c0[i];
      else if (t[i] == t0[i])
        ++c1[i];
    }
  }
  const double lo = 5.0 * perms / 10000.0, hi = 9995.0 * perms / 10000.0;
  for (size_t i = 0; i < t0.size(); ++i)
    if (double(c0[i] + c1[i]) <= lo || double(c0[i]) >= hi) return false;
  return true;
}

} // namespace tempi

extern "C" __attribute__((visibility("default"))) int tempi_sp800_90b_iid(const double *samples, int n, int perms,
                                                                          uint64_t seed) {
  return tempi::sp800_90b_iid(std::vector<double>(samples, samples + (n > 0 ? n : 0)), perms, seed) ? 1 : 0;
}
