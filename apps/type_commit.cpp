// apps/type_commit.cpp -- what MPI_Type_commit costs, after
// the reference's bench_type_commit (/root/reference/bin/bench_type_commit.cpp:
// 27-53, 72-160): for each copy extent of its list inside a 1024^3-byte
// allocation, each of its five constructions of the same 3D byte box
// (/root/reference/support/type.cpp: make_subarray :158, make_byte_v_hv :67,
// make_byte_v1_hv_hv :34, make_byte_vn_hv_hv :3, make_subarray_v :172) is
// created, committed and freed ITERS times; trimean of the create and of the
// commit time. Through libtempi the commit also canonicalises the type into
// its strided descriptor (core/types.cpp); with TEMPI_DISABLE=1 it is the
// library's commit alone.
//
// usage: mpiexec -n 1 type_commit [ITERS]     one JSON object (rank 0)
#include <mpi.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

namespace {

struct Dim3 {
  int x, y, z;
};

MPI_Datatype make_subarray(Dim3 c, Dim3 a) {
  int sizes[3] = {a.z, a.y, a.x}, subs[3] = {c.z, c.y, c.x}, starts[3] = {0, 0, 0};
  MPI_Datatype t;
  MPI_Type_create_subarray(3, sizes, subs, starts, MPI_ORDER_C, MPI_BYTE, &t);
  return t;
}

MPI_Datatype make_byte_v_hv(Dim3 c, Dim3 a) {
  MPI_Datatype plane, t;
  MPI_Type_vector(c.y, c.x, a.x, MPI_BYTE, &plane);
  MPI_Type_create_hvector(c.z, 1, MPI_Aint(a.x) * a.y, plane, &t);
  MPI_Type_free(&plane);
  return t;
}

MPI_Datatype make_byte_v1_hv_hv(Dim3 c, Dim3 a) {
  MPI_Datatype row, plane, t;
  MPI_Type_vector(1, c.x, a.x, MPI_BYTE, &row);
  MPI_Type_create_hvector(c.y, 1, a.x, row, &plane);
  MPI_Type_create_hvector(c.z, 1, MPI_Aint(a.x) * a.y, plane, &t);
  MPI_Type_free(&row);
  MPI_Type_free(&plane);
  return t;
}

MPI_Datatype make_byte_vn_hv_hv(Dim3 c, Dim3 a) {
  MPI_Datatype row, plane, t;
  MPI_Type_vector(c.x, 1, 1, MPI_BYTE, &row);
  MPI_Type_create_hvector(c.y, 1, a.x, row, &plane);
  MPI_Type_create_hvector(c.z, 1, MPI_Aint(a.x) * a.y, plane, &t);
  MPI_Type_free(&row);
  MPI_Type_free(&plane);
  return t;
}

MPI_Datatype make_subarray_v(Dim3 c, Dim3 a) {
  int sizes[2] = {a.y, a.x}, subs[2] = {c.y, c.x}, starts[2] = {0, 0};
  MPI_Datatype plane, t;
  MPI_Type_create_subarray(2, sizes, subs, starts, MPI_ORDER_C, MPI_BYTE, &plane);
  MPI_Type_create_hvector(c.z, 1, MPI_Aint(a.x) * a.y, plane, &t);
  MPI_Type_free(&plane);
  return t;
}

double trimean(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  auto pct = [&](double p) {
    const double idx = p * double(v.size() - 1);
    const size_t lo = size_t(std::floor(idx)), hi = size_t(std::ceil(idx));
    return v[lo] + (v[hi] - v[lo]) * (idx - double(lo));
  };
  return (pct(0.25) + 2 * pct(0.5) + pct(0.75)) / 4;
}

double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

} // namespace

int main(int argc, char **argv) {
  MPI_Init(&argc, &argv);
  const int iters = argc > 1 ? std::max(1, std::atoi(argv[1])) : 1000;
  const Dim3 alloc{1024, 1024, 1024};
  // the reference's extents (bench_type_commit.cpp:84-94)
  const std::vector<Dim3> dims = {
      {1, 1024, 1024}, {2, 1024, 512},  {4, 1024, 256},  {8, 1024, 128}, {16, 1024, 64},  {32, 1024, 32},
      {64, 1024, 16},  {128, 1024, 8},  {256, 1024, 4},  {512, 1024, 2}, {1024, 1024, 1}, {1, 1024, 1},
      {2, 1024, 1},    {4, 1024, 1},    {8, 1024, 1},    {16, 1024, 1},  {32, 1024, 1},   {64, 1024, 1},
      {128, 1024, 1},  {256, 1024, 1},  {512, 1024, 1},  {12, 512, 512}, {512, 3, 512},   {512, 512, 3}};
  struct Factory {
    const char *name;
    MPI_Datatype (*make)(Dim3, Dim3);
  };
  const Factory factories[] = {{"subarray", make_subarray},
                               {"byte_v_hv", make_byte_v_hv},
                               {"byte_v1_hv_hv", make_byte_v1_hv_hv},
                               {"byte_vn_hv_hv", make_byte_vn_hv_hv},
                               {"subarray_v", make_subarray_v}};
  std::string out = "{\"iters\": " + std::to_string(iters) + ", \"alloc\": [1024, 1024, 1024], \"extents\": [";
  for (size_t i = 0; i < dims.size(); ++i)
    out += (i ? ", [" : "[") + std::to_string(dims[i].x) + ", " + std::to_string(dims[i].y) + ", " +
           std::to_string(dims[i].z) + "]";
  out += "], \"factories\": {";
  std::vector<double> allCommit;
  for (size_t f = 0; f < sizeof factories / sizeof factories[0]; ++f) {
    std::string cr, cm;
    for (size_t i = 0; i < dims.size(); ++i) {
      std::vector<double> tc, tm;
      for (int n = 0; n < iters; ++n) {
        double t0 = now_us();
        MPI_Datatype t = factories[f].make(dims[i], alloc);
        double t1 = now_us();
        MPI_Type_commit(&t);
        double t2 = now_us();
        MPI_Type_free(&t);
        tc.push_back(t1 - t0);
        tm.push_back(t2 - t1);
      }
      char buf[64];
      std::snprintf(buf, sizeof buf, "%s%.3f", i ? ", " : "", trimean(tc));
      cr += buf;
      const double m = trimean(tm);
      allCommit.push_back(m);
      std::snprintf(buf, sizeof buf, "%s%.3f", i ? ", " : "", m);
      cm += buf;
    }
    out += std::string(f ? ", " : "") + "\"" + factories[f].name + "\": {\"create_us\": [" + cr + "], \"commit_us\": [" +
           cm + "]}";
  }
  std::sort(allCommit.begin(), allCommit.end());
  char tail[160];
  std::snprintf(tail, sizeof tail, "}, \"commit_us_median\": %.3f, \"commit_us_max\": %.3f, \"tempi\": %s}",
                allCommit[allCommit.size() / 2], allCommit.back(), std::getenv("TEMPI_DISABLE") ? "false" : "true");
  out += tail;
  int rank = 0;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  if (rank == 0) std::printf("%s\n", out.c_str());
  MPI_Finalize();
  return 0;
}
