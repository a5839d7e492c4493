// tempi_amd/csrc/core/types.cpp -- datatype canonicalisation (see types.hpp).
//
// Decoding walks the constructor tree with MPI_Type_get_envelope /
// MPI_Type_get_contents like the reference's Type::from_mpi_datatype
// (/root/reference/src/internal/types.cpp:42-344), but each constructor maps
// straight to "dims over a block" and additionally covers Fortran-order
// subarrays, resized, dup, regular (h)indexed(_block) and single-type struct.
#include "types.hpp"

#include "log.hpp"
#include "next_mpi.hpp"

#include <sstream>

namespace tempi {

namespace {

struct Layout {
  bool ok = false;
  int64_t start = 0;
  int64_t block = 0;
  std::vector<Dim> dims; // outermost first
};

Layout decode(MPI_Datatype t);

// child handles returned by MPI_Type_get_contents must be freed unless
// predefined; go straight to the library so TEMPI's type cache is untouched
void release_child(MPI_Datatype t) {
  int ni, na, nd, comb;
  MPI_Type_get_envelope(t, &ni, &na, &nd, &comb);
  if (comb != MPI_COMBINER_NAMED) next.MPI_Type_free(&t);
}

int64_t type_extent(MPI_Datatype t) {
  MPI_Aint lb, ext;
  MPI_Type_get_extent(t, &lb, &ext);
  return int64_t(ext);
}

// `count` copies of `child`, at the given byte displacements, each copy a run
// of `blen` child elements
Layout from_blocks(const Layout &child, int64_t childExtent, const std::vector<int64_t> &disp,
                   const std::vector<int64_t> &blen) {
  Layout r;
  std::vector<int64_t> d, b;
  for (size_t i = 0; i < disp.size(); ++i)
    if (blen[i] > 0) {
      d.push_back(disp[i]);
      b.push_back(blen[i]);
    }
  if (!child.ok) return r;
  if (d.empty()) { // empty type map
    r.ok = true;
    r.block = 0;
    return r;
  }
  for (size_t i = 1; i < b.size(); ++i)
    if (b[i] != b[0]) return r; // ragged blocks: not a strided block
  const int64_t step = d.size() > 1 ? d[1] - d[0] : 0;
  for (size_t i = 2; i < d.size(); ++i)
    if (d[i] - d[i - 1] != step) return r; // irregular displacements
  r.ok = true;
  r.start = d[0] + child.start;
  r.block = child.block;
  if (d.size() > 1) r.dims.push_back({int64_t(d.size()), step});
  r.dims.push_back({b[0], childExtent});
  r.dims.insert(r.dims.end(), child.dims.begin(), child.dims.end());
  return r;
}

Layout decode(MPI_Datatype t) {
  Layout r;
  int ni = 0, na = 0, nd = 0, comb = 0;
  MPI_Type_get_envelope(t, &ni, &na, &nd, &comb);

  if (comb == MPI_COMBINER_NAMED) {
    int size = 0;
    MPI_Aint lb, ext;
    MPI_Type_size(t, &size);
    MPI_Type_get_extent(t, &lb, &ext);
    // a dense predefined type; pair types with padding are not
    if (size > 0 && lb == 0 && int64_t(ext) == size) {
      r.ok = true;
      r.block = size;
    }
    return r;
  }

  std::vector<int> ints(ni > 0 ? ni : 1);
  std::vector<MPI_Aint> addrs(na > 0 ? na : 1);
  std::vector<MPI_Datatype> types(nd > 0 ? nd : 1);
  MPI_Type_get_contents(t, ni, na, nd, ints.data(), addrs.data(), types.data());

  Layout child;
  int64_t ce = 0;
  bool singleChild = true;
  if (comb == MPI_COMBINER_STRUCT) {
    // only a struct whose blocks all share one type is strided
    for (int i = 1; i < nd; ++i)
      if (types[i] != types[0]) singleChild = false;
  }
  if (nd >= 1 && singleChild) {
    child = decode(types[0]);
    ce = type_extent(types[0]);
  }

  switch (comb) {
  case MPI_COMBINER_DUP:
  case MPI_COMBINER_RESIZED: // new lb/extent markers, same type map
    r = child;
    break;
  case MPI_COMBINER_CONTIGUOUS:
    if (child.ok) {
      r = child;
      r.dims.insert(r.dims.begin(), Dim{ints[0], ce});
    }
    break;
  case MPI_COMBINER_VECTOR:
    if (child.ok) {
      r = child;
      r.dims.insert(r.dims.begin(), {Dim{ints[0], int64_t(ints[2]) * ce}, Dim{ints[1], ce}});
    }
    break;
  case MPI_COMBINER_HVECTOR:
#ifdef MPI_COMBINER_HVECTOR_INTEGER
  case MPI_COMBINER_HVECTOR_INTEGER:
#endif
    if (child.ok) {
      const int64_t stride = comb == MPI_COMBINER_HVECTOR ? int64_t(addrs[0]) : int64_t(ints[2]);
      r = child;
      r.dims.insert(r.dims.begin(), {Dim{ints[0], stride}, Dim{ints[1], ce}});
    }
    break;
  case MPI_COMBINER_INDEXED:
  case MPI_COMBINER_HINDEXED:
#ifdef MPI_COMBINER_HINDEXED_INTEGER
  case MPI_COMBINER_HINDEXED_INTEGER:
#endif
  {
    const int n = ints[0];
    std::vector<int64_t> disp(n), blen(n);
    for (int i = 0; i < n; ++i) {
      blen[i] = ints[1 + i];
      if (comb == MPI_COMBINER_INDEXED)
        disp[i] = int64_t(ints[1 + n + i]) * ce;
      else if (comb == MPI_COMBINER_HINDEXED)
        disp[i] = int64_t(addrs[i]);
      else
        disp[i] = int64_t(ints[1 + n + i]);
    }
    r = from_blocks(child, ce, disp, blen);
    break;
  }
  case MPI_COMBINER_INDEXED_BLOCK:
  case MPI_COMBINER_HINDEXED_BLOCK: {
    const int n = ints[0];
    std::vector<int64_t> disp(n), blen(n, ints[1]);
    for (int i = 0; i < n; ++i)
      disp[i] = comb == MPI_COMBINER_INDEXED_BLOCK ? int64_t(ints[2 + i]) * ce : int64_t(addrs[i]);
    r = from_blocks(child, ce, disp, blen);
    break;
  }
  case MPI_COMBINER_STRUCT: {
    if (!singleChild) break;
    const int n = ints[0];
    std::vector<int64_t> disp(n), blen(n);
    for (int i = 0; i < n; ++i) {
      blen[i] = ints[1 + i];
      disp[i] = int64_t(addrs[i]);
    }
    r = from_blocks(child, ce, disp, blen);
    break;
  }
  case MPI_COMBINER_SUBARRAY: {
    if (!child.ok) break;
    const int n = ints[0];
    const int *sizes = &ints[1], *subs = &ints[1 + n], *starts = &ints[1 + 2 * n];
    const int order = ints[1 + 3 * n];
    std::vector<Dim> dims(n);
    int64_t off = 0, full = ce;
    if (order == MPI_ORDER_C) {
      for (int i = n - 1; i >= 0; --i) { // dims[0] = array dim 0 = outermost
        dims[i] = Dim{subs[i], full};
        off += int64_t(starts[i]) * full;
        full *= sizes[i];
      }
    } else { // Fortran: array dim 0 varies fastest = innermost
      for (int i = 0; i < n; ++i) {
        dims[n - 1 - i] = Dim{subs[i], full};
        off += int64_t(starts[i]) * full;
        full *= sizes[i];
      }
    }
    r = child;
    r.start += off;
    r.dims.insert(r.dims.begin(), dims.begin(), dims.end());
    break;
  }
  default:
    break; // darray, F90 types, ...: library
  }

  for (int i = 0; i < nd; ++i) release_child(types[i]);
  return r;
}

} // namespace

void simplify(StridedBlock &sb) {
  std::vector<Dim> d;
  bool empty = sb.block == 0;
  for (const Dim &x : sb.dims) {
    if (x.count == 0) empty = true;
    if (x.count != 1) d.push_back(x);
  }
  if (empty) {
    sb.dims.clear();
    sb.block = 0;
    return;
  }
  bool changed = true;
  while (changed) {
    changed = false;
    if (!d.empty() && d.back().stride == sb.block) { // dense innermost dim
      sb.block *= d.back().count;
      d.pop_back();
      changed = true;
    }
    for (size_t k = 0; k + 1 < d.size(); ++k) {
      if (d[k].stride == d[k + 1].count * d[k + 1].stride) { // contiguous nest
        d[k].count *= d[k + 1].count;
        d[k].stride = d[k + 1].stride;
        d.erase(d.begin() + k + 1);
        changed = true;
        break;
      }
    }
  }
  sb.dims = d;
}

StridedBlock canonicalise(MPI_Datatype t) {
  StridedBlock sb;
  Layout l = decode(t);
  int size = 0;
  MPI_Aint lb = 0, ext = 0;
  MPI_Type_size(t, &size);
  MPI_Type_get_extent(t, &lb, &ext);
  sb.size = size;
  sb.lb = lb;
  sb.extent = ext;
  if (!l.ok) return sb;
  sb.start = l.start;
  sb.block = l.block;
  sb.dims = l.dims;
  simplify(sb);
  // defensive: the descriptor must account for exactly the type's bytes
  if (sb.block * sb.rows() != sb.size) {
    LOG_WARN("canonical form of type " << t << " has " << sb.block * sb.rows()
                                       << " bytes, MPI says " << sb.size << "; library path");
    return sb;
  }
  sb.valid = true;
  return sb;
}

std::string StridedBlock::str() const {
  std::ostringstream s;
  s << "StridedBlock{valid:" << valid << ",start:" << start << ",block:" << block << ",dims:[";
  for (const Dim &d : dims) s << "(" << d.count << "," << d.stride << ")";
  s << "],size:" << size << ",lb:" << lb << ",extent:" << extent << "}";
  return s.str();
}

} // namespace tempi
