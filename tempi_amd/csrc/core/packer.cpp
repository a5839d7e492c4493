// tempi_amd/csrc/core/packer.cpp -- see packer.hpp
#include "packer.hpp"

#include "counters.hpp"
#include "tempi_hip.h"

#include <vector>

namespace tempi {

namespace {

// issue one launch per index of the outermost dims until the rest fits
int issue(bool pack, char *packed, char *first, int64_t block, const Dim *dims, int nd,
          void *stream) {
  if (nd <= TEMPI_HIP_MAX_DIMS) {
    tempi_hip_desc d{};
    d.block = block;
    d.ndims = nd;
    for (int k = 0; k < nd; ++k) {
      d.counts[k] = dims[k].count;
      d.strides[k] = dims[k].stride;
    }
    counters.launches++;
    return pack ? tempi_hip_pack(packed, first, &d, stream) : tempi_hip_unpack(first, packed, &d, stream);
  }
  int64_t inner = block;
  for (int k = 1; k < nd; ++k) inner *= dims[k].count;
  for (int64_t i = 0; i < dims[0].count; ++i) {
    if (int e = issue(pack, packed + i * inner, first + i * dims[0].stride, block, dims + 1, nd - 1, stream))
      return e;
  }
  return 0;
}

void collect(char *packed, char *first, int64_t block, const Dim *dims, int nd,
             std::vector<tempi_hip_batch_item> &out) {
  if (nd <= TEMPI_HIP_MAX_DIMS) {
    tempi_hip_batch_item it{};
    it.packed = packed;
    it.first = first;
    it.desc.block = block;
    it.desc.ndims = nd;
    for (int k = 0; k < nd; ++k) {
      it.desc.counts[k] = dims[k].count;
      it.desc.strides[k] = dims[k].stride;
    }
    out.push_back(it);
    return;
  }
  int64_t inner = block;
  for (int k = 1; k < nd; ++k) inner *= dims[k].count;
  for (int64_t i = 0; i < dims[0].count; ++i)
    collect(packed + i * inner, first + i * dims[0].stride, block, dims + 1, nd - 1, out);
}

} // namespace

void Packer::items(void *packed, const void *origin, int64_t count, std::vector<tempi_hip_batch_item> &out) const {
  if (count <= 0 || sb_.size == 0) return;
  StridedBlock tmp;
  tmp.block = sb_.block;
  if (count > 1) tmp.dims.push_back(Dim{count, sb_.extent});
  tmp.dims.insert(tmp.dims.end(), sb_.dims.begin(), sb_.dims.end());
  simplify(tmp);
  collect(static_cast<char *>(packed), const_cast<char *>(static_cast<const char *>(origin)) + sb_.start, tmp.block,
          tmp.dims.data(), int(tmp.dims.size()), out);
}

bool Packer::flat(int64_t count, tempi_hip_desc *out) const {
  StridedBlock tmp;
  tmp.block = sb_.block;
  if (count > 1) tmp.dims.push_back(Dim{count, sb_.extent});
  tmp.dims.insert(tmp.dims.end(), sb_.dims.begin(), sb_.dims.end());
  simplify(tmp);
  if (tmp.dims.size() > size_t(TEMPI_HIP_MAX_DIMS)) return false;
  *out = tempi_hip_desc{};
  out->block = count > 0 ? tmp.block : 0;
  out->ndims = int32_t(tmp.dims.size());
  for (size_t k = 0; k < tmp.dims.size(); ++k) {
    out->counts[k] = tmp.dims[k].count;
    out->strides[k] = tmp.dims[k].stride;
  }
  return true;
}

int Packer::launch(bool pack, char *packed, char *origin, int64_t count, void *stream, Completion *done) const {
  if (count <= 0 || sb_.size == 0) return 0;
  std::vector<Dim> dims;
  dims.reserve(sb_.dims.size() + 1);
  if (count > 1) dims.push_back(Dim{count, sb_.extent});
  dims.insert(dims.end(), sb_.dims.begin(), sb_.dims.end());
  StridedBlock tmp;
  tmp.block = sb_.block;
  tmp.dims = dims;
  simplify(tmp); // the count dimension may merge (e.g. dense types)
  const int64_t bytes = packed_bytes(count);
  if (pack) {
    counters.packs++;
    counters.pack_bytes += uint64_t(bytes);
  } else {
    counters.unpacks++;
    counters.unpack_bytes += uint64_t(bytes);
  }
  char *first = origin + sb_.start;
  if (done && tmp.dims.size() <= size_t(TEMPI_HIP_MAX_DIMS)) { // one descriptor: the ticket may fold into it
    tempi_hip_desc d{};
    d.block = tmp.block;
    d.ndims = int32_t(tmp.dims.size());
    for (size_t k = 0; k < tmp.dims.size(); ++k) {
      d.counts[k] = tmp.dims[k].count;
      d.strides[k] = tmp.dims[k].stride;
    }
    // a small object: the resident packer, if it takes it, needs no launch (and
    // no wait: the call returns once the work is done). Not while kernels are
    // timed by events on the stream (kernelProfiling): it launches nothing there
    if (!kernelProfiling) {
      int served = 0;
      const int e = pack ? tempi_hip_pack_resident(packed, first, &d, stream, &served)
                         : tempi_hip_unpack_resident(first, packed, &d, stream, &served);
      if (e) return e;
      if (served) {
        done->flag = nullptr;
        return 0;
      }
    }
    counters.launches++;
    return pack ? tempi_hip_pack_ticket(packed, first, &d, stream, &done->flag, &done->ticket)
                : tempi_hip_unpack_ticket(first, packed, &d, stream, &done->flag, &done->ticket);
  }
  const int e = issue(pack, packed, first, tmp.block, tmp.dims.data(), int(tmp.dims.size()), stream);
  if (e || !done) return e;
  return tempi_hip_stream_ticket(stream, &done->flag, &done->ticket);
}

int Packer::pack_async(void *packed, const void *origin, int64_t count, void *stream) const {
  return launch(true, static_cast<char *>(packed), const_cast<char *>(static_cast<const char *>(origin)),
                count, stream, nullptr);
}

int Packer::unpack_async(void *origin, const void *packed, int64_t count, void *stream) const {
  return launch(false, const_cast<char *>(static_cast<const char *>(packed)), static_cast<char *>(origin),
                count, stream, nullptr);
}

int Packer::pack_ticket(void *packed, const void *origin, int64_t count, void *stream, Completion *done) const {
  return launch(true, static_cast<char *>(packed), const_cast<char *>(static_cast<const char *>(origin)),
                count, stream, done);
}

int Packer::unpack_ticket(void *origin, const void *packed, int64_t count, void *stream, Completion *done) const {
  return launch(false, const_cast<char *>(static_cast<const char *>(packed)), static_cast<char *>(origin),
                count, stream, done);
}

} // namespace tempi
