/*
 * oracle/typemap.h -- TEST INFRASTRUCTURE ONLY. The CPU oracle for TEMPI's pack
 * path. Nothing in libtempi / libtempi_hip links, loads or calls this; only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg do.
 *
 * Two restatements live here:
 *
 *  1. oracle_tm_*: the MPI type map of a datatype recipe (recipe.h), built by
 *     the MPI-3.1 rules (sec. 4.1.2-4.1.7), and MPI_Pack / MPI_Unpack over it
 *     (MPI-3.1 sec. 4.2: packed bytes = the type map's bytes, in type-map
 *     order, one element after another at stride = extent). This is what the
 *     reference's own parity test treats as truth: the library MPI_Pack
 *     (/root/reference/test/pack_unpack.cpp:61-97). It is pinned against
 *     MPICH 3.3.2's MPI_Pack by tests/golden/ (see oracle/gen_golden.c).
 *
 *  2. oracle_strided_pack / _unpack: the gather/scatter the reference's
 *     packer kernels perform for a canonical StridedBlock
 *     (/root/reference/include/pack_kernels.cuh:64-120 pack_2d/unpack_2d,
 *     :350-433 pack_3d/unpack_3d; descriptor layout
 *     /root/reference/include/strided_block.hpp:12-67), restated with the
 *     outer element count as one more dimension of stride = extent, which is
 *     what MPI requires (and what the reference gets wrong for 1D).
 */
#ifndef TEMPI_ORACLE_TYPEMAP_H
#define TEMPI_ORACLE_TYPEMAP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_tm oracle_tm;

/* build a type map from a recipe string; NULL on parse error (err filled) */
oracle_tm *oracle_tm_build(const char *recipe, char *err, int errlen);
void oracle_tm_free(oracle_tm *t);

int64_t oracle_tm_size(const oracle_tm *t);   /* MPI_Type_size */
int64_t oracle_tm_lb(const oracle_tm *t);     /* MPI_Type_get_extent lb */
int64_t oracle_tm_extent(const oracle_tm *t); /* MPI_Type_get_extent extent */
int64_t oracle_tm_true_lb(const oracle_tm *t);
int64_t oracle_tm_true_extent(const oracle_tm *t);
int64_t oracle_tm_nsegs(const oracle_tm *t); /* contiguous runs, merged */
/* copy out run i: byte displacement and length */
void oracle_tm_seg(const oracle_tm *t, int64_t i, int64_t *disp, int64_t *len);

/* MPI_Pack(inbuf=base, incount, type) -> out, appended at *position.
   `base` is the buffer origin that displacements are relative to. */
void oracle_tm_pack(const oracle_tm *t, int64_t incount, const uint8_t *base,
                    uint8_t *out, int64_t *position);
void oracle_tm_unpack(const oracle_tm *t, int64_t outcount, const uint8_t *in,
                      int64_t *position, uint8_t *base);

/* Canonical strided descriptor: the first byte is at `start`; `block` bytes
   are contiguous; then ndims dims, listed OUTERMOST FIRST, each (count,
   stride in bytes). `incount` elements are `extent` bytes apart. */
void oracle_strided_pack(int64_t start, int64_t block, int ndims,
                         const int64_t *counts, const int64_t *strides,
                         int64_t incount, int64_t extent, const uint8_t *base,
                         uint8_t *out);
void oracle_strided_unpack(int64_t start, int64_t block, int ndims,
                           const int64_t *counts, const int64_t *strides,
                           int64_t outcount, int64_t extent, const uint8_t *in,
                           uint8_t *base);

#ifdef __cplusplus
}
#endif
#endif
