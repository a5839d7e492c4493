/*
 * oracle/typemap.c -- TEST INFRASTRUCTURE ONLY (see typemap.h for the contract
 * and the reference lines each function restates). Plain C, deliberately
 * naive: the type map is materialised as a list of (displacement, length)
 * runs and packing walks it byte-run by byte-run.
 */
#include "typemap.h"
#include "recipe.h"

#include <stdlib.h>
#include <string.h>

typedef struct {
  int64_t disp, len;
} run;

struct oracle_tm {
  run *runs;
  int64_t n, cap;
  int64_t size;
  int64_t lb, ub;           /* MPI lb / ub markers (extent = ub - lb) */
  int64_t true_lb, true_ub; /* min / max byte actually in the map */
};

static void push(oracle_tm *t, int64_t disp, int64_t len) {
  if (len <= 0) return;
  /* merge with the previous run when contiguous in type-map order */
  if (t->n && t->runs[t->n - 1].disp + t->runs[t->n - 1].len == disp) {
    t->runs[t->n - 1].len += len;
  } else {
    if (t->n == t->cap) {
      t->cap = t->cap ? 2 * t->cap : 16;
      t->runs = (run *)realloc(t->runs, sizeof(run) * (size_t)t->cap);
    }
    t->runs[t->n].disp = disp;
    t->runs[t->n].len = len;
    t->n++;
  }
  t->size += len;
  if (disp < t->true_lb) t->true_lb = disp;
  if (disp + len > t->true_ub) t->true_ub = disp + len;
}

static oracle_tm *empty(void) {
  oracle_tm *t = (oracle_tm *)calloc(1, sizeof(oracle_tm));
  t->true_lb = INT64_MAX;
  t->true_ub = INT64_MIN;
  t->lb = INT64_MAX;
  t->ub = INT64_MIN;
  return t;
}

/* append a copy of `c` displaced by `off`, and widen lb/ub (MPI-3.1 4.1.6:
   lb/ub of a derived type are the min/max over its entries' lb/ub) */
static void append_copy(oracle_tm *t, const oracle_tm *c, int64_t off) {
  for (int64_t i = 0; i < c->n; ++i) push(t, c->runs[i].disp + off, c->runs[i].len);
  if (c->lb + off < t->lb) t->lb = c->lb + off;
  if (c->ub + off > t->ub) t->ub = c->ub + off;
}

static void finish(oracle_tm *t) {
  if (t->lb == INT64_MAX) { /* no entries at all: zero-size type */
    t->lb = 0;
    t->ub = 0;
  }
  if (t->true_lb == INT64_MAX) {
    t->true_lb = 0;
    t->true_ub = 0;
  }
}

static int64_t ext(const oracle_tm *t) { return t->ub - t->lb; }

static oracle_tm *build(const rnode *r) {
  if (r->kind == RK_BASIC) {
    oracle_tm *t = empty();
    push(t, 0, r->size);
    t->lb = 0;
    t->ub = r->size;
    return t;
  }
  oracle_tm *c = build(r->child);
  oracle_tm *t = empty();
  const int64_t e = ext(c);
  switch (r->kind) {
  case RK_DUP:
    append_copy(t, c, 0);
    break;
  case RK_CONTIG: /* MPI_Type_contiguous: n copies at stride extent */
    for (int64_t i = 0; i < r->a[0]; ++i) append_copy(t, c, i * e);
    break;
  case RK_VECTOR:  /* n blocks of bl, block starts `stride` elements apart */
  case RK_HVECTOR: /* ... `stride` bytes apart */
  {
    const int64_t s = r->kind == RK_VECTOR ? r->a[2] * e : r->a[2];
    for (int64_t i = 0; i < r->a[0]; ++i)
      for (int64_t j = 0; j < r->a[1]; ++j) append_copy(t, c, i * s + j * e);
    break;
  }
  case RK_INDEXED:
  case RK_HINDEXED:
  case RK_STRUCT: /* MPI-3.1 4.1.2: blocks of blen[k] copies at byte disp[k] */
    for (int k = 0; k < r->narr[0]; ++k) {
      const int64_t d = r->kind == RK_INDEXED ? r->arr[1][k] * e : r->arr[1][k];
      for (int64_t j = 0; j < r->arr[0][k]; ++j) append_copy(t, c, d + j * e);
    }
    break;
  case RK_INDEXED_BLOCK:
  case RK_HINDEXED_BLOCK:
    for (int k = 0; k < r->narr[1]; ++k) {
      const int64_t d =
          r->kind == RK_INDEXED_BLOCK ? r->arr[1][k] * e : r->arr[1][k];
      for (int64_t j = 0; j < r->a[0]; ++j) append_copy(t, c, d + j * e);
    }
    break;
  case RK_RESIZED: /* same map, new lb/extent markers (MPI-3.1 4.1.7) */
    append_copy(t, c, 0);
    t->lb = r->a[0];
    t->ub = r->a[0] + r->a[1];
    break;
  case RK_SUBARRAY: {
    /* MPI-3.1 4.1.3: elements of the sub-block in array order (C: last index
       fastest, Fortran: first index fastest); the result is resized to
       lb = 0 and extent = prod(sizes) * extent(oldtype). */
    const int nd = r->narr[0];
    const int64_t *sizes = r->arr[0], *sub = r->arr[1], *st = r->arr[2];
    int64_t *stride = (int64_t *)malloc(sizeof(int64_t) * (size_t)nd);
    int64_t *idx = (int64_t *)calloc((size_t)nd, sizeof(int64_t));
    int64_t total = 1, full = 1;
    for (int d = 0; d < nd; ++d) total *= sub[d];
    if (r->order == 'C') {
      for (int d = nd - 1; d >= 0; --d) {
        stride[d] = full * e;
        full *= sizes[d];
      }
    } else {
      for (int d = 0; d < nd; ++d) {
        stride[d] = full * e;
        full *= sizes[d];
      }
    }
    for (int64_t k = 0; k < total; ++k) {
      int64_t off = 0;
      for (int d = 0; d < nd; ++d) off += (st[d] + idx[d]) * stride[d];
      append_copy(t, c, off);
      /* advance the fastest-varying index first */
      if (r->order == 'C') {
        for (int d = nd - 1; d >= 0; --d) {
          if (++idx[d] < sub[d]) break;
          idx[d] = 0;
        }
      } else {
        for (int d = 0; d < nd; ++d) {
          if (++idx[d] < sub[d]) break;
          idx[d] = 0;
        }
      }
    }
    t->lb = 0;
    t->ub = full * e;
    free(stride);
    free(idx);
    break;
  }
  default:
    break;
  }
  oracle_tm_free(c);
  finish(t);
  return t;
}

oracle_tm *oracle_tm_build(const char *recipe, char *err, int errlen) {
  rnode *r = recipe_parse(recipe, err, errlen);
  if (!r) return NULL;
  oracle_tm *t = build(r);
  recipe_free(r);
  return t;
}

void oracle_tm_free(oracle_tm *t) {
  if (!t) return;
  free(t->runs);
  free(t);
}

int64_t oracle_tm_size(const oracle_tm *t) { return t->size; }
int64_t oracle_tm_lb(const oracle_tm *t) { return t->lb; }
int64_t oracle_tm_extent(const oracle_tm *t) { return t->ub - t->lb; }
int64_t oracle_tm_true_lb(const oracle_tm *t) { return t->true_lb; }
int64_t oracle_tm_true_extent(const oracle_tm *t) {
  return t->true_ub - t->true_lb;
}
int64_t oracle_tm_nsegs(const oracle_tm *t) { return t->n; }
void oracle_tm_seg(const oracle_tm *t, int64_t i, int64_t *disp, int64_t *len) {
  *disp = t->runs[i].disp;
  *len = t->runs[i].len;
}

void oracle_tm_pack(const oracle_tm *t, int64_t incount, const uint8_t *base,
                    uint8_t *out, int64_t *position) {
  const int64_t e = ext(t);
  int64_t p = *position;
  for (int64_t i = 0; i < incount; ++i)
    for (int64_t k = 0; k < t->n; ++k) {
      memcpy(out + p, base + i * e + t->runs[k].disp, (size_t)t->runs[k].len);
      p += t->runs[k].len;
    }
  *position = p;
}

void oracle_tm_unpack(const oracle_tm *t, int64_t outcount, const uint8_t *in,
                      int64_t *position, uint8_t *base) {
  const int64_t e = ext(t);
  int64_t p = *position;
  for (int64_t i = 0; i < outcount; ++i)
    for (int64_t k = 0; k < t->n; ++k) {
      memcpy(base + i * e + t->runs[k].disp, in + p, (size_t)t->runs[k].len);
      p += t->runs[k].len;
    }
  *position = p;
}

/* odometer over (incount, counts[0..ndims-1]) with the last dim fastest */
static void strided_walk(int64_t start, int64_t block, int ndims,
                         const int64_t *counts, const int64_t *strides,
                         int64_t n, int64_t extent, uint8_t *base,
                         uint8_t *packed, int pack) {
  int64_t rows = 1;
  for (int d = 0; d < ndims; ++d) rows *= counts[d];
  int64_t p = 0;
  int64_t *idx = (int64_t *)calloc((size_t)(ndims ? ndims : 1), sizeof(int64_t));
  for (int64_t i = 0; i < n; ++i) {
    for (int d = 0; d < ndims; ++d) idx[d] = 0;
    for (int64_t r = 0; r < rows; ++r) {
      int64_t off = start + i * extent;
      for (int d = 0; d < ndims; ++d) off += idx[d] * strides[d];
      if (pack)
        memcpy(packed + p, base + off, (size_t)block);
      else
        memcpy(base + off, packed + p, (size_t)block);
      p += block;
      for (int d = ndims - 1; d >= 0; --d) {
        if (++idx[d] < counts[d]) break;
        idx[d] = 0;
      }
    }
  }
  free(idx);
}

void oracle_strided_pack(int64_t start, int64_t block, int ndims,
                         const int64_t *counts, const int64_t *strides,
                         int64_t incount, int64_t extent, const uint8_t *base,
                         uint8_t *out) {
  strided_walk(start, block, ndims, counts, strides, incount, extent,
               (uint8_t *)base, out, 1);
}

void oracle_strided_unpack(int64_t start, int64_t block, int ndims,
                           const int64_t *counts, const int64_t *strides,
                           int64_t outcount, int64_t extent, const uint8_t *in,
                           uint8_t *base) {
  strided_walk(start, block, ndims, counts, strides, outcount, extent, base,
               (uint8_t *)in, 0);
}
