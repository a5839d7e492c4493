/*
 * oracle/gen_golden.c -- TEST INFRASTRUCTURE ONLY. Golden-vector generator.
 *
 * Builds the datatype named by a recipe (recipe.h) with the HOST MPI (MPICH
 * 3.3.2 at /opt/conda in this image), fills the source buffer with the
 * reference's convention src[i] = i & 0xFF (/root/reference/test/
 * pack_unpack.cpp:54-57), and records what the library's own MPI_Pack /
 * MPI_Unpack produce -- the parity target of the north star and the oracle of
 * the reference's test (/root/reference/test/pack_unpack.cpp:61-97).
 *
 * usage: gen_golden '<recipe>' <count> <packed.bin> <unpacked.bin>
 *   stdout: one JSON object with size / lb / extent / true extent / pack size
 *           / final position / buffer geometry
 *   packed.bin  : the packed bytes
 *   unpacked.bin: MPI_Unpack of those bytes into a zeroed buffer of buflen
 * tools/make_golden.py drives it and writes tests/golden/mpich_golden.json.
 */
#include "recipe.h"

#include <mpi.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static MPI_Datatype basic(const char *n) {
  if (!strcmp(n, "byte")) return MPI_BYTE;
  if (!strcmp(n, "char")) return MPI_CHAR;
  if (!strcmp(n, "short")) return MPI_SHORT;
  if (!strcmp(n, "int")) return MPI_INT;
  if (!strcmp(n, "long")) return MPI_LONG;
  if (!strcmp(n, "float")) return MPI_FLOAT;
  if (!strcmp(n, "double")) return MPI_DOUBLE;
  fprintf(stderr, "unknown basic %s\n", n);
  exit(2);
}

static MPI_Datatype build(const rnode *r) {
  if (r->kind == RK_BASIC) return basic(r->name);
  MPI_Datatype c = build(r->child), t = MPI_DATATYPE_NULL;
  switch (r->kind) {
  case RK_DUP:
    MPI_Type_dup(c, &t);
    break;
  case RK_CONTIG:
    MPI_Type_contiguous((int)r->a[0], c, &t);
    break;
  case RK_VECTOR:
    MPI_Type_vector((int)r->a[0], (int)r->a[1], (int)r->a[2], c, &t);
    break;
  case RK_HVECTOR:
    MPI_Type_create_hvector((int)r->a[0], (int)r->a[1], (MPI_Aint)r->a[2], c, &t);
    break;
  case RK_RESIZED:
    MPI_Type_create_resized(c, (MPI_Aint)r->a[0], (MPI_Aint)r->a[1], &t);
    break;
  case RK_SUBARRAY: {
    int nd = r->narr[0];
    int *s = malloc(sizeof(int) * nd), *ss = malloc(sizeof(int) * nd),
        *st = malloc(sizeof(int) * nd);
    for (int i = 0; i < nd; ++i) {
      s[i] = (int)r->arr[0][i];
      ss[i] = (int)r->arr[1][i];
      st[i] = (int)r->arr[2][i];
    }
    MPI_Type_create_subarray(nd, s, ss, st,
                             r->order == 'C' ? MPI_ORDER_C : MPI_ORDER_FORTRAN,
                             c, &t);
    free(s);
    free(ss);
    free(st);
    break;
  }
  case RK_INDEXED:
  case RK_HINDEXED:
  case RK_STRUCT: {
    int n = r->narr[0];
    int *bl = malloc(sizeof(int) * (n ? n : 1));
    int *di = malloc(sizeof(int) * (n ? n : 1));
    MPI_Aint *da = malloc(sizeof(MPI_Aint) * (n ? n : 1));
    for (int i = 0; i < n; ++i) {
      bl[i] = (int)r->arr[0][i];
      di[i] = (int)r->arr[1][i];
      da[i] = (MPI_Aint)r->arr[1][i];
    }
    if (r->kind == RK_INDEXED) {
      MPI_Type_indexed(n, bl, di, c, &t);
    } else if (r->kind == RK_STRUCT) {
      MPI_Datatype *ty = malloc(sizeof(MPI_Datatype) * (n ? n : 1));
      for (int i = 0; i < n; ++i) ty[i] = c;
      MPI_Type_create_struct(n, bl, da, ty, &t);
      free(ty);
    } else
      MPI_Type_create_hindexed(n, bl, da, c, &t);
    free(bl);
    free(di);
    free(da);
    break;
  }
  case RK_INDEXED_BLOCK:
  case RK_HINDEXED_BLOCK: {
    int n = r->narr[1];
    int *di = malloc(sizeof(int) * (n ? n : 1));
    MPI_Aint *da = malloc(sizeof(MPI_Aint) * (n ? n : 1));
    for (int i = 0; i < n; ++i) {
      di[i] = (int)r->arr[1][i];
      da[i] = (MPI_Aint)r->arr[1][i];
    }
    if (r->kind == RK_INDEXED_BLOCK)
      MPI_Type_create_indexed_block(n, (int)r->a[0], di, c, &t);
    else
      MPI_Type_create_hindexed_block(n, (int)r->a[0], da, c, &t);
    free(di);
    free(da);
    break;
  }
  default:
    fprintf(stderr, "bad kind\n");
    exit(2);
  }
  return t;
}

int main(int argc, char **argv) {
  if (argc != 5) {
    fprintf(stderr, "usage: %s RECIPE COUNT PACKED.bin UNPACKED.bin\n", argv[0]);
    return 2;
  }
  MPI_Init(&argc, &argv);
  char err[256] = {0};
  rnode *r = recipe_parse(argv[1], err, sizeof err);
  if (!r) {
    fprintf(stderr, "parse error: %s\n", err);
    return 2;
  }
  const long count = atol(argv[2]);
  MPI_Datatype ty = build(r);
  MPI_Type_commit(&ty);

  int size = 0, packSize = 0;
  MPI_Aint lb, extent, tlb, textent;
  MPI_Type_size(ty, &size);
  MPI_Type_get_extent(ty, &lb, &extent);
  MPI_Type_get_true_extent(ty, &tlb, &textent);
  MPI_Pack_size((int)count, ty, MPI_COMM_WORLD, &packSize);

  /* buffer geometry: `origin` bytes before the address handed to MPI so that
     negative displacements stay inside the allocation */
  long lo = tlb, hi = tlb + textent;
  if (count > 1) {
    long d = (count - 1) * (long)extent;
    if (d < 0) lo += d; else hi += d;
  }
  long origin = lo < 0 ? -lo : 0;
  long buflen = origin + (hi > 0 ? hi : 0);
  if (buflen <= 0) buflen = 1;

  unsigned char *buf = malloc((size_t)buflen);
  for (long i = 0; i < buflen; ++i) buf[i] = (unsigned char)(i & 0xFF);
  unsigned char *packed = calloc((size_t)(packSize > 0 ? packSize : 1), 1);
  int position = 0;
  MPI_Pack(buf + origin, (int)count, ty, packed, packSize, &position,
           MPI_COMM_WORLD);

  unsigned char *unpacked = calloc((size_t)buflen, 1);
  int upos = 0;
  MPI_Unpack(packed, position, &upos, unpacked + origin, (int)count, ty,
             MPI_COMM_WORLD);

  FILE *f = fopen(argv[3], "wb");
  fwrite(packed, 1, (size_t)position, f);
  fclose(f);
  f = fopen(argv[4], "wb");
  fwrite(unpacked, 1, (size_t)buflen, f);
  fclose(f);

  char ver[MPI_MAX_LIBRARY_VERSION_STRING];
  int vlen = 0;
  MPI_Get_library_version(ver, &vlen);
  char *nl = strchr(ver, '\n');
  if (nl) *nl = 0;
  for (char *c = ver; *c; ++c)
    if (*c == '\t' || *c == '"' || *c == '\\') *c = ' ';

  printf("{\"size\": %d, \"lb\": %ld, \"extent\": %ld, \"true_lb\": %ld, "
         "\"true_extent\": %ld, \"pack_size\": %d, \"position\": %d, "
         "\"unpack_position\": %d, \"origin\": %ld, \"buflen\": %ld, "
         "\"library\": \"%s\"}\n",
         size, (long)lb, (long)extent, (long)tlb, (long)textent, packSize,
         position, upos, origin, buflen, ver);

  if (r->kind != RK_BASIC) MPI_Type_free(&ty);
  recipe_free(r);
  free(buf);
  free(packed);
  free(unpacked);
  MPI_Finalize();
  return 0;
}
