/*
 * oracle/recipe.h -- TEST INFRASTRUCTURE ONLY (never linked into libtempi).
 *
 * A tiny text language that names an MPI derived datatype by its constructor
 * tree, so that one case list drives three independent builders:
 *   - oracle/typemap.c   : CPU restatement of the MPI type map (the oracle),
 *   - oracle/gen_golden.c: the same type built with the host MPI (MPICH 3.3.2)
 *                          whose MPI_Pack output becomes tests/golden/,
 *   - tests/typezoo.py   : the same type built through libtempi on the GPU box.
 *
 * Grammar (whitespace ignored, integers may be negative):
 *   T := BASIC
 *      | contig(n, T)                              MPI_Type_contiguous
 *      | vector(n, bl, stride, T)                  MPI_Type_vector
 *      | hvector(n, bl, stride_bytes, T)           MPI_Type_create_hvector
 *      | subarray(C|F, [sizes], [subsizes], [starts], T)
 *      | resized(lb, extent, T)                    MPI_Type_create_resized
 *      | indexed([bl..], [disp..], T)              MPI_Type_indexed
 *      | hindexed([bl..], [disp_bytes..], T)       MPI_Type_create_hindexed
 *      | indexed_block(bl, [disp..], T)            MPI_Type_create_indexed_block
 *      | hindexed_block(bl, [disp_bytes..], T)     MPI_Type_create_hindexed_block
 *      | dup(T)                                    MPI_Type_dup
 *      | struct([bl..], [disp_bytes..], T)         MPI_Type_create_struct, T for
 *                                                  every block (the reference
 *                                                  refuses struct, types.cpp:230)
 *   BASIC := byte | char | short | int | long | float | double
 *
 * The constructors are the ones the reference decodes in
 * /root/reference/src/internal/types.cpp:42-344 (plus the ones it refuses,
 * which TEMPI must hand to the library) and the ones its type zoo uses in
 * /root/reference/support/type.cpp:3-308.
 */
#ifndef TEMPI_ORACLE_RECIPE_H
#define TEMPI_ORACLE_RECIPE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum rkind {
  RK_BASIC = 0,
  RK_CONTIG,
  RK_VECTOR,
  RK_HVECTOR,
  RK_SUBARRAY,
  RK_RESIZED,
  RK_INDEXED,
  RK_HINDEXED,
  RK_INDEXED_BLOCK,
  RK_HINDEXED_BLOCK,
  RK_DUP,
  RK_STRUCT /* one child type for every block: the type map of HINDEXED */
};

typedef struct rnode {
  int kind;
  char name[16];   /* BASIC: type name */
  int64_t size;    /* BASIC: size in bytes */
  int64_t a[3];    /* scalar args in order of the grammar */
  int narr[3];     /* lengths of array args */
  int64_t *arr[3]; /* array args in order of the grammar */
  char order;      /* subarray: 'C' or 'F' */
  struct rnode *child;
} rnode;

/* parse a recipe; returns NULL and fills err (if non-null) on failure */
rnode *recipe_parse(const char *text, char *err, int errlen);
void recipe_free(rnode *n);

#ifdef __cplusplus
}
#endif
#endif
