/*
 * oracle/recipe.c -- TEST INFRASTRUCTURE ONLY. Recursive-descent parser for the
 * datatype recipe language described in recipe.h.
 */
#include "recipe.h"

#include <ctype.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  const char *s;
  char *err;
  int errlen;
  int failed;
} pstate;

static void fail(pstate *p, const char *msg) {
  if (!p->failed && p->err && p->errlen > 0) {
    snprintf(p->err, (size_t)p->errlen, "%s at '%.20s'", msg, p->s);
  }
  p->failed = 1;
}

static void ws(pstate *p) {
  while (*p->s && isspace((unsigned char)*p->s)) p->s++;
}

static int expect(pstate *p, char c) {
  ws(p);
  if (*p->s != c) {
    char m[32];
    snprintf(m, sizeof m, "expected '%c'", c);
    fail(p, m);
    return 0;
  }
  p->s++;
  return 1;
}

static int64_t integer(pstate *p) {
  ws(p);
  char *end = NULL;
  long long v = strtoll(p->s, &end, 10);
  if (end == p->s) {
    fail(p, "expected integer");
    return 0;
  }
  p->s = end;
  return (int64_t)v;
}

static int ident(pstate *p, char *out, int n) {
  ws(p);
  int i = 0;
  while ((isalnum((unsigned char)*p->s) || *p->s == '_') && i < n - 1) {
    out[i++] = *p->s++;
  }
  out[i] = 0;
  if (!i) fail(p, "expected identifier");
  return i;
}

static int array(pstate *p, int64_t **out) {
  if (!expect(p, '[')) return 0;
  int cap = 8, n = 0;
  int64_t *v = (int64_t *)malloc(sizeof(int64_t) * (size_t)cap);
  ws(p);
  while (*p->s && *p->s != ']') {
    if (n == cap) {
      cap *= 2;
      v = (int64_t *)realloc(v, sizeof(int64_t) * (size_t)cap);
    }
    v[n++] = integer(p);
    if (p->failed) break;
    ws(p);
    if (*p->s == ',') p->s++;
    ws(p);
  }
  expect(p, ']');
  *out = v;
  return n;
}

static rnode *parse_type(pstate *p);

static const struct {
  const char *name;
  int64_t size;
} basics[] = {{"byte", 1},  {"char", 1},  {"short", 2},  {"int", 4},
              {"long", 8},  {"float", 4}, {"double", 8}, {NULL, 0}};

static rnode *parse_type(pstate *p) {
  char id[32];
  if (!ident(p, id, sizeof id)) return NULL;
  rnode *n = (rnode *)calloc(1, sizeof(rnode));
  for (int i = 0; basics[i].name; ++i) {
    if (!strcmp(id, basics[i].name)) {
      n->kind = RK_BASIC;
      snprintf(n->name, sizeof n->name, "%s", id);
      n->size = basics[i].size;
      return n;
    }
  }
  if (!expect(p, '(')) goto bad;
  if (!strcmp(id, "contig")) {
    n->kind = RK_CONTIG;
    n->a[0] = integer(p);
  } else if (!strcmp(id, "vector") || !strcmp(id, "hvector")) {
    n->kind = id[0] == 'v' ? RK_VECTOR : RK_HVECTOR;
    n->a[0] = integer(p);
    expect(p, ',');
    n->a[1] = integer(p);
    expect(p, ',');
    n->a[2] = integer(p);
  } else if (!strcmp(id, "subarray")) {
    n->kind = RK_SUBARRAY;
    ws(p);
    n->order = *p->s;
    if (n->order != 'C' && n->order != 'F') fail(p, "expected C or F");
    p->s++;
    for (int k = 0; k < 3; ++k) {
      expect(p, ',');
      n->narr[k] = array(p, &n->arr[k]);
    }
    if (n->narr[0] != n->narr[1] || n->narr[0] != n->narr[2] || !n->narr[0])
      fail(p, "subarray arrays must have equal nonzero length");
  } else if (!strcmp(id, "resized")) {
    n->kind = RK_RESIZED;
    n->a[0] = integer(p);
    expect(p, ',');
    n->a[1] = integer(p);
  } else if (!strcmp(id, "indexed") || !strcmp(id, "hindexed") || !strcmp(id, "struct")) {
    n->kind = id[0] == 'i' ? RK_INDEXED : id[0] == 'h' ? RK_HINDEXED : RK_STRUCT;
    n->narr[0] = array(p, &n->arr[0]);
    expect(p, ',');
    n->narr[1] = array(p, &n->arr[1]);
    if (n->narr[0] != n->narr[1]) fail(p, "blocklength/displacement mismatch");
  } else if (!strcmp(id, "indexed_block") || !strcmp(id, "hindexed_block")) {
    n->kind = id[0] == 'i' ? RK_INDEXED_BLOCK : RK_HINDEXED_BLOCK;
    n->a[0] = integer(p);
    expect(p, ',');
    n->narr[1] = array(p, &n->arr[1]);
  } else if (!strcmp(id, "dup")) {
    n->kind = RK_DUP;
  } else {
    fail(p, "unknown constructor");
    goto bad;
  }
  if (n->kind != RK_DUP) expect(p, ',');
  if (p->failed) goto bad;
  n->child = parse_type(p);
  if (!n->child) goto bad;
  if (!expect(p, ')')) goto bad;
  return n;
bad:
  recipe_free(n);
  return NULL;
}

rnode *recipe_parse(const char *text, char *err, int errlen) {
  pstate p = {text, err, errlen, 0};
  rnode *n = parse_type(&p);
  if (n) {
    ws(&p);
    if (*p.s) {
      fail(&p, "trailing input");
      recipe_free(n);
      return NULL;
    }
  }
  if (p.failed) {
    recipe_free(n);
    return NULL;
  }
  return n;
}

void recipe_free(rnode *n) {
  if (!n) return;
  recipe_free(n->child);
  for (int k = 0; k < 3; ++k) free(n->arr[k]);
  free(n);
}
