"""Seeded random MPI datatype recipes (grammar: oracle/recipe.h) for the
parity fuzz: the constructors the reference decodes
(/root/reference/src/internal/types.cpp: vector, hvector, subarray, contiguous,
plus the resized / dup / indexed / struct forms TEMPI canonicalises or hands to the
library), nested up to three deep, with negative strides, resized extents,
misaligned blocks and every named element size. Objects stay small (at most
a few MiB per element) so hundreds of cases run in seconds."""
import random

ELEMS = [("byte", 1), ("char", 1), ("short", 2), ("int", 4), ("float", 4), ("long", 8), ("double", 8)]


def _elem(rng):
    return rng.choice(ELEMS)


def _leaf(rng, budget):
    """a 1-level strided type over a named element: (recipe, elem size, span in bytes)"""
    name, es = _elem(rng)
    k = rng.randrange(6)
    if k == 0:  # vector, possibly negative stride
        n = rng.randrange(1, max(2, min(600, budget // 64)))
        bl = rng.choice([1, 2, 3, 4, 5, 8, 13, 16, 64])
        st = bl + rng.choice([0, 1, 3, 8, 17, bl])
        if rng.random() < 0.2:
            st = -st
        return f"vector({n},{bl},{st},{name})", es, (n * abs(st) + bl) * es
    if k == 1:  # hvector of contiguous rows (byte stride, any alignment)
        n = rng.randrange(1, max(2, min(600, budget // 64)))
        bl = rng.choice([1, 2, 3, 7, 8, 12, 24, 31, 64, 100, 256])
        st = bl * es + rng.choice([0, 1, 5, 16, 64, 511])
        if rng.random() < 0.15:
            st = -st
        return f"hvector({n},1,{st},contig({bl},{name}))", es, n * abs(st) + bl * es
    if k == 2:  # 2-D subarray, C or Fortran order
        rows, cols = rng.randrange(1, 200), rng.choice([1, 2, 3, 8, 24, 64, 100])
        R, C = rows + rng.randrange(0, 6), cols + rng.choice([0, 1, 13, 16])
        order = rng.choice("CF")
        if order == "C":
            return (f"subarray(C,[{R},{C}],[{rows},{cols}],[{rng.randrange(0, R - rows + 1)},"
                    f"{rng.randrange(0, C - cols + 1)}],{name})", es, R * C * es)
        return (f"subarray(F,[{C},{R}],[{cols},{rows}],[{rng.randrange(0, C - cols + 1)},"
                f"{rng.randrange(0, R - rows + 1)}],{name})", es, R * C * es)
    if k == 3:  # 3-D subarray
        z, y, x = rng.randrange(1, 20), rng.randrange(1, 20), rng.choice([1, 3, 8, 24, 64])
        Z, Y, X = z + rng.randrange(0, 4), y + rng.randrange(0, 4), x + rng.choice([0, 3, 16])
        return (f"subarray(C,[{Z},{Y},{X}],[{z},{y},{x}],[{rng.randrange(0, Z - z + 1)},"
                f"{rng.randrange(0, Y - y + 1)},{rng.randrange(0, X - x + 1)}],{name})", es, Z * Y * X * es)
    if k == 4:  # regular hindexed_block / indexed_block / struct (canonicalises to a vector)
        n, bl = rng.randrange(1, 100), rng.choice([1, 2, 4, 9])
        st = bl + rng.choice([0, 2, 5])
        u = rng.random()
        if u < 0.5:
            return f"indexed_block({bl},[{','.join(str(i * st) for i in range(n))}],{name})", es, n * st * es
        disps = ','.join(str(i * st * es) for i in range(n))
        if u < 0.75:
            return f"hindexed_block({bl},[{disps}],{name})", es, n * st * es
        return f"struct([{','.join([str(bl)] * n)}],[{disps}],{name})", es, n * st * es
    # contiguous run
    n = rng.randrange(1, 2000)
    return f"contig({n},{name})", es, n * es


def recipe(rng, budget=1 << 20):
    """one random recipe: a leaf, optionally wrapped once or twice"""
    r, es, span = _leaf(rng, budget)
    for _ in range(rng.choice([0, 0, 1, 1, 2])):
        w = rng.randrange(5)
        if w == 0 and span < budget:  # outer hvector of the whole thing
            n = rng.randrange(1, max(2, min(40, budget // max(span, 1))))
            st = span + rng.choice([0, 8, 100, 4096])
            if rng.random() < 0.2:
                st = -st
            r, span = f"hvector({n},1,{st},{r})", n * abs(st) + span
        elif w == 1 and span < budget:  # vector of the thing (stride in its extents)
            n = rng.randrange(1, max(2, min(20, budget // max(span, 1))))
            r, span = f"vector({n},1,{rng.choice([1, 2, 3])},{r})", n * 3 * span
        elif w == 2:  # resized: a larger extent (and sometimes a shifted lb)
            lb = rng.choice([0, 0, -es * rng.randrange(1, 8), es * rng.randrange(1, 8)])
            r, span = f"resized({lb},{span + rng.choice([0, es, 64, 4096])},{r})", span + 4096 + 64
        elif w == 3:
            r = f"dup({r})"
        elif span < budget:  # contiguous of the thing
            n = rng.randrange(1, 4)
            r, span = f"contig({n},{r})", n * span + 4096
    return r


def cases(seed, n, budget=1 << 20):
    """n (recipe, count, shift, position) tuples: count 1-4, the object's origin
    misaligned by `shift` bytes, packing at byte `position` of the output"""
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        out.append((recipe(rng, budget), rng.choice([1, 1, 2, 3, 4]), rng.choice([0, 0, 1, 3, 8, 13]),
                    rng.choice([0, 0, 1, 7, 16, 100])))
    return out
