"""Build MPI datatypes from recipe strings (grammar: oracle/recipe.h) through
libtempi.so, mirroring /root/reference/support/type.cpp's factories.
"""
import re

_TOK = re.compile(r"\s*(?:(-?\d+)|([A-Za-z_][A-Za-z_0-9]*)|(.))")

BASIC = {"byte": "BYTE", "char": "CHAR", "short": "SHORT", "int": "INT", "long": "LONG",
         "float": "FLOAT", "double": "DOUBLE"}


def _tokens(s):
    pos = 0
    out = []
    while pos < len(s):
        m = _TOK.match(s, pos)
        if not m or m.end() == pos:
            break
        pos = m.end()
        if m.group(1) is not None:
            out.append(int(m.group(1)))
        elif m.group(2) is not None:
            out.append(m.group(2))
        elif m.group(3) is not None and not m.group(3).isspace():
            out.append(m.group(3))
    return out


def parse(recipe):
    """-> nested tuples (kind, args..., child)"""
    toks = _tokens(recipe)
    i = 0

    def expect(t):
        nonlocal i
        assert toks[i] == t, f"expected {t!r} at {toks[i:i+5]} in {recipe!r}"
        i += 1

    def arr():
        nonlocal i
        expect("[")
        v = []
        while toks[i] != "]":
            v.append(toks[i])
            i += 1
            if toks[i] == ",":
                i += 1
        expect("]")
        return v

    def typ():
        nonlocal i
        name = toks[i]
        i += 1
        if name in BASIC:
            return ("basic", name)
        expect("(")
        if name == "contig":
            n = toks[i]; i += 1
            args = (n,)
        elif name in ("vector", "hvector"):
            a = toks[i]; expect_comma(); b = toks[i]; expect_comma(); c = toks[i]; i += 1
            args = (a, b, c)
        elif name == "subarray":
            order = toks[i]; i += 1
            expect(","); s = arr(); expect(","); ss = arr(); expect(","); st = arr()
            args = (order, s, ss, st)
        elif name == "resized":
            a = toks[i]; expect_comma(); b = toks[i]; i += 1
            args = (a, b)
        elif name in ("indexed", "hindexed", "struct"):
            a = arr(); expect(","); b = arr()
            args = (a, b)
        elif name in ("indexed_block", "hindexed_block"):
            a = toks[i]; i += 1; expect(","); b = arr()
            args = (a, b)
        elif name == "dup":
            args = ()
        else:
            raise ValueError(name)
        if name != "dup":
            expect(",")
        child = typ()
        expect(")")
        return (name,) + args + (child,)

    def expect_comma():
        nonlocal i
        i += 1
        expect(",")

    t = typ()
    assert i == len(toks), f"trailing tokens in {recipe!r}"
    return t


def build(mpi, recipe, commit=True):
    """Create (and commit) the datatype; returns (handle, [intermediate handles])."""
    temps = []

    def mk(node):
        kind = node[0]
        if kind == "basic":
            return getattr(mpi, BASIC[node[1]])
        child = mk(node[-1])
        if kind == "contig":
            t = mpi.Type_contiguous(node[1], child)
        elif kind == "vector":
            t = mpi.Type_vector(node[1], node[2], node[3], child)
        elif kind == "hvector":
            t = mpi.Type_create_hvector(node[1], node[2], node[3], child)
        elif kind == "subarray":
            order = mpi.ORDER_C if node[1] == "C" else mpi.ORDER_FORTRAN
            t = mpi.Type_create_subarray(node[2], node[3], node[4], order, child)
        elif kind == "resized":
            t = mpi.Type_create_resized(child, node[1], node[2])
        elif kind == "indexed":
            t = mpi.Type_indexed(node[1], node[2], child)
        elif kind == "hindexed":
            t = mpi.Type_create_hindexed(node[1], node[2], child)
        elif kind == "struct":
            t = mpi.Type_create_struct(node[1], node[2], [child] * len(node[1]))
        elif kind == "indexed_block":
            t = mpi.Type_create_indexed_block(node[1], node[2], child)
        elif kind == "hindexed_block":
            t = mpi.Type_create_hindexed_block(node[1], node[2], child)
        elif kind == "dup":
            t = mpi.Type_dup(child)
        else:
            raise ValueError(kind)
        temps.append(t)
        return t

    t = mk(parse(recipe))
    is_basic = not temps
    if temps:
        temps.pop()  # the result itself
    if commit and not is_basic:
        t = mpi.Type_commit(t)
    return t, temps, is_basic


def free(mpi, t, temps, is_basic):
    for x in temps:
        mpi.Type_free(x)
    if not is_basic:
        mpi.Type_free(t)
