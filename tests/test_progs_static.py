"""Every script a GPU test launches must at least be able to start. The MPI
programs under tests/mpi_progs/ mostly need a GPU, so the CPU suite cannot run
all of them; this is a pyflakes-style check (pyflakes is not in the image)
that every name a script reads is bound somewhere it can be seen -- at module
level, before the statement that reads it. The other Python files of the
repository (tools/, tempi_amd/, oracle/, tests/) are held to the same check.
Round 3's fuzz.py read `modes` two lines before assigning it, and that one
NameError hid ~290 GPU tests behind pytest -x."""
import ast
import builtins
import os

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
PROGS = sorted(os.path.join(ROOT, "tests", "mpi_progs", f)
               for f in os.listdir(os.path.join(ROOT, "tests", "mpi_progs")) if f.endswith(".py"))
SCRIPTS = PROGS + [os.path.join(ROOT, f) for f in ("bench.py", "__graft_entry__.py")] + sorted(
    os.path.join(ROOT, d, f) for d in ("tools", "tempi_amd", "oracle", "tests")
    for f in os.listdir(os.path.join(ROOT, d)) if f.endswith(".py"))
BUILTINS = set(dir(builtins)) | {"__file__", "__name__", "__doc__", "__spec__", "__builtins__"}


def _targets(node):
    """names a target expression binds"""
    if isinstance(node, ast.Name):
        return {node.id}
    if isinstance(node, (ast.Tuple, ast.List)):
        return set().union(*[_targets(e) for e in node.elts]) if node.elts else set()
    if isinstance(node, ast.Starred):
        return _targets(node.value)
    return set()


def _binds(stmt):
    """names a statement binds in the scope it runs in (not inside nested defs)"""
    out = set()
    for n in _walk_scope(stmt):
        if isinstance(n, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)):
            out.add(n.name)
        elif isinstance(n, (ast.Import, ast.ImportFrom)):
            for a in n.names:
                out.add((a.asname or a.name).split(".")[0])
        elif isinstance(n, ast.Name) and isinstance(n.ctx, (ast.Store, ast.Del)):
            out.add(n.id)
        elif isinstance(n, ast.ExceptHandler) and n.name:
            out.add(n.name)
        elif isinstance(n, (ast.Global, ast.Nonlocal)):
            out.update(n.names)
        elif isinstance(n, ast.NamedExpr):
            out |= _targets(n.target)
    return out


def _walk_scope(node):
    """ast.walk that does not descend into nested function/class/lambda/comprehension scopes
    (but does yield the nested def itself, its decorators and default values)"""
    todo = [node]
    while todo:
        n = todo.pop()
        yield n
        if isinstance(n, (ast.FunctionDef, ast.AsyncFunctionDef)):
            todo.extend(n.decorator_list)
            todo.extend(n.args.defaults + [d for d in n.args.kw_defaults if d is not None])
            continue
        if isinstance(n, ast.ClassDef):
            todo.extend(n.decorator_list + n.bases)
            continue
        if isinstance(n, (ast.Lambda, ast.ListComp, ast.SetComp, ast.DictComp, ast.GeneratorExp)):
            continue
        todo.extend(ast.iter_child_nodes(n))


def _scope_locals(fn):
    args = fn.args
    names = {a.arg for a in args.posonlyargs + args.args + args.kwonlyargs}
    names |= {a.arg for a in (args.vararg, args.kwarg) if a is not None}
    if isinstance(fn, ast.Lambda):
        return names
    for s in fn.body:
        names |= _binds(s)
    return names


def _comp_locals(c):
    out = set()
    for g in c.generators:
        out |= _targets(g.target)
    return out


def _loads(node):
    """(name, lineno) read directly in this scope, plus the nested scopes to check later"""
    loads, nested = [], []
    for n in _walk_scope(node):
        if isinstance(n, ast.Name) and isinstance(n.ctx, ast.Load):
            loads.append((n.id, n.lineno))
        elif n is not node and isinstance(n, (ast.FunctionDef, ast.AsyncFunctionDef, ast.Lambda, ast.ListComp,
                                              ast.SetComp, ast.DictComp, ast.GeneratorExp, ast.ClassDef)):
            nested.append(n)
    return loads, nested


def _check_nested(n, visible, errs):
    """deferred or inner scopes: every name read must be bound in the scope,
    an enclosing one, the module (anywhere) or builtins"""
    if isinstance(n, ast.ClassDef):
        inner = set()
        for s in n.body:
            inner |= _binds(s)
        body = n.body
    elif isinstance(n, (ast.ListComp, ast.SetComp, ast.DictComp, ast.GeneratorExp)):
        inner = _comp_locals(n)
        body = [n.elt] if not isinstance(n, ast.DictComp) else [n.key, n.value]
        body = body + [g.iter for g in n.generators[1:]] + [i for g in n.generators for i in g.ifs]
        # (the first generator's iterable is evaluated in the enclosing scope)
        errs.extend(_unbound(n.generators[0].iter, visible))
        seen = visible | inner
        for b in body:
            errs.extend(_unbound(b, seen))
        return
    else:
        inner = _scope_locals(n)
        body = n.body if isinstance(n.body, list) else [n.body]
    seen = visible | inner
    for b in body:
        errs.extend(_unbound(b, seen))


def _unbound(node, visible):
    errs = []
    loads, nested = _loads(node)
    for name, line in loads:
        if name not in visible and name not in BUILTINS:
            errs.append(f"line {line}: {name!r} is not bound")
    for n in nested:
        _check_nested(n, visible, errs)
    return errs


def check_script(path):
    tree = ast.parse(open(path).read(), path)
    module_all = set()
    for s in tree.body:
        module_all |= _binds(s)
    errs, bound = [], set()

    def visit(stmts):
        for s in stmts:
            # names read by this statement's own (module-time) expressions must
            # be bound by an earlier statement, or by this one's own loop
            # target / with-item / except name before the body runs
            pre = set()
            if isinstance(s, (ast.For, ast.AsyncFor)):
                pre = _targets(s.target)
            if isinstance(s, (ast.With, ast.AsyncWith)):
                for it in s.items:
                    if it.optional_vars is not None:
                        pre |= _targets(it.optional_vars)
            if isinstance(s, (ast.If, ast.For, ast.AsyncFor, ast.While, ast.With, ast.AsyncWith, ast.Try)):
                heads = {ast.If: lambda x: [x.test], ast.While: lambda x: [x.test],
                         ast.For: lambda x: [x.iter], ast.AsyncFor: lambda x: [x.iter],
                         ast.With: lambda x: [i.context_expr for i in x.items],
                         ast.AsyncWith: lambda x: [i.context_expr for i in x.items],
                         ast.Try: lambda x: []}[type(s)](s)
                for h in heads:
                    errs.extend(_unbound(h, bound))
                bound.update(pre)
                for block in ("body", "orelse", "finalbody"):
                    visit(getattr(s, block, []))
                for h in getattr(s, "handlers", []):
                    if h.type is not None:
                        errs.extend(_unbound(h.type, bound))
                    if h.name:
                        bound.add(h.name)
                    visit(h.body)
                continue
            if isinstance(s, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)):
                # decorators/defaults/bases run now; the body later, seeing the whole module
                for d in s.decorator_list:
                    errs.extend(_unbound(d, bound))
                if isinstance(s, ast.ClassDef):
                    for b in s.bases:
                        errs.extend(_unbound(b, bound))
                    _check_nested(s, bound | module_all, errs)
                else:
                    for d in s.args.defaults + [d for d in s.args.kw_defaults if d is not None]:
                        errs.extend(_unbound(d, bound))
                    _check_nested(s, module_all | {s.name}, errs)
                bound.add(s.name)
                continue
            for name, line in _loads(s)[0]:
                if name not in bound and name not in BUILTINS:
                    errs.append(f"line {line}: {name!r} read before any module-level binding")
            for n in _loads(s)[1]:
                # comprehensions and lambdas at module level: run now (comprehension) or
                # later (lambda); checked against the whole module either way, except the
                # comprehension's first iterable, which must already be bound
                if isinstance(n, (ast.ListComp, ast.SetComp, ast.DictComp, ast.GeneratorExp)):
                    errs.extend(_unbound(n.generators[0].iter, bound))
                    _check_nested(n, bound | module_all, errs)
                else:
                    _check_nested(n, module_all, errs)
            bound.update(_binds(s))

    visit(tree.body)
    return sorted(set(errs))


@pytest.mark.parametrize("path", SCRIPTS, ids=[os.path.relpath(p, ROOT) for p in SCRIPTS])
def test_script_names_are_bound(path):
    errs = check_script(path)
    assert not errs, f"{os.path.relpath(path, ROOT)}:\n" + "\n".join(errs)


def test_checker_catches_use_before_assign(tmp_path):
    """the checker finds round 3's fuzz.py bug (and passes the fixed form)"""
    bad = tmp_path / "bad.py"
    bad.write_text("import sys\nif modes:\n    pass\nmodes = '--modes' in sys.argv\n")
    assert any("'modes'" in e for e in check_script(str(bad)))
    good = tmp_path / "good.py"
    good.write_text("import sys\nmodes = '--modes' in sys.argv\nif modes:\n    pass\n"
                    "def f(a):\n    return [a + x for x in range(3)] + [later]\nlater = 1\n")
    assert check_script(str(good)) == []
    typo = tmp_path / "typo.py"
    typo.write_text("def f(a):\n    return a + undefined_thing\n")
    assert any("undefined_thing" in e for e in check_script(str(typo)))
