#!/usr/bin/env python
"""Report global names a Python file reads but never binds (no linter is
installed in the image): a function body that refers to a name no module-level
statement assigns, imports or defines, and that is not a builtin, fails only
when that line runs -- on the GPU box, at round end.

    python scripts/undefined_names.py bench.py tencent_recommendation_2025_amd/*.py
"""
import builtins
import sys
import symtable

_IMPLICIT = {'__file__', '__name__', '__doc__', '__spec__', '__loader__', '__package__', '__builtins__'}


def undefined(path):
    """[(scope name, name)] for every unbound global reference in one file."""
    with open(path) as f:
        top = symtable.symtable(f.read(), path, 'exec')
    bound = {s.get_name() for s in top.get_symbols() if s.is_assigned() or s.is_imported()}
    # `global x` in a function that assigns x binds it at module level as well
    stack, out = [top], []
    while stack:
        t = stack.pop()
        for s in t.get_symbols():
            if s.is_declared_global() and s.is_assigned():
                bound.add(s.get_name())
        stack.extend(t.get_children())
    stack = [top]
    while stack:
        t = stack.pop()
        for s in t.get_symbols():
            n = s.get_name()
            if not s.is_referenced() or n in bound or n in _IMPLICIT or hasattr(builtins, n):
                continue
            if t is top or s.is_global():
                out.append((t.get_name(), n))
        stack.extend(t.get_children())
    return out


def main(paths):
    bad = [(p, scope, n) for p in paths for scope, n in undefined(p)]
    for p, scope, n in bad:
        print(f'{p}: {scope}: {n}')
    return 1 if bad else 0


if __name__ == '__main__':
    sys.exit(main(sys.argv[1:]))
