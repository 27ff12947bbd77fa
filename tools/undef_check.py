"""Undefined global names in Python modules (no linter in this image).

usage: python tools/undef_check.py FILE.py [...]

Walks every scope with `symtable`: a name a function reads as global (or as
free from an enclosing scope that never binds it) must be bound at module
level or be a builtin.  Catches the NameErrors of code paths the CPU suite
cannot run (bench.py's GPU legs).  Exit 1 and one line per finding."""
import builtins
import symtable
import sys


def check(path):
    src = open(path).read()
    top = symtable.symtable(src, path, "exec")
    module_names = {s.get_name() for s in top.get_symbols()
                    if s.is_assigned() or s.is_imported() or s.is_namespace()}
    known = module_names | set(dir(builtins)) | {"__file__", "__name__", "__doc__"}
    bad = []

    def walk(t):
        for s in t.get_symbols():
            if t.get_type() != "module" and s.is_global() and not s.is_declared_global():
                if s.get_name() not in known:
                    bad.append(f"{path}:{t.get_lineno()}: {t.get_name()}: undefined {s.get_name()}")
        for c in t.get_children():
            walk(c)
    walk(top)
    return bad


if __name__ == "__main__":
    out = [b for p in sys.argv[1:] for b in check(p)]
    print("\n".join(out))
    sys.exit(1 if out else 0)
