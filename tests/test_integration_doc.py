"""CPU: the Rust binding INTEGRATION.md §2 shows a maintainer (the `extern "C"`
block over libbfrs.so) declares only functions include/bfrs.h declares, with
the same number of parameters and the same pointer/scalar shape per
parameter, so the documented binding cannot drift from the C-ABI."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rust_decls():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    block = text[text.index('extern "C" {'):]
    block = block[:block.index("\n}\n")]
    decls = {}
    for m in re.finditer(r"pub fn (bfrs_\w+)\((.*?)\)\s*(?:->\s*[\w:* ]+)?;", block, re.S):
        params = [p.strip() for p in m.group(2).replace("\n", " ").split(",") if p.strip()]
        decls[m.group(1)] = ["*" in p.split(":", 1)[1] for p in params]
    return decls


def _c_decls():
    text = open(os.path.join(ROOT, "include", "bfrs.h")).read()
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    text = re.sub(r"//[^\n]*", " ", text)
    decls = {}
    for m in re.finditer(r"\b(bfrs_\w+)\s*\(([^;{]*?)\)\s*;", text, re.S):
        params = [p.strip() for p in m.group(2).split(",") if p.strip() and p.strip() != "void"]
        decls[m.group(1)] = ["*" in p or "[" in p for p in params]
    return decls


def test_rust_binding_matches_header():
    rust, c = _rust_decls(), _c_decls()
    assert len(rust) >= 30, sorted(rust)
    missing = sorted(set(rust) - set(c))
    assert not missing, f"INTEGRATION.md binds functions bfrs.h lacks: {missing}"
    for name, shape in rust.items():
        assert len(shape) == len(c[name]), (name, len(shape), len(c[name]))
        assert shape == c[name], (name, shape, c[name])
