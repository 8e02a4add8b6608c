"""Freeze the reference's public call signatures (the drop-in boundary) as data.

Runs ONLY in the build container (it reads /root/reference as text; nothing is imported or
executed from it). For every public class of src/model.py and every public module-level
function of src/model.py and src/retrieval.py, it records each method's parameters with `ast`:
name, kind (positional / keyword-only / *args / **kwargs) and the default's source text. The
output, `ref_signatures.json`, is what tests/test_signatures_cpu.py compares triad_amd's mirror
against (same names, same order, same defaults; extra trailing optional parameters allowed).

Usage:  python tests/golden/gen_signatures.py
"""
import ast
import json
import os

REF = "/root/reference/src"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ref_signatures.json")
# reference module -> mirror module in triad_amd
MODULES = {"model.py": "triad_amd.model", "retrieval.py": "triad_amd.retrieval"}


def _params(fn: ast.FunctionDef):
    a = fn.args
    out = []
    pos = a.posonlyargs + a.args
    pos_defaults = [None] * (len(pos) - len(a.defaults)) + list(a.defaults)
    for p, d in zip(pos, pos_defaults):
        out.append({"name": p.arg, "kind": "POSITIONAL_OR_KEYWORD",
                    "default": None if d is None else ast.unparse(d)})
    if a.vararg:
        out.append({"name": a.vararg.arg, "kind": "VAR_POSITIONAL", "default": None})
    for p, d in zip(a.kwonlyargs, a.kw_defaults):
        out.append({"name": p.arg, "kind": "KEYWORD_ONLY", "default": None if d is None else ast.unparse(d)})
    if a.kwarg:
        out.append({"name": a.kwarg.arg, "kind": "VAR_KEYWORD", "default": None})
    return out


def _public(name):
    return name == "__init__" or not name.startswith("_")


def main():
    sigs = {}
    for fname, mirror in MODULES.items():
        path = os.path.join(REF, fname)
        tree = ast.parse(open(path).read(), filename=path)
        mod = {"classes": {}, "functions": {}, "source": f"src/{fname}"}
        for node in tree.body:
            if isinstance(node, ast.ClassDef) and _public(node.name):
                meths = {}
                for m in node.body:
                    if isinstance(m, ast.FunctionDef) and _public(m.name):
                        meths[m.name] = {"line": m.lineno, "params": _params(m)}
                mod["classes"][node.name] = {"line": node.lineno, "methods": meths}
            elif isinstance(node, ast.FunctionDef) and _public(node.name):
                mod["functions"][node.name] = {"line": node.lineno, "params": _params(node)}
        sigs[mirror] = mod
    with open(OUT, "w") as f:
        json.dump(sigs, f, indent=1, sort_keys=True)
    print(f"wrote {OUT}")


if __name__ == "__main__":
    main()
