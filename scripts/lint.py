#!/usr/bin/env python
"""Dependency-free lint for this repository (the image ships no flake8/ruff/
clang-format).  Mirrors the reference's pre-commit intent (SURVEY.md R19:
isort/black/flake8/cpplint/shellcheck) with checks that need only the stdlib:

Python: parses (ast), no unused imports (names never referenced; ``__init__``
re-exports and ``# noqa`` lines exempt), no wildcard imports, no bare
``except:``, lines <= 120 columns, no tabs / trailing whitespace.
C++/HIP: lines <= 120 columns, no tabs / trailing whitespace, and the
MI355X-only rules of this project: no CUDA headers, no ``__HIP_PLATFORM_*``
dual paths, no hipify markers.
Shell: ``set -e``/``set -u`` style guard present in GPU scripts.

Exit status 1 with one ``path:line: message`` per finding.
"""
from __future__ import annotations

import ast
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SKIP_DIRS = {".git", "gpurun_out", "__pycache__", "lib", "profiles", ".pytest_cache", "abtmp"}  # abtmp: A/B worktrees
MAXLEN = 120
CXX_BANNED = [
    (re.compile(r"#\s*include\s*[<\"]cuda"), "CUDA header in a gfx950-only source"),
    (re.compile(r"__HIP_PLATFORM_(NVIDIA|NVCC|AMD)__"), "platform dual path (write CDNA4 code directly)"),
    (re.compile(r"hipify", re.I), "hipify output"),
]


def _files(exts):
    for d, dirs, files in os.walk(ROOT):
        dirs[:] = [x for x in dirs if x not in SKIP_DIRS]
        for f in files:
            if f.endswith(exts):
                yield os.path.join(d, f)


def _text_checks(path, lines, out, maxlen=MAXLEN):
    for i, ln in enumerate(lines, 1):
        s = ln.rstrip("\n")
        if len(s) > maxlen:
            out.append(f"{path}:{i}: line longer than {maxlen} ({len(s)})")
        if "\t" in s:
            out.append(f"{path}:{i}: tab character")
        if s != s.rstrip():
            out.append(f"{path}:{i}: trailing whitespace")


class _Names(ast.NodeVisitor):
    def __init__(self):
        self.used = set()

    def visit_Name(self, n):
        self.used.add(n.id)

    def visit_Attribute(self, n):
        root = n
        while isinstance(root, ast.Attribute):
            root = root.value
        if isinstance(root, ast.Name):
            self.used.add(root.id)
        self.generic_visit(n)


def lint_python(path, out):
    src = open(path, encoding="utf-8").read()
    lines = src.splitlines(True)
    _text_checks(path, lines, out)
    try:
        tree = ast.parse(src, path)
    except SyntaxError as e:
        out.append(f"{path}:{e.lineno}: syntax error: {e.msg}")
        return
    v = _Names()
    v.visit(tree)
    # names used only inside string annotations / __all__
    strings = " ".join(n.value for n in ast.walk(tree) if isinstance(n, ast.Constant) and isinstance(n.value, str))
    is_init = os.path.basename(path) == "__init__.py"
    for node in ast.walk(tree):
        if isinstance(node, ast.ExceptHandler) and node.type is None:
            out.append(f"{path}:{node.lineno}: bare except")
        if isinstance(node, (ast.Import, ast.ImportFrom)):
            if isinstance(node, ast.ImportFrom) and any(a.name == "*" for a in node.names):
                out.append(f"{path}:{node.lineno}: wildcard import")
                continue
            if is_init or "noqa" in lines[node.lineno - 1] or (isinstance(node, ast.ImportFrom)
                                                               and node.module == "__future__"):
                continue
            for a in node.names:
                name = (a.asname or a.name).split(".")[0]
                if name not in v.used and not re.search(rf"\b{re.escape(name)}\b", strings):
                    out.append(f"{path}:{node.lineno}: unused import '{a.asname or a.name}'")


def lint_cxx(path, out):
    lines = open(path, encoding="utf-8").read().splitlines(True)
    _text_checks(path, lines, out)
    for i, ln in enumerate(lines, 1):
        for pat, msg in CXX_BANNED:
            if pat.search(ln) and "lint: allow" not in ln:
                out.append(f"{path}:{i}: {msg}")


def lint_shell(path, out):
    src = open(path, encoding="utf-8").read()
    _text_checks(path, src.splitlines(True), out, maxlen=200)  # long GPU command lines read better unwrapped
    if "gpurun" not in path and re.search(r"timeout\s+-k", src) and not re.search(r"set -[a-z]*[eu]", src):
        out.append(f"{path}:1: GPU script without 'set -e'/'set -u'")


def main(argv=None) -> int:
    out: list[str] = []
    for p in _files((".py",)):
        lint_python(p, out)
    for p in _files((".hip", ".cpp", ".h", ".hpp")):
        lint_cxx(p, out)
    for p in _files((".sh",)):
        lint_shell(p, out)
    for line in out:
        print(os.path.relpath(line, ROOT) if line.startswith(ROOT) else line)
    print(f"lint: {len(out)} finding(s)", file=sys.stderr)
    return 1 if out else 0


if __name__ == "__main__":
    sys.exit(main())
