"""Stdlib-only lint for the Python sources (flake8 is not installed in this image; the
configuration for it lives in tox.ini and mirrors the reference's /root/reference/tox.ini:1-3 and
.travis.yml:51).

Checks (flake8 code in brackets): syntax errors [E999], lines longer than ``max-line-length``
[E501], tab indentation [W191], trailing whitespace [W291], unused module-level imports [F401]
and ``import *`` [F403]. ``# noqa`` on a line silences it, as with flake8.

    python tools/lint.py [paths...]     (default: the package, AlphaGo/, interface/, tests/,
                                         benchmarks/, tools/, bench.py)
"""
import ast
import configparser
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT = ["rocalphago_amd", "AlphaGo", "interface", "tests", "benchmarks", "tools", "bench.py",
           "__graft_entry__.py"]


def _config():
    cp = configparser.ConfigParser()
    cp.read(os.path.join(ROOT, "tox.ini"))
    sec = cp["flake8"] if cp.has_section("flake8") else {}
    maxlen = int(sec.get("max-line-length", 100))
    excl = [e.strip() for e in sec.get("exclude", "").split(",") if e.strip()]
    return maxlen, excl


def _files(paths, excl):
    for p in paths:
        p = os.path.join(ROOT, p)
        if os.path.isfile(p):
            yield p
            continue
        for d, dirs, fs in os.walk(p):
            dirs[:] = [x for x in dirs if x != "__pycache__" and
                       not any(os.path.relpath(os.path.join(d, x), ROOT).startswith(e)
                               for e in excl)]
            for f in sorted(fs):
                if f.endswith(".py"):
                    yield os.path.join(d, f)


def _unused_imports(tree, lines):
    imported = {}
    for node in tree.body:
        if isinstance(node, (ast.Import, ast.ImportFrom)):
            if isinstance(node, ast.ImportFrom) and node.module == "__future__":
                continue
            for a in node.names:
                if a.name == "*":
                    yield node.lineno, "F403 'from %s import *' used" % node.module
                    continue
                name = (a.asname or a.name).split(".")[0]
                imported[name] = node.lineno
    if not imported:
        return
    used = set()
    for node in ast.walk(tree):
        if isinstance(node, ast.Name):
            used.add(node.id)
        elif isinstance(node, ast.Attribute):
            base = node
            while isinstance(base, ast.Attribute):
                base = base.value
            if isinstance(base, ast.Name):
                used.add(base.id)
    exported = set()
    for node in tree.body:  # __all__ = [...] re-exports
        if isinstance(node, ast.Assign) and any(getattr(t, "id", None) == "__all__"
                                                for t in node.targets):
            try:
                exported |= set(ast.literal_eval(node.value))
            except ValueError:
                pass
    for name, ln in imported.items():
        if name not in used and name not in exported:
            yield ln, "F401 '%s' imported but unused" % name


def lint_file(path, maxlen):
    errs = []
    src = open(path, encoding="utf-8").read()
    lines = src.splitlines()
    try:
        tree = ast.parse(src, path)
    except SyntaxError as e:
        return [(e.lineno or 0, "E999 SyntaxError: %s" % e.msg)]
    for i, line in enumerate(lines, 1):
        if "# noqa" in line:
            continue
        if len(line) > maxlen:
            errs.append((i, "E501 line too long (%d > %d characters)" % (len(line), maxlen)))
        if line.startswith("\t"):
            errs.append((i, "W191 indentation contains tabs"))
        if line != line.rstrip():
            errs.append((i, "W291 trailing whitespace"))
    is_init = os.path.basename(path) == "__init__.py"
    for ln, msg in _unused_imports(tree, lines):
        if is_init and msg.startswith("F401"):
            continue  # package re-exports
        if ln - 1 < len(lines) and "# noqa" in lines[ln - 1]:
            continue
        errs.append((ln, msg))
    return errs


def main(paths=None):
    maxlen, excl = _config()
    n = 0
    for f in _files(paths or DEFAULT, excl):
        for ln, msg in lint_file(f, maxlen):
            print("%s:%d: %s" % (os.path.relpath(f, ROOT), ln, msg))
            n += 1
    return n


if __name__ == "__main__":
    sys.exit(1 if main(sys.argv[1:] or None) else 0)
