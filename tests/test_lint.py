"""Lint gate (the reference runs flake8 in CI: /root/reference/.travis.yml:51, tox.ini:1-3).
flake8 is not installed in this image, so tools/lint.py applies the same tox.ini limits with
the standard library only."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_lint_clean(capsys):
    import lint
    n = lint.main()
    out = capsys.readouterr().out
    assert n == 0, out
