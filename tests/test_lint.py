"""The repository passes its own lint (scripts/lint.py) — the CI gate of the CPU tier."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_repo_lint_clean():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "lint.py")], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:]
