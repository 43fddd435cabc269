"""`make lint` is clean and `make doc` is current (CPU): the hygiene checks that replace the
reference's cpplint / pylint (`/root/reference/Makefile:97-98`), and the API reference generated
from the sources (`Makefile:100-104`)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_lint_clean():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "lint.py")],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout[-4000:]
    assert "0 findings" in p.stdout


def test_api_doc_current():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gendoc.py"), "--check"],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
