#!/usr/bin/env python3
"""`make lint`: the checks the reference's `make lint` ran through dmlc's cpplint / pylint
(`/root/reference/Makefile:97-98`), done with what this image has (no cpplint, flake8 or
clang-format are installed; there is no package index to fetch them).

C++ / HIP (csrc/, tests/cpp/, examples/*.cc):
  * lines of at most 100 columns (120 in tests/ and tools/), no tab characters, no trailing whitespace, a final newline;
  * every header has an include guard of the form XRABIT_<PATH>_H_ (public headers under
    csrc/include/rabit keep the reference's RABIT_* guards: programs written against the
    reference include them) and no `using namespace` at file scope;
  * no CUDA spellings (cuda*, __CUDA_ARCH__, <cuda...>) and no dual-platform #ifdefs.
Python (rabit_amd/, python/, tests/, tools/, bench.py, __graft_entry__.py):
  * it compiles; lines of at most 100 columns (120 in tests/ and tools/), no tabs, no trailing whitespace;
  * no unused top-level imports (names imported and never used; `# noqa` exempts a line).
Exit status 1 with one line per finding, 0 when clean.
"""
import ast
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAX_COLS = 100        # the library (C++, HIP, rabit_amd/, bench.py), as cpplint's default
MAX_COLS_AUX = 120    # tests and tools
CPP_DIRS = ["csrc", os.path.join("tests", "cpp"), "examples"]
CPP_EXT = (".h", ".cc", ".hip")
PY_DIRS = ["rabit_amd", "python", "tests", "tools"]
PY_FILES = ["bench.py", "__graft_entry__.py"]
SKIP_DIRS = {"refbuild", "__pycache__", "build"}
CUDA_RE = re.compile(r"\bcuda[A-Z]\w*\(|__CUDA_ARCH__|#\s*include\s*<cuda|__HIP_PLATFORM_NVIDIA__")


def walk(dirs, exts):
    for d in dirs:
        base = os.path.join(ROOT, d)
        for dirpath, dirnames, files in os.walk(base):
            dirnames[:] = [x for x in dirnames if x not in SKIP_DIRS]
            for f in sorted(files):
                if f.endswith(exts):
                    yield os.path.join(dirpath, f)


def text_checks(path, text, findings):
    rel = os.path.relpath(path, ROOT)
    aux = rel.replace(os.sep, "/").startswith(("tests/", "tools/"))
    cols = MAX_COLS_AUX if aux else MAX_COLS
    if text and not text.endswith("\n"):
        findings.append("%s: no newline at end of file" % rel)
    for i, line in enumerate(text.split("\n"), 1):
        if "\t" in line:
            findings.append("%s:%d: tab character" % (rel, i))
        if line.rstrip() != line:
            findings.append("%s:%d: trailing whitespace" % (rel, i))
        if len(line) > cols and "http" not in line:
            findings.append("%s:%d: %d columns (max %d)" % (rel, i, len(line), cols))


def guard_name(rel):
    parts = rel.replace(os.sep, "/").split("/")
    if parts[:2] == ["csrc", "src"]:
        parts = parts[2:]
    elif parts[:2] == ["csrc", "include"]:
        parts = parts[2:]
    return "XRABIT_" + re.sub(r"[^A-Za-z0-9]", "_", "_".join(parts)).upper() + "_"


def cpp_checks(path, text, findings):
    rel = os.path.relpath(path, ROOT)
    if CUDA_RE.search(text):
        findings.append("%s: CUDA spelling or dual-platform guard" % rel)
    if path.endswith(".h"):
        public = rel.replace(os.sep, "/").startswith("csrc/include/rabit/")
        m = re.search(r"#ifndef\s+(\w+)[^\n]*\n\s*#define\s+(\w+)", text)
        if not m or m.group(1) != m.group(2):
            findings.append("%s: missing include guard" % rel)
        elif not public and m.group(1) != guard_name(rel):
            findings.append("%s: include guard %s, expected %s" % (rel, m.group(1), guard_name(rel)))
        for i, line in enumerate(text.split("\n"), 1):
            if line.startswith("using namespace"):
                findings.append("%s:%d: `using namespace` at file scope in a header" % (rel, i))


def py_checks(path, text, findings):
    rel = os.path.relpath(path, ROOT)
    try:
        tree = ast.parse(text, rel)
    except SyntaxError as e:
        findings.append("%s:%s: syntax error: %s" % (rel, e.lineno, e.msg))
        return
    lines = text.split("\n")
    imported = {}
    for node in tree.body:
        if isinstance(node, (ast.Import, ast.ImportFrom)):
            if "noqa" in lines[node.lineno - 1]:
                continue
            if isinstance(node, ast.ImportFrom) and node.module == "__future__":
                continue
            for a in node.names:
                name = (a.asname or a.name).split(".")[0]
                if name != "*":
                    imported[name] = node.lineno
    if not imported or os.path.basename(path) == "__init__.py":
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
    for node in tree.body:
        if isinstance(node, ast.Assign) and any(
                isinstance(t, ast.Name) and t.id == "__all__" for t in node.targets):
            exported = {e.value for e in getattr(node.value, "elts", []) if isinstance(e, ast.Constant)}
    for name, line in sorted(imported.items(), key=lambda kv: kv[1]):
        if name not in used and name not in exported:
            findings.append("%s:%d: `%s` imported but unused" % (rel, line, name))


def main():
    findings = []
    ncpp = npy = 0
    for path in walk(CPP_DIRS, CPP_EXT):
        text = open(path, encoding="utf-8").read()
        text_checks(path, text, findings)
        cpp_checks(path, text, findings)
        ncpp += 1
    paths = list(walk(PY_DIRS, (".py",))) + [os.path.join(ROOT, f) for f in PY_FILES]
    for path in paths:
        text = open(path, encoding="utf-8").read()
        text_checks(path, text, findings)
        py_checks(path, text, findings)
        npy += 1
    for f in findings:
        print(f)
    print("lint: %d C++/HIP files, %d Python files, %d findings" % (ncpp, npy, len(findings)))
    return 1 if findings else 0


if __name__ == "__main__":
    sys.exit(main())
