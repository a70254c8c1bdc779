#!/usr/bin/env python
"""Static gates run by CI (reference: ci/*.py + pre-commit's flake8/codespell hooks).

* every Python file byte-compiles;
* tests that touch ``cuda`` / ``.cuda()`` carry ``@pytest.mark.gpu`` (the CPU suite must
  pass without a GPU) -- checked per test function;
* native sources are CDNA4-only: no CUDA headers, no NVIDIA/AMD platform ``#ifdef`` dual
  paths, no hipify markers;
* no Python file loads untrusted pickles (``pickle.load``, ``allow_pickle=True``,
  ``weights_only=False``).
Exit status 1 lists every violation.
"""

from __future__ import annotations

import ast
import pathlib
import py_compile
import re
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
PY_DIRS = ["imitation_amd", "tests", "tools", "benchmarking", "experiments", "examples", "ci"]
NATIVE_BAD = [r"#\s*include\s*<cuda", r"__HIP_PLATFORM_NVIDIA__", r"#\s*if(def)?\s+__HIP_PLATFORM_AMD__", r"hipify",
              r"__CUDACC__"]


def py_files():
    for d in PY_DIRS:
        yield from sorted((ROOT / d).rglob("*.py"))
    yield from sorted(ROOT.glob("*.py"))


def check_compile(errors):
    for f in py_files():
        try:
            py_compile.compile(str(f), doraise=True)
        except py_compile.PyCompileError as e:
            errors.append(f"{f}: does not compile: {e.msg}")


def _marked_gpu(node, module_marked: bool) -> bool:
    if module_marked:
        return True
    for dec in getattr(node, "decorator_list", []):
        src = ast.unparse(dec)
        if src in ("gpu", "pytest.mark.gpu") or src.endswith("mark.gpu"):
            return True
    return False


def check_gpu_marks(errors):
    for f in sorted((ROOT / "tests").rglob("test_*.py")):
        tree = ast.parse(f.read_text())
        module_marked = "pytestmark = pytest.mark.gpu" in f.read_text()
        for node in ast.walk(tree):
            if isinstance(node, ast.FunctionDef) and node.name.startswith("test_"):
                body = ast.unparse(node)
                uses_gpu = re.search(r"\"cuda\"|'cuda'|\.cuda\(\)|device=\"cuda", body) is not None
                guarded = "cuda.is_available()" in body
                if uses_gpu and not guarded and not _marked_gpu(node, module_marked):
                    errors.append(f"{f}:{node.lineno}: {node.name} uses the GPU but is not marked @pytest.mark.gpu")


def check_native(errors):
    for f in sorted((ROOT / "csrc").rglob("*")):
        if f.suffix not in (".hip", ".h", ".cpp", ".hpp"):
            continue
        text = f.read_text()
        for pat in NATIVE_BAD:
            for m in re.finditer(pat, text):
                line = text[: m.start()].count("\n") + 1
                errors.append(f"{f}:{line}: CUDA / dual-path construct {m.group(0)!r}")


def check_pickle(errors):
    """Calls that unpickle (``pickle.load(s)``, ``cloudpickle.loads``) and ``allow_pickle=True`` /
    ``weights_only=False`` keywords, unless the line is annotated ``# noqa: pickle`` (an
    explicit trusted-source opt-in)."""
    for f in py_files():
        if f.name == "check_code.py":
            continue
        text = f.read_text()
        lines = text.splitlines()
        for node in ast.walk(ast.parse(text)):
            if not isinstance(node, ast.Call):
                continue
            bad = None
            fn = ast.unparse(node.func)
            if fn in ("pickle.load", "pickle.loads", "cloudpickle.loads", "cloudpickle.load", "joblib.load", "dill.load"):
                bad = fn
            for kw in node.keywords:
                if kw.arg in ("allow_pickle", "weights_only") and isinstance(kw.value, ast.Constant):
                    if (kw.arg == "allow_pickle") == bool(kw.value.value):
                        bad = f"{kw.arg}={kw.value.value}"
            if bad and "noqa: pickle" not in lines[node.lineno - 1]:
                errors.append(f"{f}:{node.lineno}: unsafe deserialisation {bad}")


def check_test_basenames(errors):
    """``tests/`` subdirectories are rootdir-relative modules (no ``__init__.py``), so two test
    files with one basename make pytest's collection fail with "import file mismatch" -- which
    stops every ``-x`` run before its first test (round-3 GPU step)."""
    seen: dict = {}
    for f in sorted((ROOT / "tests").rglob("*.py")):
        if not f.name.startswith("test_"):
            continue
        if f.name in seen:
            errors.append(f"{f}: test module basename also used by {seen[f.name]} (pytest collection error)")
        else:
            seen[f.name] = f


def check_collect(errors):
    """``pytest --collect-only`` over the whole suite reports no collection error (CPU, no GPU)."""
    import subprocess

    proc = subprocess.run([sys.executable, "-m", "pytest", "--collect-only", "-q", "-p", "no:cacheprovider",
                           str(ROOT / "tests")], cwd=ROOT, capture_output=True, text=True, timeout=900)
    tail = proc.stdout.strip().splitlines()[-1:] if proc.stdout.strip() else [proc.stderr.strip()[-400:]]
    if proc.returncode != 0 or any("error" in line for line in tail):
        errors.append(f"pytest --collect-only failed (rc {proc.returncode}): {tail}")


def main(collect: bool = False) -> int:
    errors: list = []
    checks = [check_compile, check_gpu_marks, check_native, check_pickle, check_test_basenames]
    if collect:
        checks.append(check_collect)
    for check in checks:
        check(errors)
    for e in errors:
        print(e)
    print(f"{len(errors)} violation(s)")
    return 1 if errors else 0


if __name__ == "__main__":
    sys.exit(main(collect="--collect" in sys.argv))
