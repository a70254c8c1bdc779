"""The CI static gates (ci/check_code.py) pass on the tree."""

import importlib.util
import pathlib


def test_static_gates_pass():
    path = pathlib.Path(__file__).resolve().parents[1] / "ci" / "check_code.py"
    spec = importlib.util.spec_from_file_location("check_code", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    assert mod.main() == 0
