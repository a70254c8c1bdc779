"""The CI static gates (ci/check_code.py) pass on the tree."""

import importlib.util
import pathlib

ROOT = pathlib.Path(__file__).resolve().parents[1]


def _load():
    spec = importlib.util.spec_from_file_location("check_code", ROOT / "ci" / "check_code.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_static_gates_pass():
    assert _load().main() == 0


def test_no_duplicate_test_basenames():
    errors: list = []
    _load().check_test_basenames(errors)
    assert errors == []


def test_duplicate_basename_gate_fires(tmp_path, monkeypatch):
    mod = _load()
    (tmp_path / "tests" / "a").mkdir(parents=True)
    (tmp_path / "tests" / "b").mkdir(parents=True)
    (tmp_path / "tests" / "a" / "test_x.py").write_text("")
    (tmp_path / "tests" / "b" / "test_x.py").write_text("")
    monkeypatch.setattr(mod, "ROOT", tmp_path)
    errors: list = []
    mod.check_test_basenames(errors)
    assert len(errors) == 1 and "test_x.py" in errors[0]


def test_suite_collects_cleanly():
    """``pytest --collect-only`` of the whole suite has no collection error (the round-3 GPU
    step stopped at one)."""
    errors: list = []
    _load().check_collect(errors)
    assert errors == []
