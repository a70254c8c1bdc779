"""util helpers and registry (reference: tests/util/test_util.py, test_registry.py)."""

import numpy as np
import pytest
import torch as th

from imitation_amd.util import registry, util


def test_oric():
    x = np.array([0.4, 1.4, 2.2])
    r = util.oric(x)
    assert r.sum() == round(x.sum()) and np.all(np.abs(r - x) < 1)
    assert util.oric(np.array([1.0, 2.0, 3.0])).tolist() == [1, 2, 3]


def test_make_seeds():
    rng = np.random.default_rng(0)
    s = util.make_seeds(rng, 5)
    assert len(s) == 5 and len(set(s)) == 5
    assert isinstance(util.make_seeds(np.random.default_rng(0)), int)


def test_endless_iter():
    it = util.endless_iter([1, 2])
    assert [next(it) for _ in range(5)] == [1, 2, 1, 2, 1]
    with pytest.raises(ValueError):
        next(util.endless_iter([]))


def test_safe_conversions():
    a = np.zeros((2, 2), dtype=np.float32)
    a.flags.writeable = False
    t = util.safe_to_tensor(a)
    assert isinstance(t, th.Tensor) and t.shape == (2, 2)
    assert isinstance(util.safe_to_numpy(th.ones(2)), np.ndarray)
    assert util.safe_to_numpy(None) is None


def test_tensor_iter_norm():
    ts = [th.tensor([3.0]), th.tensor([4.0])]
    assert float(util.tensor_iter_norm(ts)) == pytest.approx(5.0)
    assert float(util.tensor_iter_norm(ts, ord=1)) == pytest.approx(7.0)


def test_get_first_iter_element():
    first, it = util.get_first_iter_element(iter([1, 2, 3]))
    assert first == 1 and list(it) == [1, 2, 3]
    with pytest.raises(ValueError):
        util.get_first_iter_element([])


def test_parse_path(tmp_path):
    assert util.parse_path("a/b", base_directory=tmp_path) == tmp_path / "a" / "b"
    with pytest.raises(ValueError):
        util.parse_path("rel", allow_relative=False)
    assert util.parse_optional_path(None) is None


def test_registry():
    r = registry.Registry()
    r.register("a", value=1)
    r.register("b", indirect="imitation_amd.util.util:oric")
    assert r.get("a") == 1 and r.get("b") is util.oric and set(r.keys()) == {"a", "b"}
    with pytest.raises(KeyError):
        r.register("a", value=2)
    with pytest.raises(ValueError):
        r.register("c")
    with pytest.raises(KeyError):
        r.get("zzz")


def test_endless_iter_errors():

    with pytest.raises(ValueError, match="no elements"):
        util.endless_iter([])
    with pytest.raises(ValueError, match="needs a non-iterator Iterable"):
        util.endless_iter(x for x in range(5))

def test_first_iter_element_of_a_generator_keeps_every_element():

    with pytest.raises(ValueError, match="had no elements"):
        util.get_first_iter_element([])
    seq = [4, 1, 7]
    first, same = util.get_first_iter_element(seq)
    assert first == 4 and same is seq
    gen = (x for x in seq)
    first, rest = util.get_first_iter_element(gen)
    assert first == 4 and list(rest) == seq and list(rest) == []

def test_oric_keeps_integral_sums():
    g = np.random.default_rng(0)
    for n in range(1, 11):
        x = g.uniform(1e-3, 1e6, n)
        x = x - (x.sum() - np.floor(x.sum())) / n
        r = util.oric(x)
        assert np.allclose(r.sum(), x.sum()) and np.abs(x - r).max() <= 1.0
        assert np.allclose(r, np.round(r))

def test_dict_get_nested():
    from imitation_amd.util import sacred as sacred_util

    assert sacred_util.dict_get_nested({}, "asdf.foo", default=4) == 4
    assert sacred_util.dict_get_nested({"a": {"b": "c"}}, "a.b") == "c"
