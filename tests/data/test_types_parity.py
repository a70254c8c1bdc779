"""Trajectory / Transitions container behaviour over the space matrix of the reference's
``tests/data/test_types.py`` (TestData :137-406, zero length :409, parse_path :416, DictObs
:461): validity and length for every observation / action space and length, equality against
other types, copies and perturbations, save / load round trips (dataset directory and a
pickled list this test writes itself), input validation messages, Transitions indexing and
slicing per field, and the DictObs API."""

import contextlib
import copy
import dataclasses
import os
import pathlib
import pickle

import numpy as np
import pytest

from imitation_amd.data import serialize, types
from imitation_amd.envs import spaces
from imitation_amd.util import util

SPACES = [
    spaces.Discrete(3),
    spaces.MultiDiscrete([3, 4]),
    spaces.Box(-1, 1, shape=(1,)),
    spaces.Box(-1, 1, shape=(2,)),
    spaces.Box(-np.inf, np.inf, shape=(2,)),
]
DICT_SPACE = spaces.Dict({"a": spaces.Discrete(3), "b": spaces.Box(-1, 1, shape=(2,))})
OBS_SPACES = SPACES + [DICT_SPACE]
ACT_SPACES = SPACES
LENGTHS = [0, 1, 2, 10]


def _check_1d_shape(fn, length: int, expected_msg: str):
    for shape in [(), (length, 1), (length, 2), (length - 1,), (length + 1,)]:
        with pytest.raises(ValueError, match=expected_msg):
            fn(np.zeros(shape))


@pytest.fixture
def trajectory(obs_space, act_space, length) -> types.Trajectory:
    if length == 0:
        pytest.skip()
    raw_obs = [obs_space.sample() for _ in range(length + 1)]
    obs = types.DictObs.from_obs_list(raw_obs) if isinstance(obs_space, spaces.Dict) else np.array(raw_obs)
    acts = np.array([act_space.sample() for _ in range(length)])
    infos = np.array([{f"key{i}": i} for i in range(length)])
    return types.Trajectory(obs=obs, acts=acts, infos=infos, terminal=True)


@pytest.fixture
def trajectory_rew(trajectory) -> types.TrajectoryWithRew:
    return types.TrajectoryWithRew(**types.dataclass_quick_asdict(trajectory), rews=np.random.randn(len(trajectory)))


@pytest.fixture
def transitions_min(obs_space, act_space, length) -> types.TransitionsMinimal:
    raw = [obs_space.sample() for _ in range(length)]
    obs = types.DictObs.from_obs_list(raw) if isinstance(obs_space, spaces.Dict) and length else np.array(raw)
    acts = np.array([act_space.sample() for _ in range(length)])
    infos = np.array([{i: i} for i in range(length)])
    return types.TransitionsMinimal(obs=obs, acts=acts, infos=infos)


@pytest.fixture
def transitions(transitions_min, obs_space, length) -> types.Transitions:
    raw = [obs_space.sample() for _ in range(length)]
    next_obs = types.DictObs.from_obs_list(raw) if isinstance(obs_space, spaces.Dict) and length else np.array(raw)
    return types.Transitions(**types.dataclass_quick_asdict(transitions_min), next_obs=next_obs,
                             dones=np.zeros(length, dtype=bool))


@pytest.fixture
def transitions_rew(transitions, length) -> types.TransitionsWithRew:
    return types.TransitionsWithRew(**types.dataclass_quick_asdict(transitions), rews=np.random.randn(length))


def _check_transitions_get_item(trans, key):
    item = trans[key]
    for field in dataclasses.fields(trans):
        observed = item[field.name] if isinstance(item, dict) else getattr(item, field.name)
        expected = getattr(trans, field.name)[key]
        if isinstance(expected, np.ndarray):
            assert observed.dtype == expected.dtype
        if isinstance(expected, types.DictObs):
            assert observed == expected
        else:
            np.testing.assert_array_equal(observed, expected)


@contextlib.contextmanager
def pushd(dir_path):
    orig = pathlib.Path.cwd()
    try:
        os.chdir(dir_path)
        yield
    finally:
        os.chdir(orig)


@pytest.mark.parametrize("obs_space", OBS_SPACES)
@pytest.mark.parametrize("act_space", ACT_SPACES)
@pytest.mark.parametrize("length", LENGTHS)
class TestData:
    def test_valid_trajectories(self, trajectory, trajectory_rew, length):
        trajs = [trajectory, trajectory_rew]
        trajs += [dataclasses.replace(t, infos=None) for t in trajs]
        for t in trajs:
            assert len(t) == length

    def test_traj_unequal_to_other_types(self, trajectory, trajectory_rew):
        for t in [trajectory, trajectory_rew]:
            assert t != 42
            assert t != "foobar"
        assert trajectory != trajectory_rew

    def test_traj_equal_to_self_and_copies(self, trajectory, trajectory_rew):
        for t in [trajectory, trajectory_rew]:
            assert t == t
            assert t == copy.copy(t)

    def test_traj_unequal_to_perturbations(self, trajectory, trajectory_rew, length):
        new_length = length - 1
        if new_length > 0:
            assert trajectory != types.Trajectory(obs=trajectory.obs[: new_length + 1], acts=trajectory.acts[:new_length],
                                                  infos=trajectory.infos[:new_length], terminal=trajectory.terminal)
        for t in [trajectory, trajectory_rew]:
            as_dict = types.dataclass_quick_asdict(t)
            for k in as_dict:
                perturbed = dict(as_dict)
                if k == "infos":
                    perturbed["infos"] = [{"foo": 42}] * len(as_dict["infos"])
                elif isinstance(as_dict[k], types.DictObs):
                    perturbed[k] = as_dict[k].map_arrays(lambda x: x + 1)
                else:
                    perturbed[k] = as_dict[k] + 1
                assert t != type(t)(**perturbed)

    def test_invalid_trajectories(self, trajectory, trajectory_rew):
        for traj in [trajectory, trajectory_rew]:
            with pytest.raises(ValueError, match=r"expected one more observations than actions.*"):
                dataclasses.replace(traj, obs=traj.obs[:-1])
            with pytest.raises(ValueError, match=r"expected one more observations than actions.*"):
                dataclasses.replace(traj, acts=traj.acts[:-1])
            with pytest.raises(ValueError, match=r"infos when present must be present for each action.*"):
                dataclasses.replace(traj, infos=traj.infos[:-1])
            with pytest.raises(ValueError, match=r"infos when present must be present for each action.*"):
                dataclasses.replace(traj, obs=traj.obs[:-1], acts=traj.acts[:-1])
        _check_1d_shape(lambda rews: dataclasses.replace(trajectory_rew, rews=rews), len(trajectory_rew),
                        r"rewards must be 1D array.*")
        with pytest.raises(ValueError, match=r"rewards dtype.* not a float"):
            dataclasses.replace(trajectory_rew, rews=np.zeros(len(trajectory_rew), dtype=int))

    def test_valid_transitions(self, transitions_min, transitions, transitions_rew, length, n_checks: int = 20):
        rng = np.random.default_rng(length)
        for trans in [transitions_min, transitions, transitions_rew]:
            assert len(trans) == length
            for _ in range(n_checks):
                if length != 0:
                    index = int(rng.integers(length))
                    assert isinstance(trans[index], dict)
                    _check_transitions_get_item(trans, index)
                start, stop = int(rng.integers(-2, length)), int(rng.integers(0, length + 2))
                step = int(rng.integers(-2, 4)) or 1
                s = slice(start, stop, step)
                if isinstance(trans.obs, types.DictObs) and len(range(*s.indices(length))) == 0:
                    continue  # an empty DictObs has no length to validate against
                assert type(trans[s]) is type(trans)
                _check_transitions_get_item(trans, s)

    def test_invalid_transitions(self, transitions_min, transitions, transitions_rew, length):
        if length == 0:
            pytest.skip()
        for trans in [transitions_min, transitions, transitions_rew]:
            with pytest.raises(ValueError, match=r"obs and acts must have same number of timesteps:.*"):
                dataclasses.replace(trans, acts=trans.acts[:-1])
            with pytest.raises(ValueError, match=r"obs and infos must have same number of timesteps:.*"):
                dataclasses.replace(trans, infos=[{}] * (length - 1))
        for trans in [transitions, transitions_rew]:
            with pytest.raises(ValueError, match=r"obs and next_obs must have same shape:.*"):
                dataclasses.replace(trans, next_obs=np.zeros((len(trans), 4, 2)))
            if not isinstance(trans.obs, types.DictObs):
                with pytest.raises(ValueError, match=r"obs and next_obs must have the same dtype:.*"):
                    dataclasses.replace(trans, next_obs=np.zeros_like(trans.next_obs, dtype=bool))
            _check_1d_shape(lambda d: dataclasses.replace(trans, dones=d), len(trans), r"dones must be 1D array.*")
            with pytest.raises(ValueError, match=r"dones must be boolean"):
                dataclasses.replace(trans, dones=np.zeros(len(trans), dtype=int))
        _check_1d_shape(lambda r: dataclasses.replace(transitions_rew, rews=r), len(transitions_rew),
                        r"rewards must be 1D array.*")
        with pytest.raises(ValueError, match=r"rewards dtype.* not a float"):
            dataclasses.replace(transitions_rew, rews=np.zeros(len(transitions_rew), dtype=int))


# save / load round trips on a reduced matrix (each dataset save is ~10 ms of file IO)
@pytest.mark.parametrize("obs_space", [SPACES[0], SPACES[4], DICT_SPACE])
@pytest.mark.parametrize("act_space", [SPACES[1], SPACES[3]])
@pytest.mark.parametrize("length", [1, 10])
@pytest.mark.parametrize("type_safe", [False, True])
@pytest.mark.parametrize("use_pickle", [False, True])
@pytest.mark.parametrize("use_rewards", [False, True])
@pytest.mark.parametrize("use_chdir", [False, True])
def test_save_trajectories(trajectory, trajectory_rew, use_chdir, tmpdir, use_pickle, use_rewards, type_safe):
    if isinstance(trajectory.obs, types.DictObs) and not use_pickle:
        pytest.xfail("Saving/loading dictobs trajectories as a dataset is not supported (as in the reference)")
    ctx = pushd(tmpdir) if use_chdir else contextlib.nullcontext()
    with ctx:
        save_dir = util.parse_path("" if use_chdir else tmpdir)
        trajs = [trajectory_rew if use_rewards else trajectory]
        save_path = save_dir / "trajs"
        if use_pickle:
            with open(save_path, "wb") as f:
                pickle.dump(trajs, f)
            with pytest.raises(ValueError, match="refusing to unpickle"):
                serialize.load(save_path)  # a pickle only loads on explicit opt-in
        else:
            serialize.save(save_path, trajs)
            if use_rewards:
                with pytest.raises(ValueError):
                    serialize.save(save_path, [trajectory, trajectory_rew])
        kw = dict(allow_pickle=True) if use_pickle else {}  # noqa: pickle -- the list this test pickled itself
        if type_safe:
            if use_rewards:
                loaded = serialize.load_with_rewards(save_path, **kw)
            else:
                with pytest.raises(ValueError):
                    serialize.load_with_rewards(save_path, **kw)
                loaded = serialize.load(save_path, **kw)
        else:
            loaded = serialize.load(save_path, **kw)
        assert len(trajs) == len(loaded)
        for t1, t2 in zip(trajs, loaded):
            assert t1 == t2


def test_zero_length_fails():
    with pytest.raises(ValueError, match=r"Degenerate trajectory.*"):
        types.Trajectory(obs=np.array([42]), acts=np.array([]), infos=None, terminal=True)


def test_parse_path():
    assert util.parse_path("/foo/bar") == pathlib.Path("/foo/bar")
    assert util.parse_path(pathlib.Path("/foo/bar")) == pathlib.Path("/foo/bar")
    assert util.parse_path(b"/foo/bar") == pathlib.Path("/foo/bar")
    assert util.parse_path("foo/bar") == pathlib.Path.cwd() / "foo/bar"
    assert util.parse_path(pathlib.Path("foo/bar")) == pathlib.Path.cwd() / "foo/bar"
    assert util.parse_path(b"foo/bar") == pathlib.Path.cwd() / "foo/bar"
    base = pathlib.Path("/foo/bar")
    assert util.parse_path("baz", base_directory=base) == base / "baz"
    assert util.parse_path(pathlib.Path("baz"), base_directory=base) == base / "baz"
    assert util.parse_path(b"baz", base_directory=base) == base / "baz"
    with pytest.raises(ValueError, match="Path .* is not absolute"):
        util.parse_path("foo/bar", allow_relative=False)
    with pytest.raises(ValueError, match="If `base_directory` is specified, then `allow_relative` must be True."):
        util.parse_path("foo/bar", base_directory=pathlib.Path("/foo/bar"), allow_relative=False)
    assert util.parse_optional_path(None) is None
    assert util.parse_optional_path("/foo/bar") == util.parse_path("/foo/bar")


def test_dict_obs():
    A = np.random.rand(3, 4)
    B = np.random.rand(3, 7, 1)
    C = np.random.rand(4)
    ab = types.DictObs({"a": A, "b": B})
    abc = types.DictObs({"a": A, "b": B, "c": C})
    assert len(ab) == 3
    with pytest.raises(RuntimeError):
        len(abc)
    with pytest.raises(RuntimeError):
        len(types.DictObs({}))
    assert abc.dict_len == 3
    np.testing.assert_equal(abc[0].get("a"), A[0])
    np.testing.assert_equal(abc[0].get("c"), np.array(C[0]))
    np.testing.assert_equal(abc[0:2].get("a"), np.array(A[0:2]))
    np.testing.assert_equal(ab[:, 0].get("a"), np.array(A[:, 0]))
    with pytest.raises(IndexError):
        abc[:, 0]
    for i, a_row in enumerate(A):
        np.testing.assert_equal(a_row, ab[i].get("a"))
    assert ab[0] == next(iter(ab))
    assert abc == types.DictObs({"a": A, "b": B, "c": C})
    assert abc == types.DictObs({"a": np.array(A), "b": np.array(B), "c": np.array(C)})
    assert abc != types.DictObs({"a": A, "c": B, "b": C})
    assert abc != types.DictObs({"a": A, "b": B + 1, "c": C})
    assert abc != {"a": A, "b": B + 1, "c": C}
    assert abc != ab
    assert abc.shape == {"a": A.shape, "b": B.shape, "c": C.shape}
    assert abc.dtype == {"a": A.dtype, "b": B.dtype, "c": C.dtype}
    assert types.maybe_wrap_in_dictobs({"a": A, "b": B, "c": C}) == abc
    assert abc.unwrap() == {"a": A, "b": B, "c": C}
    assert abc.map_arrays(lambda arr: arr + 1) == types.DictObs({"a": A + 1, "b": B + 1, "c": C + 1})
    assert types.DictObs.stack(list(iter(ab))) == ab
    np.testing.assert_equal(types.DictObs.concatenate([abc, abc]).get("a"), np.concatenate([A, A]))
    with pytest.raises(AssertionError):
        types.assert_not_dictobs(abc)
    with pytest.raises(TypeError):
        types.DictObs({"a": "not an array"})
