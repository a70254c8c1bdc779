"""Trajectory / Transitions containers (reference: tests/data/test_types.py)."""

import numpy as np
import pytest
import torch as th

from imitation_amd.data import types


def _traj(n=5, with_rew=True, terminal=True):
    obs = np.arange((n + 1) * 2, dtype=np.float32).reshape(n + 1, 2)
    acts = np.arange(n, dtype=np.int64)
    infos = np.array([{"i": i} for i in range(n)], dtype=object)
    if with_rew:
        return types.TrajectoryWithRew(obs=obs, acts=acts, infos=infos, terminal=terminal, rews=np.ones(n, np.float32))
    return types.Trajectory(obs=obs, acts=acts, infos=infos, terminal=terminal)


def test_trajectory_validation():
    t = _traj()
    assert len(t) == 5
    with pytest.raises(ValueError):
        types.Trajectory(obs=np.zeros((5, 2)), acts=np.zeros(5), infos=None, terminal=True)
    with pytest.raises(ValueError):
        types.Trajectory(obs=np.zeros((6, 2)), acts=np.zeros(5), infos=np.array([{}] * 4), terminal=True)
    with pytest.raises(ValueError):
        types.TrajectoryWithRew(obs=np.zeros((6, 2)), acts=np.zeros(5), infos=None, terminal=True, rews=np.zeros(4))


def test_trajectory_equality():
    assert _traj() == _traj()
    other = _traj()
    other.obs[0, 0] = 100.0
    assert _traj() != other
    assert _traj(terminal=False) != _traj(terminal=True)


def test_transitions_indexing_and_collate():
    n = 6
    tr = types.Transitions(
        obs=np.random.rand(n, 3).astype(np.float32), acts=np.arange(n), infos=np.array([{}] * n, dtype=object),
        next_obs=np.random.rand(n, 3).astype(np.float32), dones=np.zeros(n, bool),
    )
    assert len(tr) == n
    sl = tr[1:4]
    assert isinstance(sl, types.Transitions) and len(sl) == 3
    item = tr[2]
    assert set(item.keys()) >= {"obs", "acts", "next_obs", "dones", "infos"}
    batch = types.transitions_collate_fn([tr[i] for i in range(4)])
    assert batch["obs"].shape == (4, 3) and isinstance(batch["acts"], th.Tensor)
    assert isinstance(batch["infos"], list) and len(batch["infos"]) == 4


def test_transitions_length_mismatch():
    with pytest.raises(ValueError):
        types.Transitions(obs=np.zeros((3, 2)), acts=np.zeros(4), infos=np.array([{}] * 3),
                          next_obs=np.zeros((3, 2)), dones=np.zeros(3, bool))


def test_dictobs_roundtrip():
    d = types.DictObs({"a": np.zeros((4, 2)), "b": np.ones((4, 3))})
    assert len(d) == 4
    assert d[1:3].shape == {"a": (2, 2), "b": (2, 3)}
    st = types.DictObs.stack([d[0], d[1]])
    assert st.shape == {"a": (2, 2), "b": (2, 3)}
    cat = types.DictObs.concatenate([d, d])
    assert len(cat) == 8
    assert types.maybe_unwrap_dictobs(d)["a"].shape == (4, 2)
    assert isinstance(types.maybe_wrap_in_dictobs({"a": np.zeros(2)}), types.DictObs)
