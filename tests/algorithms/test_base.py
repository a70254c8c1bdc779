"""BaseImitationAlgorithm horizon checks and make_data_loader validation / format equivalence
(upstream tests/algorithms/test_base.py)."""

import numpy as np
import pytest
import torch as th

from imitation_amd.algorithms import base
from imitation_amd.data import types


def test_fixed_horizon_check(custom_logger):
    algo = base.BaseImitationAlgorithm(custom_logger=custom_logger)
    algo._check_fixed_horizon([])
    assert algo._horizon is None
    algo._check_fixed_horizon([7, 7])
    assert algo._horizon == 7
    algo._check_fixed_horizon([])
    for bad in ([6], [8], [7, 1]):
        with pytest.raises(ValueError, match="Episodes of different length"):
            algo._check_fixed_horizon(bad)
    assert algo._horizon == 7


def test_variable_horizon_allowed(custom_logger):
    algo = base.BaseImitationAlgorithm(custom_logger=custom_logger, allow_variable_horizon=True)
    algo._check_fixed_horizon([3])
    algo._check_fixed_horizon([30, 3])
    assert algo._horizon is None


def _drain(*args, **kwargs):
    for _ in base.make_data_loader(*args, **kwargs):
        pass


def test_data_loader_batch_size_validation():
    for bs in (0, -3):
        with pytest.raises(ValueError, match="must be positive"):
            base.make_data_loader([], batch_size=bs)
    batches = [{"obs": np.zeros((4, 2)), "acts": np.zeros((4, 1))}]
    _drain(batches, batch_size=4)
    for bs in (3, 5):
        with pytest.raises(ValueError, match="Expected batch size"):
            _drain(batches, batch_size=bs)
    with pytest.raises(ValueError, match="Expected batch size"):
        _drain([{"obs": np.zeros((4, 2)), "acts": np.zeros((3, 1))}], batch_size=4)
    trans = types.TransitionsMinimal(obs=np.zeros((4, 2)), acts=np.zeros((4, 1)), infos=np.array([{}] * 4))
    for bs in range(1, 5):
        base.make_data_loader(trans, batch_size=bs)
    with pytest.raises(ValueError, match="smaller than batch size"):
        base.make_data_loader(trans, batch_size=5)


def test_data_loader_same_batches_from_every_format():
    trajs = [types.Trajectory(obs=np.array([0, 1]), acts=np.array([10]), infos=None, terminal=True),
             types.Trajectory(obs=np.array([2, 3, 4]), acts=np.array([11, 12]), infos=None, terminal=False)]
    trans = types.Transitions(obs=np.array([0, 2, 3]), acts=np.array([10, 11, 12]), next_obs=np.array([1, 3, 4]),
                              dones=np.array([True, False, False]), infos=np.array([{}] * 3))
    expected = [{"obs": [0, 2], "acts": [10, 11], "next_obs": [1, 3], "dones": [True, False]},
                {"obs": [3], "acts": [12], "next_obs": [4], "dones": [False]}]
    for data in (trajs, trans):
        loader = base.make_data_loader(data, batch_size=2, data_loader_kwargs=dict(shuffle=False, drop_last=False))
        got = list(loader)
        assert len(got) == len(expected)
        for b, e in zip(got, expected):
            for k, v in e.items():
                x = b[k].numpy() if isinstance(b[k], th.Tensor) else np.asarray(b[k])
                np.testing.assert_array_equal(x, np.asarray(v))
