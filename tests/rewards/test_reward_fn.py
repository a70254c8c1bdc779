"""RewardFn subclassing and ValidateRewardFn shape checking (upstream tests/rewards/test_reward_fn.py)."""

import numpy as np
import pytest

from imitation_amd.rewards import reward_function, serialize

_RNG = np.random.default_rng(0)
OBS = _RNG.integers(0, 10, (32, 12)).astype(np.float32)
DONES = np.zeros(32, dtype=bool)


class _IndexReward(reward_function.RewardFn):
    def __call__(self, state, action, next_state, done=None):
        return np.arange(len(state), dtype=np.float32)


def test_subclass_is_a_reward_fn():
    fn = _IndexReward()
    np.testing.assert_array_equal(fn(OBS, OBS, OBS, DONES), np.arange(32, dtype=np.float32))
    with pytest.raises(TypeError):
        reward_function.RewardFn()  # abstract


def test_validate_reward_fn_checks_length():
    ok = serialize.ValidateRewardFn(_IndexReward())
    assert ok(OBS, OBS, OBS, DONES).shape == (32,)
    short = serialize.ValidateRewardFn(lambda s, a, n, d: np.arange(len(s) - 1, dtype=np.float32))
    with pytest.raises(AssertionError):
        short(OBS, OBS, OBS, DONES)
    wide = serialize.ValidateRewardFn(lambda s, a, n, d: np.zeros((len(s), 1), np.float32))
    with pytest.raises(AssertionError):
        wide(OBS, OBS, OBS, DONES)
