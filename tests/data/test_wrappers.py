"""BufferingWrapper / RolloutInfoWrapper (reference: tests/data/test_wrappers.py)."""

import numpy as np
import pytest

from imitation_amd.data import wrappers
from imitation_amd.envs import core, spaces
from imitation_amd.envs.vec_env import DummyVecEnv


class _CountingEnv(core.Env):
    """obs = t, reward = 10 t, episode length ``episode_length``."""

    def __init__(self, episode_length=5):
        self.episode_length = episode_length
        self.observation_space = spaces.Box(low=0, high=np.inf, shape=(), dtype=np.float32)
        self.action_space = spaces.Box(low=0, high=np.inf, shape=(), dtype=np.float32)
        self.timestep = None

    def reset(self, *, seed=None, options=None):
        self.timestep = 0
        return np.array(self.timestep, dtype=np.float32), {}

    def step(self, action):
        if self.timestep is None:
            raise RuntimeError("Need to reset before first step().")
        self.timestep += 1
        return (np.array(self.timestep, dtype=np.float32), self.timestep * 10.0,
                self.timestep >= self.episode_length, False, {})


def _venv(n_envs=1, episode_length=5):
    return wrappers.BufferingWrapper(DummyVecEnv([lambda: _CountingEnv(episode_length)] * n_envs))


@pytest.mark.parametrize("n_envs", [1, 2])
def test_pop_trajectories_and_transitions(n_envs):
    venv = _venv(n_envs, episode_length=3)
    venv.reset()
    for t in range(7):
        venv.step(np.zeros(n_envs, dtype=np.float32))
    trajs, lens = venv.pop_trajectories()
    # two finished episodes per env (auto-reset), plus one partial of length 1 per env
    assert sum(len(tr) for tr in trajs) == 7 * n_envs
    finished = [tr for tr in trajs if tr.terminal]
    assert len(finished) == 2 * n_envs
    for tr in finished:
        np.testing.assert_array_equal(tr.obs, [0, 1, 2, 3])
        np.testing.assert_array_equal(tr.rews, [10, 20, 30])
    # after popping, nothing is left
    venv.step(np.zeros(n_envs, dtype=np.float32))
    tr2 = venv.pop_transitions()
    assert len(tr2) == n_envs


def test_premature_reset_raises():
    venv = _venv(1)
    venv.reset()
    venv.step(np.zeros(1, dtype=np.float32))
    with pytest.raises(RuntimeError):
        venv.reset()
    venv.error_on_premature_reset = False
    venv.reset()


def test_rollout_info_wrapper_records_episode():
    env = wrappers.RolloutInfoWrapper(_CountingEnv(2))
    env.reset()
    env.step(np.float32(0))
    _, _, term, _, info = env.step(np.float32(0))
    assert term
    ro = info["rollout"]
    assert len(ro["obs"]) == 3 and list(ro["rews"]) == [10.0, 20.0]
