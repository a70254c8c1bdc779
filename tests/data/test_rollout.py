"""Rollout engine (reference: tests/data/test_rollout.py)."""

import numpy as np
import pytest

from imitation_amd.data import rollout, types, wrappers
from imitation_amd.envs import core, spaces
from imitation_amd.envs.vec_env import DummyVecEnv
from imitation_amd.policies.base import RandomPolicy
from imitation_amd.util import util


class TerminalSentinelEnv(core.Env):
    """Episode ends after ``max_acts`` steps; obs is the step count."""

    def __init__(self, max_acts: int):
        self.max_acts = max_acts
        self.current_step = 0
        self.action_space = spaces.Discrete(1)
        self.observation_space = spaces.Box(np.array([0]), np.array([np.inf]), dtype=np.int64)

    def reset(self, *, seed=None, options=None):
        self.current_step = 0
        return np.array([0]), {}

    def step(self, action):
        self.current_step += 1
        done = self.current_step >= self.max_acts
        return np.array([self.current_step]), 0.0, done, False, {}


def _sentinel_venv(n_envs, max_acts):
    return DummyVecEnv([lambda: wrappers.RolloutInfoWrapper(TerminalSentinelEnv(max_acts)) for _ in range(n_envs)])


@pytest.mark.parametrize("n_envs", [1, 3])
def test_complete_trajectories(n_envs, rng):
    venv = _sentinel_venv(n_envs, max_acts=4)
    trajs = rollout.generate_trajectories(RandomPolicy(venv.observation_space, venv.action_space), venv,
                                          rollout.make_sample_until(min_episodes=5), rng=rng)
    assert len(trajs) >= 5
    for t in trajs:
        assert len(t) == 4
        assert t.terminal
        np.testing.assert_array_equal(t.obs[:, 0], np.arange(5))


def test_unbiased_sampling(rng):
    """Episodes from every env slot show up; no env's episodes dominate."""
    venv = DummyVecEnv([lambda i=i: wrappers.RolloutInfoWrapper(TerminalSentinelEnv(2 + i)) for i in range(3)])
    trajs = rollout.generate_trajectories(None, venv, rollout.make_sample_until(min_episodes=12), rng=rng)
    lens = sorted({len(t) for t in trajs})
    assert lens == [2, 3, 4]


def test_sample_until():
    trajs = [types.TrajectoryWithRew(obs=np.zeros((4, 1)), acts=np.zeros(3), infos=None, terminal=True, rews=np.zeros(3))] * 3
    assert rollout.make_min_episodes(3)(trajs)
    assert not rollout.make_min_episodes(4)(trajs)
    assert rollout.make_min_timesteps(9)(trajs)
    assert not rollout.make_min_timesteps(10)(trajs)
    assert rollout.make_sample_until(min_timesteps=9, min_episodes=3)(trajs)
    with pytest.raises(ValueError):
        rollout.make_sample_until(min_timesteps=None, min_episodes=None)


def test_rollout_stats():
    trajs = [
        types.TrajectoryWithRew(obs=np.zeros((n + 1, 1)), acts=np.zeros(n), infos=None, terminal=True, rews=np.ones(n))
        for n in (2, 4)
    ]
    s = rollout.rollout_stats(trajs)
    assert s["n_traj"] == 2
    assert s["return_mean"] == 3.0 and s["len_max"] == 4 and s["return_min"] == 2.0


def test_flatten_trajectories():
    trajs = [
        types.TrajectoryWithRew(obs=np.arange(n + 1, dtype=np.float32)[:, None], acts=np.zeros(n), infos=None,
                                terminal=term, rews=np.ones(n))
        for n, term in ((3, True), (2, False))
    ]
    tr = rollout.flatten_trajectories_with_rew(trajs)
    assert len(tr) == 5
    np.testing.assert_array_equal(tr.dones, [False, False, True, False, False])
    np.testing.assert_array_equal(tr.obs[:, 0], [0, 1, 2, 0, 1])
    np.testing.assert_array_equal(tr.next_obs[:, 0], [1, 2, 3, 1, 2])


def test_discounted_sum():
    arr = np.array([1.0, 2.0, 3.0])
    assert rollout.discounted_sum(arr, 1.0) == 6.0
    np.testing.assert_allclose(rollout.discounted_sum(arr, 0.5), 1 + 1 + 0.75)
    np.testing.assert_allclose(rollout.discounted_sum(np.ones((3, 2)), 0.5), [1.75, 1.75])


def test_generate_transitions_native(rng):
    venv = util.make_vec_env("seals/CartPole-v0", n_envs=2, rng=rng, post_wrappers=[lambda e, _: wrappers.RolloutInfoWrapper(e)])
    tr = rollout.generate_transitions(None, venv, n_timesteps=50, rng=rng, truncate=True)
    assert len(tr) == 50
    assert tr.obs.shape == (50, 4)


def test_expert_rollout_is_good(cartpole_expert_policy, cartpole_venv, rng):
    trajs = rollout.rollout(cartpole_expert_policy, cartpole_venv, rollout.make_sample_until(min_episodes=4), rng=rng)
    assert np.mean([t.rews.sum() for t in trajs]) > 400
