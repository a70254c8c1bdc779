"""BufferingWrapper behaviours of the reference's tests/data/test_wrappers.py, expressed against
this package (CPU): popped transitions of a counting env over episode lengths, step counts and
intermediate pops (array and Dict observations), and the transition count / empty-pop error."""

import itertools

import numpy as np
import pytest

from imitation_amd.data import rollout, types
from imitation_amd.data.wrappers import BufferingWrapper
from imitation_amd.envs import core, spaces
from imitation_amd.envs.vec_env import DummyVecEnv


class _Counting(core.Env):
    """obs = timestep (0 after reset), reward = 10 x the new timestep, fixed episode length."""

    def __init__(self, episode_length=5, dict_obs=False):
        self.episode_length = episode_length
        self.dict_obs = dict_obs
        box = spaces.Box(low=0.0, high=float("inf"), shape=(), dtype=np.float32)
        self.observation_space = spaces.Dict({"t": box}) if dict_obs else box
        self.action_space = spaces.Box(low=0.0, high=float("inf"), shape=(), dtype=np.float32)
        self.t = 0

    def _obs(self):
        o = np.array(self.t, dtype=np.float32)
        return {"t": o} if self.dict_obs else o

    def reset(self, *, seed=None, options=None):
        self.t = 0
        return self._obs(), {}

    def step(self, action):
        self.t += 1
        return self._obs(), float(self.t * 10), self.t >= self.episode_length, False, {}


def _t(obs):
    if isinstance(obs, types.DictObs):
        return obs.get("t")
    if isinstance(obs, dict):
        return obs["t"]
    return obs


@pytest.mark.parametrize("dict_obs", [False, True])
@pytest.mark.parametrize("episode_lengths,n_steps,extra_pops", list(itertools.product(
    [(1,), (6,), (3, 3, 3), (3, 5, 1, 2)], [1, 2, 10, 19], [(), (5,), (3, 8)])))
def test_popped_transitions_cover_every_step(dict_obs, episode_lengths, n_steps, extra_pops):
    if any(not 1 <= p < n_steps for p in extra_pops):
        pytest.skip("pop steps outside this run")
    venv = BufferingWrapper(DummyVecEnv([(lambda n=n: _Counting(n, dict_obs)) for n in episode_lengths]))
    obs = venv.reset()
    np.testing.assert_array_equal(_t(obs), np.zeros(len(episode_lengths)))
    pops = []
    for t in range(1, n_steps + 1):
        obs, *_ = venv.step(_t(obs) * 2.1)
        if t in extra_pops:
            pops.append(venv.pop_transitions())
    pops.append(venv.pop_transitions())
    want = []
    for n in episode_lengths:
        full, rest = divmod(n_steps, n)
        want += [np.arange(n)] * full + [np.arange(rest)]
    want = np.sort(np.concatenate(want).astype(np.float32))
    got_obs = np.concatenate([_t(p.obs).reshape(-1) for p in pops])
    got_next = np.concatenate([_t(p.next_obs).reshape(-1) for p in pops])
    acts = np.concatenate([p.acts.reshape(-1) for p in pops])
    rews = np.concatenate([p.rews.reshape(-1) for p in pops])
    np.testing.assert_allclose(np.sort(got_obs), want)
    np.testing.assert_allclose(np.sort(got_next), want + 1)
    np.testing.assert_allclose(np.sort(acts), want * 2.1, rtol=1e-6)
    np.testing.assert_allclose(np.sort(rews), (want + 1) * 10)


@pytest.mark.parametrize("dict_obs", [False, True])
def test_transition_count_and_empty_pop(dict_obs):
    venv = BufferingWrapper(DummyVecEnv([lambda: _Counting(10, dict_obs)] * 2))
    venv.reset()
    trajs, lens = venv.pop_trajectories()
    assert list(trajs) == [] and list(lens) == []
    zeros = np.zeros(2, dtype=np.float32)
    venv.step(zeros)
    assert venv.n_transitions == 2
    venv.step(zeros)
    assert venv.n_transitions == 4
    venv.pop_transitions()
    assert venv.n_transitions == 0
    with pytest.raises(RuntimeError, match="empty"):
        venv.pop_transitions()


def test_popped_trajectories_are_whole_or_partial_episodes():
    venv = BufferingWrapper(DummyVecEnv([lambda: _Counting(3)] * 2))
    obs = venv.reset()
    for _ in range(4):
        obs, *_ = venv.step(obs * 0)
    trajs, lens = venv.pop_trajectories()
    assert sorted(len(t) for t in trajs) == [1, 1, 3, 3] and sorted(lens) == [3, 3]  # lengths of finished episodes
    for t in trajs:
        np.testing.assert_array_equal(t.obs, np.arange(len(t) + 1))
    assert rollout.rollout_stats([t for t in trajs if t.terminal])["n_traj"] == 2
