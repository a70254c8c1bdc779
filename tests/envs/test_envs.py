"""Environment layer: spaces, native batched envs (C++ runtime), VecEnv semantics."""

import math

import numpy as np
import pytest

from imitation_amd.envs import core, spaces
from imitation_amd.envs.vec_env import DummyVecEnv, NativeEnv, NativeVecEnv, SubprocVecEnv, VecNormalize
from imitation_amd.util import util


def _cartpole_step(s, a):
    """gymnasium CartPole-v1 Euler dynamics."""
    x, xd, th, thd = s
    g, mc, mp, l, fm, tau = 9.8, 1.0, 0.1, 0.5, 10.0, 0.02
    force = fm if a == 1 else -fm
    ct, st = math.cos(th), math.sin(th)
    temp = (force + mp * l * thd ** 2 * st) / (mc + mp)
    thacc = (g * st - ct * temp) / (l * (4.0 / 3.0 - mp * ct ** 2 / (mc + mp)))
    xacc = temp - mp * l * thacc * ct / (mc + mp)
    return np.array([x + tau * xd, xd + tau * xacc, th + tau * thd, thd + tau * thacc])


def test_native_cartpole_matches_reference_dynamics():
    env = NativeEnv("CartPole-v1")
    obs, _ = env.reset(seed=3)
    s = obs.astype(np.float64)
    rng = np.random.default_rng(0)
    for _ in range(30):
        a = int(rng.integers(2))
        obs, r, term, trunc, _ = env.step(a)
        s = _cartpole_step(s, a)
        np.testing.assert_allclose(obs, s, rtol=1e-4, atol=1e-5)
        if term:
            break
        assert r == 1.0


def test_pendulum_reward_and_bounds():
    env = NativeEnv("Pendulum-v1")
    obs, _ = env.reset(seed=0)
    assert obs.shape == (3,) and abs(obs[0] ** 2 + obs[1] ** 2 - 1) < 1e-5
    _, r, term, trunc, _ = env.step(np.array([2.0], np.float32))
    assert r <= 0 and not term


@pytest.mark.parametrize("env_id", ["seals/CartPole-v0", "Pendulum-v1", "seals/HalfCheetah-v1", "MountainCar-v0",
                                    "Acrobot-v1", "seals/Hopper-v1"])
def test_native_vec_env_api(env_id):
    venv = util.make_vec_env(env_id, n_envs=3, rng=np.random.default_rng(0))
    assert isinstance(venv, NativeVecEnv)
    obs = venv.reset()
    assert obs.shape == (3,) + venv.observation_space.shape
    for _ in range(5):
        acts = np.stack([venv.action_space.sample() for _ in range(3)])
        obs, rew, done, infos = venv.step(acts)
        assert obs.shape[0] == 3 and rew.shape == (3,) and done.shape == (3,) and len(infos) == 3


def test_seals_fixed_horizon_and_terminal_obs():
    venv = util.make_vec_env("seals/CartPole-v0", n_envs=2, rng=np.random.default_rng(0), max_episode_steps=7)
    venv.reset()
    for t in range(7):
        obs, rew, done, infos = venv.step(np.zeros(2, dtype=np.int64))
    assert done.all()
    assert all("terminal_observation" in i and i.get("TimeLimit.truncated", True) for i in infos)


def test_native_seeding_reproducible():
    def roll(seed):
        venv = util.make_vec_env("seals/HalfCheetah-v1", n_envs=2, rng=np.random.default_rng(seed))
        out = [venv.reset()]
        for _ in range(3):
            out.append(venv.step(np.full((2, 6), 0.3, np.float32))[0])
        return np.stack(out)

    np.testing.assert_array_equal(roll(1), roll(1))
    assert not np.array_equal(roll(1), roll(2))


class _Count(core.Env):
    def __init__(self):
        self.observation_space = spaces.Box(0, 100, (1,))
        self.action_space = spaces.Discrete(2)
        self.t = 0

    def reset(self, *, seed=None, options=None):
        self.t = 0
        return np.array([0.0], np.float32), {}

    def step(self, a):
        self.t += 1
        return np.array([self.t], np.float32), float(a), self.t >= 3, False, {}


@pytest.mark.parametrize("cls", [DummyVecEnv, SubprocVecEnv])
def test_python_vec_envs_autoreset(cls):
    venv = cls([_Count, _Count])
    venv.reset()
    for _ in range(3):
        obs, rew, done, infos = venv.step(np.array([1, 0]))
    assert done.all() and np.all(obs == 0)
    np.testing.assert_array_equal(infos[0]["terminal_observation"], [3.0])
    np.testing.assert_array_equal(rew, [1.0, 0.0])
    venv.close()


def test_vec_normalize():
    venv = VecNormalize(DummyVecEnv([_Count]), norm_obs=True, norm_reward=True)
    venv.reset()
    for _ in range(20):
        obs, rew, _, _ = venv.step(np.array([1]))
    assert np.all(np.abs(obs) <= venv.clip_obs)


def test_spaces_flatten_and_contains():
    b = spaces.Box(-1, 1, (2, 3))
    x = b.sample()
    assert b.contains(x) and spaces.flatdim(b) == 6 and spaces.flatten(b, x).shape == (6,)
    d = spaces.Discrete(4)
    assert spaces.flatten(d, 2).tolist() == [0, 0, 1, 0]
    md = spaces.MultiDiscrete([2, 3])
    assert spaces.flatdim(md) == 5
    inf = spaces.Box(np.array([0]), np.array([np.inf]), dtype=np.int64)
    assert inf.high[0] == np.iinfo(np.int64).max


def test_registry_and_time_limit():
    env = core.make("seals/CartPole-v0")
    assert env.spec.max_episode_steps == 500
    env = core.make("seals/RandomTransition-v0", n_states=4, n_actions=2, branch_factor=2, horizon=5, random_obs=False)
    env.reset(seed=0)
    for _ in range(5):
        _, _, term, trunc, _ = env.step(0)
    assert trunc or term
