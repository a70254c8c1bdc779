"""RL algorithms over ``spaces.Dict`` observations (SB3 ``MultiInputPolicy`` +
``DictRolloutBuffer`` / ``DictReplayBuffer`` surface; CPU)."""

import numpy as np
import pytest
import torch as th

from imitation_amd.envs import core, spaces
from imitation_amd.envs.vec_env import DummyVecEnv
from imitation_amd.rl.buffers import DictReplayBuffer, DictRolloutBuffer
from imitation_amd.rl.policies import MultiInputActorCriticPolicy
from imitation_amd.rl.ppo import PPO
from imitation_amd.rl.sac import SAC


class _DictEnv(core.Env):
    """obs {"a": Box(2), "b": Box(3)}, continuous action, reward -|a|, 5-step episodes."""

    def __init__(self):
        self.action_space = spaces.Box(-1.0, 1.0, (1,))
        self.observation_space = spaces.Dict({"a": spaces.Box(-1.0, 1.0, (2,)), "b": spaces.Box(0.0, 1.0, (3,))})
        self.t = 0
        self.g = np.random.default_rng(0)

    def _obs(self):
        return {"a": self.g.uniform(-1, 1, 2).astype(np.float32), "b": self.g.uniform(0, 1, 3).astype(np.float32)}

    def reset(self, *, seed=None, options=None):
        self.t = 0
        return self._obs(), {}

    def step(self, action):
        self.t += 1
        return self._obs(), float(-abs(action[0])), self.t >= 5, False, {}


def test_sac_multi_input_policy_fills_a_dict_replay_buffer():
    venv = DummyVecEnv([_DictEnv, _DictEnv])
    algo = SAC("MultiInputPolicy", venv, buffer_size=64, learning_starts=4, batch_size=8, device="cpu", seed=0)
    before = [p.detach().clone() for p in algo.policy.parameters()]
    algo.learn(40)
    rb = algo.replay_buffer
    assert isinstance(rb, DictReplayBuffer) and rb.size() == 20
    s = rb.sample(8)
    assert {k: tuple(v.shape) for k, v in s.observations.items()} == {"a": (8, 2), "b": (8, 3)}
    assert set(s.next_observations) == {"a", "b"} and s.actions.shape == (8, 1) and s.rewards.shape == (8, 1)
    assert th.all(s.rewards <= 0)
    assert any(not th.equal(a, b) for a, b in zip(before, algo.policy.parameters()))


def test_dict_replay_buffer_ring_and_terminal_observations():
    space = _DictEnv().observation_space
    rb = DictReplayBuffer(4, space, spaces.Box(-1.0, 1.0, (1,)), device="cpu")
    for i in range(6):
        o = {"a": np.full((1, 2), i, np.float32), "b": np.full((1, 3), i, np.float32)}
        n = {"a": np.full((1, 2), i + 1, np.float32), "b": np.full((1, 3), i + 1, np.float32)}
        rb.add(o, n, np.zeros((1, 1)), np.array([float(i)]), np.array([False]), [{}])
    assert rb.full and rb.pos == 2
    s = rb.sample(64)
    a = s.observations["a"][:, 0]
    assert set(a.tolist()) <= {2.0, 3.0, 4.0, 5.0}  # the 4 newest rows
    np.testing.assert_array_equal(s.next_observations["b"][:, 0].numpy(), a.numpy() + 1)
    np.testing.assert_array_equal(s.rewards[:, 0].numpy(), a.numpy())
    rb.extend({"a": np.full((3, 2), 9, np.float32), "b": np.zeros((3, 3), np.float32)},
              {"a": np.zeros((3, 2), np.float32), "b": np.zeros((3, 3), np.float32)}, np.zeros((3, 1)), np.ones(3),
              np.zeros(3))
    assert rb.pos == 1 and (rb.observations["a"][:, 0, 0] == 9).sum() == 3
    # more rows than the ring holds: only the newest 4 survive, in FIFO slots
    rows = np.arange(10, dtype=np.float32)
    rb.extend({"a": np.repeat(rows[:, None], 2, 1), "b": np.zeros((10, 3), np.float32)},
              {"a": np.zeros((10, 2), np.float32), "b": np.zeros((10, 3), np.float32)}, np.zeros((10, 1)), rows,
              np.zeros(10))
    assert rb.pos == (1 + 10) % 4 and rb.full
    # slot (pos + j) % 4 holds the j-th oldest survivor: rows 6, 7, 8, 9
    order = [(rb.pos + j) % 4 for j in range(4)]
    assert rb.observations["a"][order, 0, 0].tolist() == [6.0, 7.0, 8.0, 9.0]
    assert rb.rewards[order, 0].tolist() == [6.0, 7.0, 8.0, 9.0]
    with pytest.raises(AssertionError, match="optimize_memory_usage"):
        DictReplayBuffer(4, space, spaces.Box(-1.0, 1.0, (1,)), device="cpu", optimize_memory_usage=True)


def test_ppo_multi_input_policy_uses_a_dict_rollout_buffer():
    venv = DummyVecEnv([_DictEnv, _DictEnv])
    algo = PPO(MultiInputActorCriticPolicy, venv, n_steps=16, batch_size=16, n_epochs=2, device="cpu", seed=0)
    before = [p.detach().clone() for p in algo.policy.parameters()]
    algo.learn(32)
    assert isinstance(algo.rollout_buffer, DictRolloutBuffer)
    assert {k: tuple(v.shape) for k, v in algo.rollout_buffer.observations.items()} == {"a": (16, 2, 2), "b": (16, 2, 3)}
    assert any(not th.equal(a, b) for a, b in zip(before, algo.policy.parameters()))


class _DictDiscreteEnv(_DictEnv):
    def __init__(self):
        super().__init__()
        self.action_space = spaces.Discrete(3)

    def step(self, action):
        self.t += 1
        return self._obs(), float(action == 1), self.t >= 5, False, {}


def test_dqn_multi_input_policy():
    from imitation_amd.rl.dqn import DQN

    venv = DummyVecEnv([_DictDiscreteEnv])
    algo = DQN("MultiInputPolicy", venv, buffer_size=100, learning_starts=8, batch_size=8, train_freq=4, device="cpu", seed=0)
    before = [p.detach().clone() for p in algo.policy.parameters()]
    algo.learn(40)
    assert isinstance(algo.replay_buffer, DictReplayBuffer) and algo.replay_buffer.size() == 40
    assert any(not th.equal(a, b) for a, b in zip(before, algo.policy.parameters()))
    acts, _ = algo.predict({"a": np.zeros((1, 2), np.float32), "b": np.zeros((1, 3), np.float32)}, deterministic=True)
    assert acts.shape == (1,) and 0 <= int(acts[0]) < 3
