"""Policies, serialization, exploration / replay-relabel / interactive wrappers
(reference: tests/policies/*)."""

import collections
from unittest import mock

import numpy as np
import pytest
import torch as th

from imitation_amd.data import rollout
from imitation_amd.envs import spaces
from imitation_amd.policies import base, exploration_wrapper, interactive, replay_buffer_wrapper, serialize
from imitation_amd.rewards import reward_nets
from imitation_amd.rl import buffers
from imitation_amd.util import networks, util


@pytest.mark.parametrize("policy_type", ["random", "zero"])
def test_non_trainable_policies(policy_type, cartpole_venv, rng):
    pol = serialize.load_policy(policy_type, cartpole_venv)
    trajs = rollout.generate_trajectories(pol, cartpole_venv, rollout.make_min_timesteps(20), rng=rng)
    acts = np.concatenate([t.acts for t in trajs])
    if policy_type == "zero":
        assert np.all(acts == 0)


def test_ppo_policy_roundtrip(tmp_path, cartpole_venv):
    from imitation_amd.rl.ppo import PPO

    model = PPO("MlpPolicy", cartpole_venv, n_steps=16, batch_size=16, device="cpu")
    serialize.save_stable_model(tmp_path / "m", model)
    pol = serialize.load_policy("ppo", cartpole_venv, path=str(tmp_path / "m"))
    obs = np.random.rand(10, 4).astype(np.float32)
    np.testing.assert_array_equal(model.policy.predict(obs, deterministic=True)[0], pol.predict(obs, deterministic=True)[0])
    with pytest.raises(FileNotFoundError):
        serialize.load_policy("ppo", cartpole_venv, path=str(tmp_path))


def test_vec_normalize_pkl_rejected(tmp_path, cartpole_venv):
    from imitation_amd.rl.ppo import PPO

    model = PPO("MlpPolicy", cartpole_venv, n_steps=16, batch_size=16, device="cpu")
    serialize.save_stable_model(tmp_path, model)
    (tmp_path / "vec_normalize.pkl").write_bytes(b"x")
    with pytest.raises(FileExistsError):
        serialize.load_policy("ppo", cartpole_venv, path=str(tmp_path))


@pytest.mark.parametrize("cls", [base.FeedForward32Policy, base.SAC1024Policy])
def test_policy_save_load_weights_only(cls, tmp_path):
    o, a = spaces.Box(-1, 1, (3,)), spaces.Box(-1, 1, (2,))
    if cls is base.SAC1024Policy:
        from imitation_amd.rl.sac import SACPolicy  # noqa: F401
        pol = cls(observation_space=o, action_space=a, lr_schedule=lambda _: 1e-3)
    else:
        pol = cls(observation_space=o, action_space=a, lr_schedule=lambda _: 1e-3)
    util.save_policy(pol, tmp_path / "p.pt")
    assert th.load(tmp_path / "p.pt", weights_only=True)["format"] == "imitation_amd.policy.v1"
    from imitation_amd.rl.policies import load_policy_file

    re = load_policy_file(tmp_path / "p.pt", device="cpu")
    obs = np.random.rand(5, 3).astype(np.float32)
    np.testing.assert_allclose(pol.predict(obs, deterministic=True)[0], re.predict(obs, deterministic=True)[0], rtol=1e-6)


def test_normalize_features_extractor():
    o = spaces.Box(-np.inf, np.inf, (4,))
    fe = base.NormalizeFeaturesExtractor(o, normalize_class=networks.RunningNorm)
    x = th.randn(64, 4) * 5 + 3
    with networks.training(fe):
        for _ in range(50):
            fe(x)
    with networks.evaluating(fe):
        y = fe(x)
    assert abs(float(y.mean())) < 0.1 and abs(float(y.std()) - 1) < 0.1


def test_homogenous_policy_batches_agents():
    o, a = spaces.Box(-1, 1, (3,)), spaces.Box(-1, 1, (2,))
    obs_over = lambda i, obs: obs[:, 3 * i: 3 * i + 3]  # noqa: E731
    act_over = lambda i, act: act[:, 2 * i: 2 * i + 2]  # noqa: E731
    pol = base.HomogenousFeedForward32Policy(obs_over, act_over, 2, observation_space=o, action_space=a,
                                             lr_schedule=lambda _: 1e-3)
    acts, _ = pol.predict(np.random.rand(5, 6).astype(np.float32))
    assert acts.shape == (5, 4) and np.all(np.abs(acts) <= 1)


def test_exploration_wrapper(cartpole_venv, rng):
    zero = base.ZeroPolicy(cartpole_venv.observation_space, cartpole_venv.action_space)
    wrapped = exploration_wrapper.ExplorationWrapper(zero, cartpole_venv, random_prob=1.0, switch_prob=1.0, rng=rng)
    obs = cartpole_venv.reset()
    acts = np.concatenate([wrapped(obs, None, None)[0] for _ in range(50)])
    assert 0 < acts.mean() < 1  # random actions mixed in
    never = exploration_wrapper.ExplorationWrapper(zero, cartpole_venv, random_prob=0.0, switch_prob=1.0, rng=rng)
    assert np.all(np.concatenate([never(obs, None, None)[0] for _ in range(20)]) == 0)
    with pytest.raises(ValueError):
        never(obs, (np.zeros(1),), None)


def test_replay_buffer_reward_wrapper():
    o, a = spaces.Box(-1, 1, (2,)), spaces.Box(-1, 1, (1,))
    rn = reward_nets.BasicRewardNet(o, a)
    for fn in (rn.predict_processed, lambda state, action, next_state, done: np.full(len(state), 7.0)):
        buf = replay_buffer_wrapper.ReplayBufferRewardWrapper(100, o, a, replay_buffer_class=buffers.ReplayBuffer,
                                                              reward_fn=fn, device="cpu")
        for _ in range(10):
            buf.add(np.random.rand(1, 2), np.random.rand(1, 2), np.random.rand(1, 1), np.array([1.0]),
                    np.array([False]), [{}])
        s = buf.sample(8)
        assert s.rewards.shape == (8, 1)
        if not isinstance(fn, type(rn.predict_processed)):
            assert th.all(s.rewards == 7.0)
        else:
            exp = rn.predict_processed(s.observations.numpy(), s.actions.numpy(), s.next_observations.numpy(),
                                       s.dones.numpy().reshape(-1))
            np.testing.assert_allclose(s.rewards.numpy().reshape(-1), exp, rtol=1e-5, atol=1e-6)
        assert buf.size() == 10 and buf.pos == 10


def test_interactive_policy_reads_keys():
    o = spaces.Box(0, 255, (4, 4, 1), dtype=np.uint8)
    keys = collections.OrderedDict([("w", "up"), ("s", "down")])

    class _Pol(interactive.DiscreteInteractivePolicy):
        def _render(self, obs):
            return None

    pol = _Pol(o, spaces.Discrete(2), keys, clear_screen_on_query=False)
    with mock.patch("builtins.input", side_effect=["x", "s"]):
        acts, _ = pol.predict(np.zeros((1, 4, 4, 1), np.uint8))
    assert acts.tolist() == [1]


def test_atari_interactive_key_map():
    class _Env:
        observation_space = spaces.Box(0, 255, (8, 8, 4), dtype=np.uint8)
        action_space = spaces.Discrete(6)

        def get_action_meanings(self):
            return interactive.PONG_ACTION_MEANINGS

    pol = interactive.AtariInteractivePolicy(_Env(), clear_screen_on_query=False)
    assert list(pol.action_keys_names.values()) == interactive.PONG_ACTION_MEANINGS
