"""RL substrate: PPO / SAC / DQN (SB3-compatible surface the reference depends on)."""

import numpy as np
import pytest
import torch as th

from imitation_amd.data import rollout
from imitation_amd.rl import dqn, ppo, sac
from imitation_amd.rl.buffers import RolloutBuffer
from imitation_amd.ops import rl as rl_ops
from imitation_amd.util import util

from tests.conftest import CARTPOLE_EXPERT_ZIP


def _returns(model, venv, rng, n=8):
    trajs = rollout.rollout(model.policy, venv, rollout.make_min_episodes(n), rng=rng, deterministic_policy=True, unwrap=False)
    return np.mean([t.rews.sum() for t in trajs])


def test_ppo_learns_cartpole(rng):
    venv = util.make_vec_env("CartPole-v1", rng=rng, n_envs=8)
    model = ppo.PPO("MlpPolicy", venv, n_steps=128, batch_size=256, n_epochs=4, learning_rate=2.5e-3, seed=0, device="cpu",
                    policy_kwargs=dict(net_arch=[32, 32]))
    before = _returns(model, venv, rng)
    model.learn(25_000)
    after = _returns(model, venv, rng)
    assert after > before + 50 and after > 120


def test_ppo_save_load_roundtrip(tmp_path, rng):
    venv = util.make_vec_env("Pendulum-v1", rng=rng, n_envs=2)
    model = ppo.PPO("MlpPolicy", venv, n_steps=32, batch_size=32, n_epochs=1, device="cpu")
    model.learn(64)
    model.save(tmp_path / "m.zip")
    loaded = ppo.PPO.load(tmp_path / "m.zip", env=venv, device="cpu")
    obs = np.random.rand(7, 3).astype(np.float32)
    np.testing.assert_allclose(model.policy.predict(obs, deterministic=True)[0], loaded.policy.predict(obs, deterministic=True)[0],
                               rtol=1e-6)
    assert loaded.n_steps == 32 and loaded.num_timesteps == model.num_timesteps


def test_load_sb3_model_zip_without_pickle(rng):
    """The checked-in SB3 expert loads through JSON side fields + weights_only tensors."""
    venv = util.make_vec_env("CartPole-v1", rng=rng, n_envs=2)
    model = ppo.PPO.load(CARTPOLE_EXPERT_ZIP, env=venv, device="cpu")
    assert _returns(model, venv, rng, n=4) > 450


@pytest.mark.parametrize("gamma,lam", [(0.99, 0.95), (0.9, 1.0), (1.0, 0.0)])
def test_gae_matches_loop(gamma, lam):
    T, N = 37, 5
    g = th.Generator().manual_seed(0)
    rew = th.randn(T, N, generator=g)
    val = th.randn(T, N, generator=g)
    starts = (th.rand(T, N, generator=g) < 0.1).float()
    last_v = th.randn(N, generator=g)
    dones = (th.rand(N, generator=g) < 0.5).float()
    adv, ret = rl_ops.gae(rew, val, starts, last_v, dones, gamma, lam)
    # SB3 RolloutBuffer.compute_returns_and_advantage loop
    exp = th.zeros(T, N)
    last = th.zeros(N)
    for t in reversed(range(T)):
        if t == T - 1:
            nnt, nv = 1.0 - dones, last_v
        else:
            nnt, nv = 1.0 - starts[t + 1], val[t + 1]
        delta = rew[t] + gamma * nv * nnt - val[t]
        last = delta + gamma * lam * nnt * last
        exp[t] = last
    th.testing.assert_close(adv, exp, rtol=1e-5, atol=1e-5)
    th.testing.assert_close(ret, exp + val, rtol=1e-5, atol=1e-5)


def test_dqn_runs_and_saves(tmp_path, rng):
    venv = util.make_vec_env("CartPole-v1", rng=rng, n_envs=1)
    model = dqn.DQN("MlpPolicy", venv, learning_starts=50, buffer_size=1000, batch_size=32, device="cpu", seed=0)
    model.learn(300)
    model.save(tmp_path / "dqn.zip")
    loaded = dqn.DQN.load(tmp_path / "dqn.zip", env=venv, device="cpu")
    obs = np.random.rand(5, 4).astype(np.float32)
    np.testing.assert_array_equal(model.predict(obs, deterministic=True)[0], loaded.predict(obs, deterministic=True)[0])


def test_sac_runs_and_saves(tmp_path, rng):
    venv = util.make_vec_env("Pendulum-v1", rng=rng, n_envs=1)
    model = sac.SAC("MlpPolicy", venv, learning_starts=50, buffer_size=1000, batch_size=32, device="cpu", seed=0,
                    policy_kwargs=dict(net_arch=[32, 32]))
    model.learn(200)
    model.save(tmp_path / "sac.zip")
    loaded = sac.SAC.load(tmp_path / "sac.zip", env=venv, device="cpu")
    obs = np.random.rand(5, 3).astype(np.float32)
    np.testing.assert_allclose(model.predict(obs, deterministic=True)[0], loaded.predict(obs, deterministic=True)[0], rtol=1e-5)


@pytest.mark.parametrize("name", ["TD3", "DDPG"])
def test_td3_ddpg_run_and_save(tmp_path, rng, name):
    from imitation_amd.rl import noise, td3

    cls = getattr(td3, name)
    venv = util.make_vec_env("Pendulum-v1", rng=rng, n_envs=1)
    an = noise.NormalActionNoise(np.zeros(1), 0.1 * np.ones(1), rng=np.random.default_rng(0))
    model = cls("MlpPolicy", venv, learning_starts=50, buffer_size=1000, batch_size=32, device="cpu", seed=0,
                action_noise=an, policy_kwargs=dict(net_arch=[32, 32]))
    model.learn(200)
    model.save(tmp_path / f"{name}.zip")
    loaded = cls.load(tmp_path / f"{name}.zip", env=venv, device="cpu")
    obs = np.random.rand(5, 3).astype(np.float32)
    np.testing.assert_allclose(model.predict(obs, deterministic=True)[0], loaded.predict(obs, deterministic=True)[0], rtol=1e-5)


def test_action_noise_resets_only_the_finished_env(rng):
    """with n_envs > 1 an episode end resets that env's noise process only
    (SB3 passes ``indices=[idx]``), not every env's Ornstein-Uhlenbeck state."""
    from imitation_amd.rl import noise, td3

    class Recording(noise.VectorizedActionNoise):
        calls = []

        def reset(self, indices=None):
            self.calls.append(None if indices is None else list(indices))
            super().reset(indices)

    venv = util.make_vec_env("Pendulum-v1", rng=rng, n_envs=2)
    base = noise.OrnsteinUhlenbeckActionNoise(np.zeros(1), 0.1 * np.ones(1), rng=np.random.default_rng(0))
    an = Recording(base, n_envs=2)
    model = td3.TD3("MlpPolicy", venv, learning_starts=50, buffer_size=1000, batch_size=32, device="cpu", seed=0,
                    action_noise=an, policy_kwargs=dict(net_arch=[16]))
    model.learn(2 * 210)  # every env finishes one 200-step episode
    assert Recording.calls and all(c is not None and len(c) == 1 for c in Recording.calls)
    assert sorted(c[0] for c in Recording.calls) == [0, 1]


def test_ou_noise_is_temporally_correlated_and_resets():
    from imitation_amd.rl import noise

    ou = noise.OrnsteinUhlenbeckActionNoise(np.zeros(2), 0.3 * np.ones(2), rng=np.random.default_rng(0))
    xs = np.stack([ou() for _ in range(2000)])
    assert xs.shape == (2000, 2)
    assert np.corrcoef(xs[:-1, 0], xs[1:, 0])[0, 1] > 0.9
    ou.reset()
    assert np.all(ou.noise_prev == 0)
    vec = noise.VectorizedActionNoise(noise.NormalActionNoise(np.zeros(3), np.ones(3)), n_envs=4)
    assert vec().shape == (4, 3)


def test_rollout_buffer_generator_covers_all_rows():
    from imitation_amd.envs import spaces

    buf = RolloutBuffer(8, spaces.Box(-1, 1, (2,)), spaces.Discrete(2), device="cpu", n_envs=3)
    for t in range(8):
        buf.add(np.full((3, 2), t, np.float32), np.zeros(3, np.int64), np.ones(3), np.zeros(3), th.zeros(3), th.zeros(3))
    buf.compute_returns_and_advantage(th.zeros(3), np.zeros(3))
    seen = th.cat([b.observations[:, 0] for b in buf.get(batch_size=5)])
    assert sorted(seen.tolist()) == sorted([float(t) for t in range(8) for _ in range(3)])


def test_distribution_detach_releases_forward_graph():
    """``Distribution.detach_`` drops the last forward's autograd graph the policy's shared
    distribution object keeps (needed before a HIP-graph capture, utils/graphs.py)."""
    import torch as th

    from imitation_amd.rl import distributions as D

    x = th.randn(4, 5, requires_grad=True)
    cat = D.CategoricalDistribution(5).proba_distribution(x * 2)
    assert cat.raw_logits.grad_fn is not None
    assert cat.detach_().raw_logits.grad_fn is None
    multi = D.MultiCategoricalDistribution([2, 3]).proba_distribution(x * 2)
    multi.detach_()
    assert all(d.raw_logits.grad_fn is None for d in multi.dists)
    g = D.DiagGaussianDistribution(5).proba_distribution(x * 2, th.zeros(5, requires_grad=True) + 0)
    g.detach_()
    assert g.mean_actions.grad_fn is None and g.log_std.grad_fn is None
    assert th.isfinite(g.log_prob(th.zeros(4, 5))).all()
