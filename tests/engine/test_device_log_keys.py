"""The device engines' per-round generator records match the host-loop trainer's (CPU).

Reference: a GAIL round logs SB3 ``PPO.train`` / ``OnPolicyAlgorithm._dump_logs`` keys and the
reward wrapper's ``rollout/ep_rew_wrapped_mean`` (``adversarial/common.py:234-240, 414-419``).
The device round's recording methods run here on host stand-ins of their inputs (the pinned
statistics the GPU update copies out), against one real host-loop GAIL round."""

import collections

import numpy as np
import torch as th

from imitation_amd.engine.gail import DeviceEngineMixin, DeviceGeneratorCore
from imitation_amd.ops import rl as rl_ops


class _Recorder:
    def __init__(self):
        self.keys = {}

    def record(self, key, value, exclude=None):
        self.keys[key] = exclude

    def record_mean(self, key, value, exclude=None):
        self.keys[key] = exclude


class _FakeEvent:
    def synchronize(self):
        pass


class _FakeRound:
    """The recording methods of a device engine round, with host tensors for the staged data."""

    _record_round_metrics = DeviceGeneratorCore._record_round_metrics
    _ppo_log_values = DeviceGeneratorCore._ppo_log_values
    _fail_if_nonfinite = DeviceGeneratorCore._fail_if_nonfinite
    _track_wrapped_returns = DeviceEngineMixin._track_wrapped_returns
    _log_gen = DeviceEngineMixin._log_gen

    def __init__(self, gen_algo, N=4, T=16, gaussian=False, A=2):
        self.gen_algo, self.N, self.T, self.A = gen_algo, N, T, A
        self.logger = _Recorder()
        self._ppo_log_host = th.rand(5 + 4 * N)
        self._ppo_std_host = th.zeros(A) if gaussian else None
        self._ppo_log_event = _FakeEvent()
        self._last_ppo_info = (T * N, 8)
        self._last_clip_range = 0.2
        self._last_lr = 3e-4


def _host_gen_keys(cartpole_venv, expert_transitions):
    from imitation_amd.algorithms.adversarial import gail
    from imitation_amd.rewards import reward_nets
    from imitation_amd.rl.ppo import PPO
    from imitation_amd.util import logger, networks

    lg = logger.configure(format_strs=[])
    seen = {}
    orig = lg.record

    def record(key, val, exclude=None):
        if lg._scope is not None and lg._scope.name == "gen":
            seen[key] = exclude
        return orig(key, val, exclude)

    lg.record = record
    gen = PPO("MlpPolicy", cartpole_venv, n_steps=32, batch_size=32, n_epochs=2, seed=0, device="cpu",
              policy_kwargs=dict(net_arch=[16, 16]))
    rn = reward_nets.BasicRewardNet(cartpole_venv.observation_space, cartpole_venv.action_space,
                                    normalize_input_layer=networks.RunningNorm)
    tr = gail.GAIL(demonstrations=expert_transitions, demo_batch_size=64, venv=cartpole_venv, gen_algo=gen,
                   reward_net=rn, n_disc_updates_per_round=1, custom_logger=lg)
    # two rounds: the wrapped-reward mean is logged at a rollout START, once episodes ended
    tr.train(total_timesteps=40 * tr.gen_train_timesteps)
    return seen, gen


def test_device_round_logs_the_host_trainers_keys(cartpole_venv, cartpole_expert_trajectories):
    from imitation_amd.data import rollout

    transitions = rollout.flatten_trajectories(cartpole_expert_trajectories[:4])
    host_keys, gen = _host_gen_keys(cartpole_venv, transitions)
    fake = _FakeRound(gen)
    gen.ep_info_buffer = collections.deque([{"r": 1.0, "l": 5, "t": 0.0}], maxlen=100)
    T, N = fake.T, fake.N
    dones = np.zeros((T, N), bool)
    dones[3, 0] = dones[9, 1] = True
    fake._track_wrapped_returns(dones, np.ones((T, N), np.float32))
    fake._track_wrapped_returns(dones, np.ones((T, N), np.float32))
    fake._fps_mark = (0.0, 0)
    gen.num_timesteps += T * N
    fake._log_gen()
    dev_keys = fake.logger.keys
    host = {k.split("/", 2)[-1] if k.startswith("raw/") else k: v for k, v in host_keys.items()}
    assert set(dev_keys) == set(host), (sorted(set(dev_keys) ^ set(host)))
    # tensorboard exclusions as the host records them
    for k in ("train/n_updates", "time/total_timesteps", "time/iterations", "time/time_elapsed"):
        if k in host:
            assert dev_keys[k] == "tensorboard" and host[k] == "tensorboard", k


def test_wrapped_episode_returns_match_reward_wrapper():
    """``_track_wrapped_returns`` == RewardVecEnvWrapper's per-env running sums over rounds."""
    rng = np.random.default_rng(0)
    T, N = 37, 5
    fake = _FakeRound(None, N=N, T=T)
    carry = np.zeros(N)
    want = collections.deque(maxlen=100)
    for _ in range(4):
        dones = rng.random((T, N)) < 0.08
        rew = rng.standard_normal((T, N)).astype(np.float32)
        before = (sum(want) / len(want)) if want else None
        fake._track_wrapped_returns(dones, rew)
        assert (fake._wrapped_mean_at_start is None) == (before is None)
        if before is not None:
            assert np.isclose(fake._wrapped_mean_at_start, before)
        for t in range(T):  # the wrapper's loop
            carry += rew[t]
            for n in range(N):
                if dones[t, n]:
                    want.append(carry[n])
            carry[dones[t]] = 0
        np.testing.assert_allclose(list(fake._wrapped_eps), list(want), rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(fake._wrapped_cum, carry, rtol=1e-5, atol=1e-5)


def test_explained_variance_from_gae_moments():
    """SB3 explained_variance(values, returns) from the GAE pass's per-env moment sums."""
    rng = np.random.default_rng(1)
    T, N = 64, 8
    rew = th.tensor(rng.standard_normal((T, N)), dtype=th.float32)
    val = th.tensor(rng.standard_normal((T, N)), dtype=th.float32)
    starts = th.tensor(rng.random((T, N)) < 0.05, dtype=th.float32)
    mom = th.zeros(N, 4)
    adv, ret = rl_ops.gae(rew, val, starts, th.zeros(N), th.zeros(N), 0.99, 0.95, moments=mom)
    y, yp = ret.numpy().ravel(), val.numpy().ravel()
    want = 1 - np.var(y - yp) / np.var(y)
    assert np.isclose(rl_ops.explained_variance_from_moments(mom.numpy(), T * N), want, rtol=1e-4)


def test_nonfinite_round_statistics_raise():
    """Fail-fast on the host copy of a round's statistics (no device sync)."""
    import pytest

    from imitation_amd.utils.watchdog import NonFiniteError

    fake = _FakeRound(None)
    fake._global_step = 7
    fake._fail_if_nonfinite({"train/loss": 1.0}, "PPO update")
    with pytest.raises(NonFiniteError, match="round 7.*train/value_loss"):
        fake._fail_if_nonfinite({"train/loss": 1.0, "train/value_loss": float("nan")}, "PPO update")
