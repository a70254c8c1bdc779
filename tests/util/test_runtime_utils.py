"""Tests for imitation_amd.utils: profiling, watchdog, determinism, full-trainer checkpoints."""

import json
import os
import random
import subprocess
import sys
import time

import numpy as np
import pytest
import torch as th

from imitation_amd.utils import checkpoint, determinism, profiling, watchdog


def test_step_timer_reports_throughput():
    t = profiling.StepTimer()
    with t.phase("rollout"):
        time.sleep(0.01)
    with t.phase("rollout"):
        pass
    t.add_env_steps(1000)
    rep = t.report()
    assert rep["env_steps"] == 1000
    assert rep["node_env_steps_per_s"] == rep["rank_env_steps_per_s"] > 0
    assert t.phase_n["rollout"] == 2
    assert rep["phase_s/rollout"] >= 0.01


def test_roctx_range_is_noop_when_disabled():
    profiling.enable_roctx(False)
    with profiling.range("x"):
        pass
    profiling.enable_roctx(True)
    try:
        with profiling.range("phase"):  # works with or without the library
            profiling.mark("m")
    finally:
        profiling.enable_roctx(False)


def test_check_finite():
    watchdog.check_finite({"a": th.ones(3), "b": th.zeros(2)})
    with pytest.raises(watchdog.NonFiniteError, match="b"):
        watchdog.check_finite({"a": th.ones(3), "b": th.tensor([1.0, float("nan")])}, where="loss")
    m = th.nn.Linear(2, 2)
    watchdog.assert_finite_module(m)
    with th.no_grad():
        m.weight[0, 0] = float("inf")
    with pytest.raises(watchdog.NonFiniteError, match="weight"):
        watchdog.assert_finite_module(m)


def test_watchdog_fires_callback():
    fired = []
    wd = watchdog.Watchdog(timeout_s=0.2, poll_s=0.05, on_timeout=lambda: fired.append(1)).start()
    time.sleep(0.6)
    wd.stop()
    assert wd.fired and fired


def test_watchdog_beats_keep_alive():
    wd = watchdog.Watchdog(timeout_s=0.3, poll_s=0.05, on_timeout=lambda: None).start()
    for _ in range(10):
        time.sleep(0.05)
        wd.beat()
    wd.stop()
    assert not wd.fired


def test_watchdog_aborts_process():
    code = ("import time; from imitation_amd.utils.watchdog import Watchdog; "
            "Watchdog(0.2, exit_code=42, poll_s=0.05).start(); time.sleep(5)")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60,
                       cwd=os.path.dirname(os.path.dirname(os.path.dirname(__file__))))
    assert r.returncode == 42
    assert "no heartbeat" in r.stderr


def test_rng_state_roundtrip():
    determinism.seed_everything(3)
    st = determinism.capture_rng_state()
    a = (random.random(), np.random.rand(), th.rand(1).item())
    determinism.restore_rng_state(st)
    b = (random.random(), np.random.rand(), th.rand(1).item())
    assert a == b
    g = np.random.default_rng(5)
    gs = determinism.generator_state(g)
    x = g.random(3)
    determinism.set_generator_state(g, gs)
    np.testing.assert_array_equal(g.random(3), x)


_DEMOS = None


def _small_gail(seed=0):
    from imitation_amd.algorithms.adversarial.gail import GAIL
    from imitation_amd.models import synthetic_demonstrations
    from imitation_amd.policies.base import FeedForward32Policy, NormalizeFeaturesExtractor
    from imitation_amd.rewards.reward_nets import BasicRewardNet, NormalizedRewardNet
    from imitation_amd.rl.ppo import PPO
    from imitation_amd.util import logger as imit_logger
    from imitation_amd.util.networks import RunningNorm
    from imitation_amd.util.util import make_vec_env

    global _DEMOS
    if _DEMOS is None:  # the same demonstrations for every trainer (as on a real restart)
        determinism.seed_everything(1234)
        _DEMOS = synthetic_demonstrations("seals/CartPole-v0", 300, n_envs=2)
    demos = _DEMOS
    determinism.seed_everything(seed)
    venv = make_vec_env("seals/CartPole-v0", rng=np.random.default_rng(seed), n_envs=2)
    gen = PPO(FeedForward32Policy, venv, n_steps=32, batch_size=32, n_epochs=2, seed=seed,
              policy_kwargs=dict(features_extractor_class=NormalizeFeaturesExtractor,
                                 features_extractor_kwargs=dict(normalize_class=RunningNorm)))
    rn = NormalizedRewardNet(BasicRewardNet(venv.observation_space, venv.action_space,
                                            normalize_input_layer=RunningNorm), RunningNorm)
    return GAIL(demonstrations=demos, demo_batch_size=32, venv=venv, gen_algo=gen, reward_net=rn,
                n_disc_updates_per_round=2, custom_logger=imit_logger.configure(format_strs=[]))


def _params(tr):
    return [p.detach().clone() for p in list(tr.gen_algo.policy.parameters()) + list(tr._reward_net.parameters())]


def test_adversarial_checkpoint_resumes_exactly(tmp_path):
    tr = _small_gail()
    tr.train(64)
    ck = checkpoint.save_checkpoint(tr, str(tmp_path / "ck"), meta={"note": "x"})
    meta = json.loads(open(os.path.join(ck, "meta.json")).read())
    assert meta["format"] == "imitation_amd.adversarial.v1" and meta["note"] == "x"
    # the state file is loadable without unpickling arbitrary objects
    th.load(os.path.join(ck, "state.pt"), weights_only=True)
    tr.train(64)
    expect = _params(tr)
    tr2 = _small_gail(seed=99)  # different init / RNG: everything must come from the checkpoint
    checkpoint.load_checkpoint(tr2, ck)
    assert tr2._global_step == 1 and tr2.gen_algo.num_timesteps == tr.gen_algo.num_timesteps - 64
    tr2.train(64)
    for a, b in zip(expect, _params(tr2)):
        th.testing.assert_close(a, b, rtol=0, atol=0)


def test_checkpoint_manager_keeps_latest(tmp_path):
    tr = _small_gail()
    mgr = checkpoint.CheckpointManager(str(tmp_path / "run"), keep=2, rank=0)
    assert mgr.restore_latest(tr) == 0
    for step in (1, 2, 3):
        mgr.save(tr, step)
    assert mgr.list() == [2, 3]
    tr2 = _small_gail(seed=5)
    assert mgr.restore_latest(tr2) == 3
    for a, b in zip(_params(tr), _params(tr2)):
        th.testing.assert_close(a, b, rtol=0, atol=0)
    other = checkpoint.CheckpointManager(str(tmp_path / "run"), keep=2, rank=1)
    assert other.list() == []  # rank shards are separate


def test_rl_algo_checkpoint(tmp_path):
    from imitation_amd.rl.ppo import PPO
    from imitation_amd.util.util import make_vec_env

    venv = make_vec_env("seals/CartPole-v0", rng=np.random.default_rng(0), n_envs=2)
    algo = PPO("MlpPolicy", venv, n_steps=32, batch_size=32, n_epochs=1, seed=0)
    algo.learn(64)
    ck = checkpoint.save_checkpoint(algo, str(tmp_path / "rl"))
    algo.learn(64, reset_num_timesteps=False)
    expect = [p.detach().clone() for p in algo.policy.parameters()]
    algo2 = PPO("MlpPolicy", venv, n_steps=32, batch_size=32, n_epochs=1, seed=3)
    checkpoint.load_checkpoint(algo2, ck)
    algo2.learn(64, reset_num_timesteps=False)
    for a, b in zip(expect, algo2.policy.parameters()):
        th.testing.assert_close(a, b, rtol=0, atol=0)


def test_checkpoint_rejects_unknown_trainer(tmp_path):
    with pytest.raises(TypeError):
        checkpoint.save_checkpoint(object(), str(tmp_path / "bad"))
    assert not os.path.exists(tmp_path / "bad")
