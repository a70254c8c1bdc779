"""DAgger (reference: tests/algorithms/test_dagger.py)."""

import os

import numpy as np
import pytest

from imitation_amd.algorithms import bc, dagger
from imitation_amd.data import rollout
from imitation_amd.testing import reward_improvement


def test_beta_schedules():
    lin = dagger.LinearBetaSchedule(10)
    assert lin(0) == 1.0 and lin(5) == 0.5 and lin(10) == 0.0 and lin(20) == 0.0
    exp = dagger.ExponentialBetaSchedule(0.5)
    assert exp(0) == 1.0 and exp(2) == 0.25
    with pytest.raises(ValueError):
        dagger.ExponentialBetaSchedule(1.5)


def _bc(venv, rng, custom_logger=None):
    return bc.BC(observation_space=venv.observation_space, action_space=venv.action_space, rng=rng,
                 batch_size=32, custom_logger=custom_logger)


def test_trainer_needs_demos(tmp_path, cartpole_venv, rng, custom_logger):
    trainer = dagger.DAggerTrainer(venv=cartpole_venv, scratch_dir=tmp_path, rng=rng, bc_trainer=_bc(cartpole_venv, rng),
                                   custom_logger=custom_logger)
    with pytest.raises(dagger.NeedsDemosException):
        trainer.extend_and_update(dict(n_epochs=1))


def test_trajectory_collector_saves_demos(tmp_path, cartpole_venv, rng):
    """Learner actions are mixed in with prob 1-beta; recorded actions are always the expert's."""
    calls = []

    def robot(obs):
        calls.append(len(obs))
        return np.zeros(len(obs), dtype=np.int64)

    coll = dagger.InteractiveTrajectoryCollector(cartpole_venv, get_robot_acts=robot, beta=0.5, save_dir=tmp_path, rng=rng)
    coll.reset()
    for _ in range(510):
        coll.step(np.ones(cartpole_venv.num_envs, dtype=np.int64))
    files = [f for f in os.listdir(tmp_path) if f.endswith(".npz")]
    assert len(files) >= cartpole_venv.num_envs  # seals CartPole: fixed 500-step episodes
    assert sum(calls) > 0
    from imitation_amd.data import serialize

    traj = serialize.load(tmp_path / files[0])[0]
    assert np.all(traj.acts == 1)


def test_simple_dagger_improves_and_checkpoints(tmp_path, cartpole_venv, cartpole_expert_policy, rng, custom_logger):
    trainer = dagger.SimpleDAggerTrainer(venv=cartpole_venv, scratch_dir=tmp_path, expert_policy=cartpole_expert_policy,
                                         rng=rng, bc_trainer=_bc(cartpole_venv, rng, custom_logger),
                                         beta_schedule=dagger.LinearBetaSchedule(2), custom_logger=custom_logger)
    before = rollout.rollout(trainer.policy, cartpole_venv, rollout.make_min_episodes(10), rng=rng, deterministic_policy=True)
    trainer.train(500 * cartpole_venv.num_envs + 1, rollout_round_min_episodes=1, rollout_round_min_timesteps=500, bc_train_kwargs=dict(n_epochs=3))
    after = rollout.rollout(trainer.policy, cartpole_venv, rollout.make_min_episodes(10), rng=rng, deterministic_policy=True)
    assert trainer.round_num >= 2
    old, new = [t.rews.sum() for t in before], [t.rews.sum() for t in after]
    assert np.mean(new) > np.mean(old) or np.mean(new) > 450
    # checkpoint round trip (weights_only files)
    ckpt, pol = trainer.save_trainer()
    assert ckpt.exists() and pol.exists()
    re = dagger.reconstruct_trainer(tmp_path, cartpole_venv, custom_logger=custom_logger, device="cpu")
    assert isinstance(re, dagger.SimpleDAggerTrainer) and re.round_num == trainer.round_num
    obs = np.stack([cartpole_venv.observation_space.sample() for _ in range(16)]).astype(np.float32)
    np.testing.assert_array_equal(trainer.policy.predict(obs, deterministic=True)[0], re.policy.predict(obs, deterministic=True)[0])
    # resume training from the checkpoint
    re.train(600, rollout_round_min_episodes=1, rollout_round_min_timesteps=500, bc_train_kwargs=dict(n_batches=5))
    assert re.round_num > trainer.round_num


def test_mismatched_expert_spaces(tmp_path, cartpole_venv, rng):
    from imitation_amd.envs import spaces
    from imitation_amd.policies.base import RandomPolicy

    bad = RandomPolicy(spaces.Box(-1, 1, (3,)), cartpole_venv.action_space)
    with pytest.raises(ValueError):
        dagger.SimpleDAggerTrainer(venv=cartpole_venv, scratch_dir=tmp_path, expert_policy=bad, rng=rng,
                                   bc_trainer=_bc(cartpole_venv, rng))
