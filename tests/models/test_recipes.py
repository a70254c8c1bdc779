"""Model recipes build the headline configurations with the reference's tuned hyper-parameters."""

import numpy as np
import pytest
import torch as th

from imitation_amd import models
from imitation_amd.utils import checkpoint


def test_recipe_registry():
    assert set(models.RECIPES) == {"gail_halfcheetah", "airl_hopper", "dagger_pong", "preference_walker2d", "bc_cartpole"}
    with pytest.raises(KeyError):
        models.build("nope")


def test_gail_halfcheetah_config(tmp_path):
    from imitation_amd.algorithms.adversarial.gail import GAIL

    b = models.build("gail_halfcheetah", n_demo_timesteps=8192, engine="host", log_dir=str(tmp_path))
    tr = b.trainer
    assert isinstance(tr, GAIL)
    assert tr.demo_batch_size == 8192 and tr.n_disc_updates_per_round == 8
    assert tr._gen_replay_buffer.capacity == 512
    g = tr.gen_algo
    assert g.n_steps * g.n_envs == 4096 and g.batch_size == 64 and g.n_epochs == 5
    assert b.env_steps_per_round == 4096
    assert [l.out_features for l in g.policy.mlp_extractor.policy_net if hasattr(l, "out_features")] == [32, 32]
    assert b.venv.observation_space.shape == (17,) and b.venv.action_space.shape == (6,)


def test_airl_hopper_config(tmp_path):
    from imitation_amd.algorithms.adversarial.airl import AIRL
    from imitation_amd.rewards.reward_nets import BasicShapedRewardNet

    b = models.build("airl_hopper", n_demo_timesteps=2048, engine="host", log_dir=str(tmp_path))
    tr = b.trainer
    assert isinstance(tr, AIRL)
    assert isinstance(tr._reward_net.base, BasicShapedRewardNet)
    assert tr.demo_batch_size == 2048 and tr.n_disc_updates_per_round == 16
    g = tr.gen_algo
    assert g.n_steps * g.n_envs == 8192 and g.batch_size == 512 and g.n_epochs == 20
    assert [l.out_features for l in g.policy.mlp_extractor.policy_net if hasattr(l, "out_features")] == [64, 64]


def test_bc_cartpole_trains(tmp_path):
    b = models.build("bc_cartpole", n_demo_timesteps=500, log_dir=str(tmp_path))
    b.trainer.train(n_batches=5)
    assert b.extras["expert"] is not None  # local hub fixture provides the checked-in expert


def test_preference_walker2d_trains_and_checkpoints(tmp_path):
    b = models.build("preference_walker2d", n_envs=2, n_steps=64, num_iterations=2, fragment_length=10,
                     log_dir=str(tmp_path / "log"))
    pc = b.trainer
    pc.train(total_timesteps=256, total_comparisons=20)
    ck = checkpoint.save_checkpoint(pc, str(tmp_path / "ck"))
    st = th.load(f"{ck}/state.pt", weights_only=True)
    assert st["format"] == "imitation_amd.preference_comparisons.v1"
    b2 = models.build("preference_walker2d", n_envs=2, n_steps=64, num_iterations=2, fragment_length=10,
                      log_dir=str(tmp_path / "log2"), seed=3)
    checkpoint.load_checkpoint(b2.trainer, ck)
    assert len(b2.trainer.dataset) == len(pc.dataset) > 0
    assert b2.trainer._iteration == pc._iteration
    for a, c in zip(pc.model.parameters(), b2.trainer.model.parameters()):
        th.testing.assert_close(a, c, rtol=0, atol=0)
    np.testing.assert_array_equal(b2.trainer.dataset.preferences, pc.dataset.preferences)


def test_dagger_pong_builds(tmp_path):
    from imitation_amd.algorithms.dagger import SimpleDAggerTrainer
    from imitation_amd.rl.torch_layers import NatureCNN

    b = models.build("dagger_pong", n_envs=2, scratch_dir=str(tmp_path / "scratch"), log_dir=str(tmp_path / "log"))
    assert isinstance(b.trainer, SimpleDAggerTrainer)
    assert isinstance(b.trainer.bc_trainer.policy.features_extractor, NatureCNN)
    assert b.venv.observation_space.shape == (84, 84, 4)


def test_dp_ranks_get_independent_env_streams(tmp_path):
    """PPO(seed=...) re-seeds the env with the shared seed; the recipe re-seeds per rank so
    the weak-scaled DP batch is made of independent rollouts."""
    obs = []
    for rank in (0, 1, 1):
        b = models.build("gail_halfcheetah", n_demo_timesteps=1024, engine="host", rank=rank,
                         log_dir=str(tmp_path / str(rank)))
        obs.append(np.asarray(b.venv.reset()))
    assert not np.allclose(obs[0], obs[1])
    np.testing.assert_array_equal(obs[1], obs[2])  # still deterministic per rank
