"""Fail-fast on NaN/Inf: BC and the DRLHP reward trainer raise
``NonFiniteError`` instead of training on (and logging) NaN for the rest of a run."""

import numpy as np
import pytest
import torch as th

from imitation_amd.algorithms import bc
from imitation_amd.data import rollout
from imitation_amd.utils.watchdog import NonFiniteError


def _poison(module):
    with th.no_grad():
        p = list(module.parameters())[-1]  # an output bias: a NaN there reaches the loss whatever the ReLUs do
        p.view(-1)[0] = float("nan")


def test_bc_nan_policy_raises_at_the_first_logged_batch(cartpole_venv, cartpole_expert_trajectories, rng):
    trainer = bc.BC(observation_space=cartpole_venv.observation_space, action_space=cartpole_venv.action_space, rng=rng,
                    demonstrations=rollout.flatten_trajectories(cartpole_expert_trajectories[:10]), batch_size=32)
    trainer.train(n_batches=2)
    _poison(trainer.policy.action_net)
    with pytest.raises(NonFiniteError, match="BC metrics at batch 0"):
        trainer.train(n_batches=5)


def test_preference_comparisons_nan_reward_model_raises(rng):
    from imitation_amd import models

    b = models.build("preference_walker2d", device="cpu", n_envs=2, n_steps=64, num_iterations=2, fragment_length=10,
                     total_timesteps=256, engine="host")
    _poison(b.trainer.model)
    with pytest.raises(NonFiniteError, match="non-finite (preference probabilities|reward-model loss)"):
        b.trainer.train(256, 40)


@pytest.mark.gpu
def test_fused_cnn_bc_epoch_nan_raises_at_train_end(tmp_path):
    """The graphed device BC epochs (DAgger-Pong learner) check one async finiteness flag per
    epoch: a poisoned learner raises by the end of the train() call."""
    from imitation_amd.engine.dagger import DeviceDemoAggregate, DeviceTransitionsLoader
    from imitation_amd.rl.policies import ActorCriticCnnPolicy
    from imitation_amd.util import logger as ilog
    from imitation_amd.util.util import make_vec_env

    venv = make_vec_env("PongNoFrameskip-v4", rng=np.random.default_rng(0), n_envs=1)
    g = th.Generator(device="cuda").manual_seed(5)
    obs = th.randint(0, 256, (32 * 6, 84, 84, 4), generator=g, device="cuda", dtype=th.int64).to(th.uint8)
    acts = th.randint(0, int(venv.action_space.n), (32 * 6,), generator=g, device="cuda")
    pol = ActorCriticCnnPolicy(venv.observation_space, venv.action_space, lambda _: th.finfo(th.float32).max).cuda()
    agg = DeviceDemoAggregate("cuda")
    agg.append(obs, acts, gather=False)
    trainer = bc.BC(observation_space=venv.observation_space, action_space=venv.action_space,
                    rng=np.random.default_rng(0), policy=pol, batch_size=32, device="cuda",
                    custom_logger=ilog.configure(format_strs=[]))
    trainer.set_demonstrations(DeviceTransitionsLoader(agg, 32, 7))
    trainer.train(n_epochs=1, progress_bar=False, log_interval=10**9)
    _poison(pol.action_net)
    with pytest.raises(NonFiniteError, match="non-finite BC metrics"):
        trainer.train(n_epochs=2, progress_bar=False, log_interval=10**9)


@pytest.mark.gpu
def test_device_preference_nan_reward_model_raises():
    """DRLHP on the device path (fused reward-model minibatches, device agent): a NaN reward model
    ends the iteration with NonFiniteError (no device-side assert, no NaN training)."""
    from imitation_amd import models

    b = models.build("preference_walker2d", device="cuda", n_envs=8, n_steps=128, num_iterations=2, fragment_length=20,
                     total_timesteps=4096, engine="device")
    assert b.extras["engine"] == "device"
    _poison(b.trainer.model)
    with pytest.raises(NonFiniteError, match="non-finite"):
        b.trainer.train(4096, 40)
