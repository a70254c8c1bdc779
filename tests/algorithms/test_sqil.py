"""SQIL (reference: tests/algorithms/test_sqil.py)."""

import numpy as np
import pytest
import torch as th

from imitation_amd.algorithms import sqil
from imitation_amd.data import rollout
from imitation_amd.rl import dqn, policies, sac


@pytest.fixture
def cartpole_transitions(cartpole_expert_trajectories):
    return rollout.flatten_trajectories(cartpole_expert_trajectories[:4])


@pytest.mark.parametrize("kind", ["transitions", "trajectories"])
def test_sqil_demonstration_buffer(kind, cartpole_venv, cartpole_expert_trajectories, cartpole_transitions):
    demos = cartpole_transitions if kind == "transitions" else cartpole_expert_trajectories[:4]
    model = sqil.SQIL(venv=cartpole_venv, demonstrations=demos, policy="MlpPolicy")
    assert isinstance(model.policy, policies.BasePolicy)
    assert isinstance(model.rl_algo.replay_buffer, sqil.SQILReplayBuffer)
    eb = model.rl_algo.replay_buffer.expert_buffer
    n = len(cartpole_transitions)
    assert len(eb.observations) == n
    for i in (0, 7, n - 1):
        np.testing.assert_array_equal(eb.observations[i, 0].numpy(), cartpole_transitions.obs[i])
        np.testing.assert_array_equal(eb.actions[i, 0].numpy().reshape(-1)[0], cartpole_transitions.acts[i])
        np.testing.assert_array_equal(eb.next_observations[i, 0].numpy(), cartpole_transitions.next_obs[i])
        assert float(eb.dones[i, 0]) == float(cartpole_transitions.dones[i])


def test_sqil_batch_mixes_expert_reward_one(cartpole_venv, cartpole_transitions):
    model = sqil.SQIL(venv=cartpole_venv, demonstrations=cartpole_transitions, policy="MlpPolicy",
                      rl_kwargs=dict(learning_starts=10, batch_size=32))
    model.train(total_timesteps=200)
    batch = model.rl_algo.replay_buffer.sample(32)
    r = batch.rewards.reshape(-1).numpy()
    assert set(np.unique(r)) <= {0.0, 1.0}
    assert r[:16].sum() == 0 and r[16:].sum() == 16  # learner half reward 0, expert half reward 1


def test_sqil_no_crash_discrete(cartpole_venv, cartpole_transitions):
    model = sqil.SQIL(venv=cartpole_venv, demonstrations=cartpole_transitions, policy="MlpPolicy",
                      rl_algo_class=dqn.DQN, rl_kwargs=dict(learning_starts=100))
    model.train(total_timesteps=500)


def test_sqil_no_crash_continuous(pendulum_venv, pendulum_expert_trajectories):
    model = sqil.SQIL(venv=pendulum_venv, demonstrations=rollout.flatten_trajectories(pendulum_expert_trajectories[:2]),
                      policy="MlpPolicy", rl_algo_class=sac.SAC, rl_kwargs=dict(learning_starts=50, batch_size=32))
    model.train(total_timesteps=150)


@pytest.mark.parametrize("illegal_kw", ["replay_buffer_class", "replay_buffer_kwargs"])
def test_sqil_constructor_raises(illegal_kw, cartpole_venv):
    with pytest.raises(ValueError, match=".*SQIL uses a custom replay buffer.*"):
        sqil.SQIL(venv=cartpole_venv, demonstrations=None, policy="MlpPolicy", rl_kwargs={illegal_kw: None})
