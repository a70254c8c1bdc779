"""SQIL (reference: tests/algorithms/test_sqil.py)."""

import numpy as np
import pytest
import torch as th

from imitation_amd.algorithms import sqil
from imitation_amd.data import rollout
from imitation_amd.rl import dqn, evaluation, policies, sac, td3
from imitation_amd.testing import reward_improvement

RL_ALGOS_CONT_ACTIONS = [td3.DDPG, sac.SAC, td3.TD3]


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


@pytest.fixture
def pendulum_single_venv(rng):
    from imitation_amd.data.wrappers import RolloutInfoWrapper
    from imitation_amd.util.util import make_vec_env

    return make_vec_env("Pendulum-v1", rng=rng, n_envs=1, post_wrappers=[lambda e, _: RolloutInfoWrapper(e)])


@pytest.fixture
def pendulum_transitions(pendulum_expert_trajectories):
    return rollout.flatten_trajectories(pendulum_expert_trajectories)


@pytest.mark.parametrize("rl_algo_class", RL_ALGOS_CONT_ACTIONS)
def test_sqil_no_crash_continuous(pendulum_single_venv, pendulum_transitions, rl_algo_class):
    """Reference ``test_sqil_no_crash_continuous`` (DDPG / SAC / TD3 on Pendulum, 500 steps)."""
    model = sqil.SQIL(venv=pendulum_single_venv, demonstrations=pendulum_transitions, policy="MlpPolicy",
                      rl_algo_class=rl_algo_class, rl_kwargs=dict(batch_size=64))
    model.train(total_timesteps=500)
    assert model.rl_algo.num_timesteps >= 500


def test_sqil_few_demonstrations_discrete(cartpole_venv, cartpole_transitions):
    """Five expert transitions are enough to train (reference ``_test_sqil_few_demonstrations``)."""
    model = sqil.SQIL(venv=cartpole_venv, demonstrations=cartpole_transitions[:5], policy="MlpPolicy",
                      rl_algo_class=dqn.DQN, rl_kwargs=dict(learning_starts=10, seed=42))
    assert len(model.rl_algo.replay_buffer.expert_buffer.observations) == 5
    model.train(total_timesteps=100)


@pytest.mark.parametrize("rl_algo_class", RL_ALGOS_CONT_ACTIONS)
def test_sqil_few_demonstrations_continuous(pendulum_single_venv, pendulum_transitions, rl_algo_class):
    model = sqil.SQIL(venv=pendulum_single_venv, demonstrations=pendulum_transitions[:5], policy="MlpPolicy",
                      rl_algo_class=rl_algo_class, rl_kwargs=dict(seed=42, batch_size=64))
    model.train(total_timesteps=100)


def test_sqil_performance_discrete(cartpole_venv, cartpole_expert_trajectories):
    """Reference ``test_sqil_performance_discrete``: DQN-SQIL on CartPole improves the return
    significantly within 1000 steps (permutation test over 100 episodes before / after)."""
    demos = rollout.flatten_trajectories(cartpole_expert_trajectories)
    model = sqil.SQIL(venv=cartpole_venv, demonstrations=demos, policy="MlpPolicy", rl_algo_class=dqn.DQN,
                      rl_kwargs=dict(learning_starts=500, learning_rate=0.002, batch_size=220, seed=42))
    cartpole_venv.seed(42)
    before, _ = evaluation.evaluate_policy(model.policy, cartpole_venv, 100, return_episode_rewards=True)
    model.train(total_timesteps=1_000)
    cartpole_venv.seed(42)
    after, _ = evaluation.evaluate_policy(model.policy, cartpole_venv, 100, return_episode_rewards=True)
    assert reward_improvement.is_significant_reward_improvement(before, after), (np.mean(before), np.mean(after))


def test_td3_and_ddpg_learn_pendulum_q_targets(pendulum_single_venv):
    """TD3 / DDPG (SB3 semantics) as standalone learners: critics move, the DDPG plan has one
    critic and no target smoothing, TD3 updates the actor every ``policy_delay`` critic steps."""
    for cls, n_critics in ((td3.TD3, 2), (td3.DDPG, 1)):
        algo = cls("MlpPolicy", pendulum_single_venv, learning_starts=50, batch_size=32, seed=0,
                   policy_kwargs=dict(net_arch=[32, 32]))
        assert len(algo.critic.q_networks) == n_critics
        a0 = [p.detach().clone() for p in algo.actor.parameters()]
        t0 = [p.detach().clone() for p in algo.actor_target.parameters()]
        algo.learn(150)
        assert algo._n_updates > 0
        assert any(not th.equal(a, b) for a, b in zip(a0, algo.actor.parameters()))
        # Polyak: the target moved, but less than the online actor
        moved = [float((b.detach() - a).abs().max()) for a, b in zip(t0, algo.actor_target.parameters())]
        online = [float((b.detach() - a).abs().max()) for a, b in zip(a0, algo.actor.parameters())]
        assert max(moved) > 0 and max(moved) < max(online)
        obs = pendulum_single_venv.reset()
        act, _ = algo.predict(obs, deterministic=True)
        assert act.shape == (1, 1) and np.all(np.abs(act) <= 2.0)


@pytest.mark.parametrize("illegal_kw", ["replay_buffer_class", "replay_buffer_kwargs"])
def test_sqil_constructor_raises(illegal_kw, cartpole_venv):
    with pytest.raises(ValueError, match=".*SQIL uses a custom replay buffer.*"):
        sqil.SQIL(venv=cartpole_venv, demonstrations=None, policy="MlpPolicy", rl_kwargs={illegal_kw: None})
