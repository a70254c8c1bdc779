"""Preference comparisons (reference: tests/algorithms/test_preference_comparisons.py)."""

import re

import numpy as np
import pytest
import torch as th

from imitation_amd.algorithms import preference_comparisons as pc
from imitation_amd.data import types
from imitation_amd.envs import core, spaces
from imitation_amd.envs.vec_env import DummyVecEnv
from imitation_amd.ops import preference as pref_ops
from imitation_amd.regularization import regularizers, updaters
from imitation_amd.rewards import reward_nets
from imitation_amd.rl import evaluation
from imitation_amd.rl.ppo import PPO
from imitation_amd.testing import reward_improvement
from imitation_amd.testing import reward_nets as testing_reward_nets
from imitation_amd.util import util


@pytest.fixture
def venv(rng):
    return util.make_vec_env("seals/CartPole-v0", n_envs=1, rng=rng)


@pytest.fixture(params=["basic", "ensemble", "std_ensemble"])
def reward_net(request, venv):
    o, a = venv.observation_space, venv.action_space
    if request.param == "basic":
        return reward_nets.BasicRewardNet(o, a)
    if request.param == "ensemble":
        return testing_reward_nets.make_ensemble(o, a)
    return reward_nets.AddSTDRewardWrapper(testing_reward_nets.make_ensemble(o, a))


@pytest.fixture
def agent(venv):
    return PPO("MlpPolicy", venv, n_epochs=1, batch_size=2, n_steps=10, device="cpu")


@pytest.fixture
def random_fragmenter(rng):
    return pc.RandomFragmenter(rng=rng, warning_threshold=0)


@pytest.fixture
def agent_trainer(agent, reward_net, venv, rng):
    return pc.AgentTrainer(agent, reward_net, venv, rng)


@pytest.fixture
def preference_model(venv):
    return pc.PreferenceModel(model=reward_nets.BasicRewardNet(venv.observation_space, venv.action_space))


def _traj(n, rews=None, terminal=True, d=4):
    return types.TrajectoryWithRew(obs=np.random.rand(n + 1, d).astype(np.float32), acts=np.zeros(n, np.int64),
                                   infos=None, terminal=terminal,
                                   rews=np.ones(n, np.float32) if rews is None else np.asarray(rews, np.float32))


def test_mismatched_spaces(venv, agent, rng):
    other = util.make_vec_env("Pendulum-v1", n_envs=1, rng=rng)
    bad = reward_nets.BasicRewardNet(other.observation_space, venv.action_space)
    with pytest.raises(ValueError, match="Observation spaces do not match"):
        pc.AgentTrainer(agent, bad, venv, rng)


def test_trajectory_dataset_seeding(rng):
    trajs = [_traj(10) for _ in range(20)]
    s1 = pc.TrajectoryDataset(trajs, np.random.default_rng(0)).sample(100)
    s2 = pc.TrajectoryDataset(trajs, np.random.default_rng(0)).sample(100)
    assert [id(t) for t in s1] == [id(t) for t in s2]
    s3 = pc.TrajectoryDataset(trajs, np.random.default_rng(1)).sample(100)
    assert [id(t) for t in s1] != [id(t) for t in s3]


@pytest.mark.parametrize("num_steps", [0, 199, 200, 201, 400])
def test_trajectory_dataset_len(num_steps, rng):
    ds = pc.TrajectoryDataset([_traj(100) for _ in range(5)], rng)
    trajs = ds.sample(num_steps)
    assert sum(len(t) for t in trajs) >= num_steps
    if num_steps > 0:
        assert sum(len(t) for t in trajs[:-1]) < num_steps


def test_trajectory_dataset_too_long(rng):
    with pytest.raises(RuntimeError, match="Asked for.*but only.* available"):
        pc.TrajectoryDataset([_traj(10)], rng).sample(11)


def test_transitions_left_in_buffer(agent_trainer):
    agent_trainer.venv.reset()
    agent_trainer.venv.step(np.zeros(1, dtype=np.int64))
    with pytest.raises(RuntimeError, match=re.escape("There are 1 transitions left in the buffer.")):
        agent_trainer.train(steps=1)


@pytest.mark.parametrize("schedule", ["constant", "hyperbolic", "inverse_quadratic", lambda t: 1 / (1 + t ** 3)])
def test_preference_comparisons_raises(agent_trainer, reward_net, random_fragmenter, preference_model, custom_logger,
                                       schedule, rng):
    reward_trainer = pc.BasicRewardTrainer(preference_model, pc.CrossEntropyRewardLoss(), rng=rng)
    gatherer = pc.SyntheticGatherer(rng=rng)
    no_rng = ".*don't provide.*random state.*provide.*fragmenter.*preference gatherer.*reward_trainer.*"

    def build(g, t, f, r):
        pc.PreferenceComparisons(agent_trainer, reward_net, num_iterations=2, transition_oversampling=2,
                                 reward_trainer=t, preference_gatherer=g, fragmenter=f, custom_logger=custom_logger,
                                 query_schedule=schedule, rng=r)

    for args in ((gatherer, None, None), (None, reward_trainer, None), (None, None, random_fragmenter)):
        with pytest.raises(ValueError, match=no_rng):
            build(*args, None)
    build(gatherer, reward_trainer, random_fragmenter, None)
    with pytest.raises(ValueError, match="provide.*fragmenter.*preference gatherer.*reward trainer.*don't need.*random state.*"):
        build(gatherer, reward_trainer, random_fragmenter, rng)
    build(None, None, None, rng)
    with pytest.raises(ValueError, match="Unknown query schedule"):
        pc.PreferenceComparisons(agent_trainer, reward_net, num_iterations=2, rng=rng, query_schedule="nope")


@pytest.mark.parametrize("schedule", ["constant", "hyperbolic", "inverse_quadratic", lambda t: 1 / (1 + t ** 3)])
def test_trainer_no_crash(agent_trainer, reward_net, random_fragmenter, custom_logger, schedule, rng):
    th.manual_seed(0)  # the accuracy of 10 tiny comparisons depends on the global torch stream (xdist order)
    main = pc.PreferenceComparisons(agent_trainer, reward_net, num_iterations=2, transition_oversampling=2,
                                    fragment_length=2, fragmenter=random_fragmenter, custom_logger=custom_logger,
                                    query_schedule=schedule, initial_epoch_multiplier=2, rng=rng)
    result = main.train(100, 10)
    assert result["reward_loss"] > 0.0
    assert 0.0 < result["reward_accuracy"] <= 1.0


def test_reward_ensemble_trainer_raises_type_error(venv, rng):
    pm = pc.PreferenceModel(model=reward_nets.BasicRewardNet(venv.observation_space, venv.action_space))
    with pytest.raises(TypeError, match=r"PreferenceModel of a RewardEnsemble expected by EnsembleTrainer."):
        pc.EnsembleTrainer(pm, pc.CrossEntropyRewardLoss(), rng=rng)


def test_correct_reward_trainer_used_by_default(agent_trainer, reward_net, random_fragmenter, custom_logger, rng):
    main = pc.PreferenceComparisons(agent_trainer, reward_net, num_iterations=2, rng=rng, custom_logger=custom_logger)
    base = pc.get_base_model(reward_net)
    if isinstance(base, reward_nets.RewardEnsemble):
        assert isinstance(main.reward_trainer, pc.EnsembleTrainer)
    else:
        assert isinstance(main.reward_trainer, pc.BasicRewardTrainer)


def test_init_raises_error_when_trying_use_improperly_wrapped_ensemble(venv):
    ens = testing_reward_nets.make_ensemble(venv.observation_space, venv.action_space)
    bad = reward_nets.NormalizedRewardNet(ens, reward_nets.networks.RunningNorm)
    with pytest.raises(ValueError, match=r"RewardEnsemble can only be wrapped by AddSTDRewardWrapper"):
        pc.PreferenceModel(bad)


@pytest.mark.parametrize("discount", [0.9, 1.0])
def test_discount_rate_no_crash(agent_trainer, venv, random_fragmenter, custom_logger, rng, discount):
    rn = reward_nets.BasicRewardNet(venv.observation_space, venv.action_space)
    pm = pc.PreferenceModel(rn, discount_factor=discount)
    trainer = pc.BasicRewardTrainer(pm, pc.CrossEntropyRewardLoss(), rng=rng)
    main = pc.PreferenceComparisons(agent_trainer, rn, num_iterations=2, transition_oversampling=2, fragment_length=2,
                                    fragmenter=random_fragmenter, reward_trainer=trainer,
                                    preference_gatherer=pc.SyntheticGatherer(discount_factor=discount, rng=rng),
                                    custom_logger=custom_logger)
    main.train(100, 10)


def test_batched_model_matches_per_pair_reference(venv):
    """The packed single-launch scoring equals the reference per-pair loop."""
    rn = reward_nets.BasicRewardNet(venv.observation_space, venv.action_space)
    pm = pc.PreferenceModel(rn, noise_prob=0.1, discount_factor=0.9, threshold=3.0)
    pairs = [(_traj(5, np.random.rand(5)), _traj(5, np.random.rand(5), terminal=False)) for _ in range(7)]
    probs, gt = pm(pairs)
    from imitation_amd.data import rollout

    for i, (f1, f2) in enumerate(pairs):
        r1 = pm.rewards(rollout.flatten_trajectories([f1]))
        r2 = pm.rewards(rollout.flatten_trajectories([f2]))
        th.testing.assert_close(probs[i], pm.probability(r1, r2), rtol=1e-5, atol=1e-6)
        th.testing.assert_close(gt[i], pm.probability(th.as_tensor(f1.rews), th.as_tensor(f2.rews)), rtol=1e-5, atol=1e-6)
    loss, p2 = pm.loss_and_probs(pairs, np.array([1, 0, 1, 0.5, 1, 0, 0], np.float32))
    th.testing.assert_close(p2, probs, rtol=1e-5, atol=1e-6)
    assert loss.requires_grad


def test_uneven_fragment_lengths(venv):
    rn = reward_nets.BasicRewardNet(venv.observation_space, venv.action_space)
    pm = pc.PreferenceModel(rn)
    pairs = [(_traj(3), _traj(6)), (_traj(4), _traj(2))]
    probs, _ = pm(pairs)
    from imitation_amd.data import rollout

    for i, (f1, f2) in enumerate(pairs):
        r1 = pm.rewards(rollout.flatten_trajectories([f1]))
        r2 = pm.rewards(rollout.flatten_trajectories([f2]))
        th.testing.assert_close(probs[i], pm.probability(r1.sum(0, keepdim=True), r2.sum(0, keepdim=True)), rtol=1e-5,
                                atol=1e-6)


@pytest.mark.parametrize("discount,noise,thr", [(1.0, 0.0, 50.0), (0.9, 0.1, 2.0)])
def test_bradley_terry_reference_gradients(discount, noise, thr):
    """Analytic backward used by the kernel == autograd of the reference formula."""
    r1 = th.randn(6, 9, dtype=th.float64, requires_grad=True)
    r2 = th.randn(6, 9, dtype=th.float64, requires_grad=True)
    prefs = th.tensor([1, 0, 0.5, 1, 0, 1], dtype=th.float64)
    loss, probs = pref_ops.bradley_terry_reference(r1, r2, prefs, discount, thr, noise)
    g1, g2 = th.autograd.grad(loss, (r1, r2))
    disc = discount ** th.arange(9, dtype=th.float64)
    diff = (disc * (r2 - r1)).sum(-1)
    inside = (diff.abs() <= thr).double()
    pm = 1 / (1 + th.clip(diff, -thr, thr).exp())
    p = noise / 2 + (1 - noise) * pm
    coef = (p - prefs) / (p * (1 - p)) * (-(1 - noise) * pm * (1 - pm)) * inside / 6
    th.testing.assert_close(g2, coef[:, None] * disc[None, :])
    th.testing.assert_close(g1, -coef[:, None] * disc[None, :])


def test_gradient_accumulation(agent_trainer, venv, random_fragmenter, rng):
    """minibatch accumulation == large batch (reference :468-518)."""
    th.manual_seed(0)
    rn1 = reward_nets.BasicRewardNet(venv.observation_space, venv.action_space)
    rn2 = reward_nets.BasicRewardNet(venv.observation_space, venv.action_space)
    rn2.load_state_dict(rn1.state_dict())
    trajs = agent_trainer.sample(200)
    frags = random_fragmenter(trajs, 4, 16)
    prefs = pc.SyntheticGatherer(rng=rng)(frags)
    ds = pc.PreferenceDataset()
    ds.push(frags, prefs)
    t1 = pc.BasicRewardTrainer(pc.PreferenceModel(rn1), pc.CrossEntropyRewardLoss(), rng=np.random.default_rng(0),
                               batch_size=16)
    t2 = pc.BasicRewardTrainer(pc.PreferenceModel(rn2), pc.CrossEntropyRewardLoss(), rng=np.random.default_rng(0),
                               batch_size=16, minibatch_size=4)
    # same order: no shuffle difference matters for a single full batch
    t1.train(ds)
    t2.train(ds)
    # The output bias cancels in every return difference (its gradient is ~1e-8 noise that
    # Adam's normalisation amplifies), so it is excluded from the comparison.
    params = list(zip(rn1.parameters(), rn2.parameters()))[:-1]
    for p1, p2 in params:
        np.testing.assert_allclose(p1.detach().numpy(), p2.detach().numpy(), atol=1e-5, rtol=1e-4)


def test_synthetic_gatherer_deterministic(agent_trainer, random_fragmenter, rng):
    g = pc.SyntheticGatherer(temperature=0, rng=rng)
    frags = random_fragmenter(agent_trainer.sample(10), fragment_length=2, num_pairs=2)
    p1 = g(frags)
    assert np.all(p1 == g(frags))
    assert set(np.unique(p1)) <= {0.0, 0.5, 1.0}


def test_synthetic_gatherer_raises():
    with pytest.raises(ValueError, match="If `sample` is True, then `rng` must be provided"):
        pc.SyntheticGatherer(temperature=0, sample=True)


def test_fragments_terminal(rng):
    fragmenter = pc.RandomFragmenter(rng=rng, warning_threshold=0)
    trajs = [types.TrajectoryWithRew(obs=np.arange(4)[:, None], acts=np.zeros(3), infos=None, terminal=True,
                                     rews=np.zeros(3, np.float32)),
             types.TrajectoryWithRew(obs=np.arange(4)[:, None] + 10, acts=np.zeros(3), infos=None, terminal=False,
                                     rews=np.zeros(3, np.float32))]
    for _ in range(5):
        for f1, f2 in fragmenter(trajs, fragment_length=2, num_pairs=2):
            for f in (f1, f2):
                if f.obs[-1, 0] == 3:
                    assert f.terminal
                else:
                    assert not f.terminal


def test_fragments_too_short_error(agent_trainer):
    with pytest.raises(ValueError, match="No trajectories are long enough for the desired fragment length of 1000."):
        pc.RandomFragmenter(rng=np.random.default_rng(0), warning_threshold=0)(agent_trainer.sample(2), 1000, 2)


def test_preference_dataset_errors(agent_trainer, random_fragmenter):
    ds = pc.PreferenceDataset()
    frags = random_fragmenter(agent_trainer.sample(10), 2, 2)
    with pytest.raises(ValueError, match="Unexpected preferences shape"):
        ds.push(frags, np.array([0.5], np.float32))
    with pytest.raises(ValueError, match="preferences should have dtype float32"):
        ds.push(frags, np.array([0.5, 0.5]))


def test_preference_dataset_queue(agent_trainer, random_fragmenter, rng):
    ds = pc.PreferenceDataset(max_size=5)
    gatherer = pc.SyntheticGatherer(rng=rng)
    for i in range(6):
        frags = random_fragmenter(agent_trainer.sample(10), 2, 1)
        ds.push(frags, gatherer(frags))
        assert len(ds) == min(i + 1, 5)


def test_store_and_load_preference_dataset(agent_trainer, random_fragmenter, rng, tmp_path):
    ds = pc.PreferenceDataset()
    frags = random_fragmenter(agent_trainer.sample(10), 2, 2)
    prefs = pc.SyntheticGatherer(rng=rng)(frags)
    ds.push(frags, prefs)
    ds.save(tmp_path / "prefs.npz")
    loaded = pc.PreferenceDataset.load(tmp_path / "prefs.npz")
    assert len(loaded) == len(ds)
    for (a1, a2), pa in (ds[i] for i in range(len(ds))):
        pass
    for i in range(len(ds)):
        (f1, f2), p = ds[i]
        (g1, g2), q = loaded[i]
        assert f1 == g1 and f2 == g2 and p == q


def test_exploration_no_crash(agent, reward_net, venv, random_fragmenter, custom_logger, rng):
    at = pc.AgentTrainer(agent, reward_net, venv, exploration_frac=0.5, rng=rng)
    main = pc.PreferenceComparisons(at, reward_net, num_iterations=2, transition_oversampling=2, fragment_length=5,
                                    fragmenter=random_fragmenter, custom_logger=custom_logger, rng=rng)
    main.train(100, 10)


@pytest.mark.parametrize("uncertainty_on", ["logit", "probability", "label"])
def test_active_fragmenter_discount_rate_no_crash(agent_trainer, venv, random_fragmenter, uncertainty_on, custom_logger,
                                                  rng):
    ens = testing_reward_nets.make_ensemble(venv.observation_space, venv.action_space)
    pm = pc.PreferenceModel(ens, discount_factor=0.9)
    fragmenter = pc.ActiveSelectionFragmenter(preference_model=pm, base_fragmenter=random_fragmenter,
                                              fragment_sample_factor=2, uncertainty_on=uncertainty_on,
                                              custom_logger=custom_logger)
    main = pc.PreferenceComparisons(agent_trainer, ens, num_iterations=2, transition_oversampling=2, fragment_length=2,
                                    fragmenter=fragmenter, preference_gatherer=pc.SyntheticGatherer(rng=rng),
                                    reward_trainer=pc.EnsembleTrainer(pm, pc.CrossEntropyRewardLoss(), rng=rng),
                                    custom_logger=custom_logger)
    main.train(100, 10)


def test_active_fragmenter_matches_per_pair_estimates(agent_trainer, venv, random_fragmenter):
    ens = testing_reward_nets.make_ensemble(venv.observation_space, venv.action_space, 3)
    pm = pc.PreferenceModel(ens)
    frags = random_fragmenter(agent_trainer.sample(40), 4, 6)
    from imitation_amd.data import rollout

    for unc in ("logit", "probability", "label"):
        af = pc.ActiveSelectionFragmenter(pm, random_fragmenter, 1.0, uncertainty_on=unc)
        with th.no_grad():
            r1, r2 = pm.pair_rewards(frags)
        batched = af.variance_estimates(r1, r2)
        for i, (f1, f2) in enumerate(frags):
            a = pm.rewards(rollout.flatten_trajectories([f1]))
            b = pm.rewards(rollout.flatten_trajectories([f2]))
            assert batched[i] == pytest.approx(af.variance_estimate(a, b), rel=1e-4, abs=1e-6)


def test_active_selection_errors(venv, random_fragmenter):
    pm = pc.PreferenceModel(reward_nets.BasicRewardNet(venv.observation_space, venv.action_space))
    with pytest.raises(ValueError, match="PreferenceModel not wrapped over an ensemble"):
        pc.ActiveSelectionFragmenter(pm, random_fragmenter, 2)
    pm2 = pc.PreferenceModel(testing_reward_nets.make_ensemble(venv.observation_space, venv.action_space))
    with pytest.raises(ValueError, match="not supported"):
        pc.ActiveSelectionFragmenter(pm2, random_fragmenter, 2, uncertainty_on="zzz")


def test_reward_trainer_regularization_no_crash(agent_trainer, venv, random_fragmenter, custom_logger, rng):
    rn = reward_nets.BasicRewardNet(venv.observation_space, venv.action_space)
    pm = pc.PreferenceModel(rn)
    factory = regularizers.LpRegularizer.create(initial_lambda=0.1, val_split=0.2, p=2,
                                                lambda_updater=updaters.IntervalParamScaler(0.1, (0.9, 1.1)))
    trainer = pc.BasicRewardTrainer(pm, pc.CrossEntropyRewardLoss(), rng=rng, regularizer_factory=factory,
                                    custom_logger=custom_logger)
    main = pc.PreferenceComparisons(agent_trainer, rn, num_iterations=2, transition_oversampling=2, fragment_length=2,
                                    fragmenter=random_fragmenter, reward_trainer=trainer,
                                    preference_gatherer=pc.SyntheticGatherer(rng=rng), custom_logger=custom_logger)
    main.train(50, 50)


def test_reward_trainer_regularization_raises(agent_trainer, venv, random_fragmenter, custom_logger, rng):
    rn = reward_nets.BasicRewardNet(venv.observation_space, venv.action_space)
    factory = regularizers.LpRegularizer.create(initial_lambda=0.1, val_split=0.1, p=2,
                                                lambda_updater=updaters.IntervalParamScaler(0.1, (0.9, 1.1)))
    trainer = pc.BasicRewardTrainer(pc.PreferenceModel(rn), pc.CrossEntropyRewardLoss(), rng=rng,
                                    regularizer_factory=factory, custom_logger=custom_logger)
    main = pc.PreferenceComparisons(agent_trainer, rn, num_iterations=2, transition_oversampling=2, fragment_length=2,
                                    fragmenter=random_fragmenter, reward_trainer=trainer,
                                    preference_gatherer=pc.SyntheticGatherer(rng=rng), custom_logger=custom_logger)
    with pytest.raises(ValueError, match="Not enough data samples to split into training and validation"):
        main.train(100, 10)


def test_agent_trainer_sample(venv, agent_trainer):
    trajectories = agent_trainer.sample(2)
    assert len(trajectories) > 0
    assert all(t.obs.shape[1:] == venv.observation_space.shape for t in trajectories)


class ActionIsRewardEnv(core.Env):
    """Two-step env whose reward is the action."""

    def __init__(self):
        self.action_space = spaces.Discrete(50)
        self.observation_space = spaces.Box(np.array([0.0]), np.array([1.0]))
        self.steps = 0

    def step(self, action):
        done = self.steps > 0
        self.steps += 1
        return np.array([0.0], np.float32), float(action), done, False, {}

    def reset(self, *, seed=None, options=None):
        self.steps = 0
        return np.array([0.0], np.float32), {}


def _basic_trainer(venv, rng):
    rn = reward_nets.BasicRewardNet(venv.observation_space, venv.action_space)
    return pc.BasicRewardTrainer(pc.PreferenceModel(rn, noise_prob=0.1, discount_factor=0.9, threshold=50),
                                 pc.CrossEntropyRewardLoss(), rng=rng, lr=1e-4)


def _ensemble_trainer(venv, rng):
    ens = reward_nets.RewardEnsemble(venv.observation_space, venv.action_space,
                                     members=[reward_nets.BasicRewardNet(venv.observation_space, venv.action_space)
                                              for _ in range(3)])
    return pc.EnsembleTrainer(pc.PreferenceModel(ens, noise_prob=0.1, discount_factor=0.9, threshold=50),
                              pc.CrossEntropyRewardLoss(), rng=rng, lr=1e-4)


@pytest.mark.parametrize("make_trainer", [_basic_trainer, _ensemble_trainer])
def test_that_trainer_improves(make_trainer, random_fragmenter, custom_logger, rng):
    venv = DummyVecEnv([ActionIsRewardEnv])
    th.manual_seed(0)
    agent = PPO("MlpPolicy", venv, n_epochs=1, batch_size=2, n_steps=10, device="cpu", seed=0)
    trainer = make_trainer(venv, rng)
    at = pc.AgentTrainer(agent, trainer._preference_model.model, venv, rng)
    main = pc.PreferenceComparisons(at, trainer._preference_model.model, num_iterations=2, transition_oversampling=2,
                                    fragment_length=2, fragmenter=random_fragmenter, rng=rng, reward_trainer=trainer,
                                    custom_logger=custom_logger)
    novice, _ = evaluation.evaluate_policy(agent.policy, venv, 50, return_episode_rewards=True)
    first = main.train(20, 20)
    later = main.train(100, 40)
    assert first["reward_loss"] > later["reward_loss"]
    trained, _ = evaluation.evaluate_policy(agent.policy, venv, 50, return_episode_rewards=True)
    assert reward_improvement.is_significant_reward_improvement(novice, trained)


@pytest.mark.parametrize("minibatch", [None, 5])
def test_device_resident_reward_training_matches_generic_loop(agent_trainer, venv, random_fragmenter, rng, monkeypatch,
                                                              minibatch):
    """BasicRewardTrainer's packed fast path == the per-minibatch DataLoader loop: same
    shuffling, accumulation, parameters and logged means."""
    from imitation_amd.util import logger as imit_logger

    th.manual_seed(0)
    trajs = agent_trainer.sample(200)
    frags = random_fragmenter(trajs, 4, 21)
    prefs = pc.SyntheticGatherer(rng=rng)(frags)
    ds = pc.PreferenceDataset()
    ds.push(frags, prefs)
    out = []
    for fast in ("0", "1"):
        monkeypatch.setenv("IMITATION_AMD_PREF_FAST", fast)
        th.manual_seed(1)
        rn = reward_nets.BasicRewardNet(venv.observation_space, venv.action_space)
        log = imit_logger.configure(format_strs=[])
        tr = pc.BasicRewardTrainer(pc.PreferenceModel(rn), pc.CrossEntropyRewardLoss(), rng=np.random.default_rng(3),
                                   batch_size=10, minibatch_size=minibatch, epochs=3, custom_logger=log)
        assert tr._fast_path_ok(ds) == (fast == "1")
        tr.train(ds)
        out.append(([p.detach().clone() for p in rn.parameters()], dict(log.name_to_value)))
    (p0, l0), (p1, l1) = out
    for a, b in zip(p0[:-1], p1[:-1]):
        th.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)
    assert set(l0) == set(l1)
    for k in l0:
        assert l1[k] == pytest.approx(l0[k], rel=1e-4, abs=1e-5), k


def test_batched_ensemble_trainer_equals_member_loop(monkeypatch):
    """All members in one grouped step == the reference's member-by-member bagged training
    (same bags, orders, accumulation, RunningNorm updates; same logged keys)."""
    from imitation_amd.envs import spaces
    from imitation_amd.rewards.reward_nets import BasicRewardNet, RewardEnsemble
    from imitation_amd.testing.dist_workers import _pref_dataset
    from imitation_amd.util import logger
    from imitation_amd.util.networks import RunningNorm

    results = []
    for batched in ("1", "0"):
        monkeypatch.setenv("IMITATION_AMD_ENSEMBLE_BATCHED", batched)
        th.manual_seed(0)
        obs, act = spaces.Box(-1, 1, (5,)), spaces.Box(-1, 1, (2,))
        ens = RewardEnsemble(obs, act, [BasicRewardNet(obs, act, normalize_input_layer=RunningNorm) for _ in range(3)])
        assert ens.stack() is not None
        log = logger.configure(format_strs=[])
        tr = pc.EnsembleTrainer(pc.PreferenceModel(ens),
                                                    pc.CrossEntropyRewardLoss(),
                                                    rng=np.random.default_rng(4), batch_size=8, epochs=2, lr=1e-3,
                                                    custom_logger=log)
        ds = _pref_dataset(21, 5, 1)
        assert tr._batched_ok(ds) == (batched == "1")
        tr.train(ds)
        tr.train(ds, epoch_multiplier=1.5)  # persistent stacked optimizer state across calls
        keys = sorted(k for k in log.name_to_value if "final" in k)
        # Biases are compared through the rewards they produce: the Bradley-Terry loss only
        # sees reward differences (output bias) and dead ReLU units only get rounding-noise
        # gradients (hidden biases) -- Adam normalises such noise into lr-sized steps.
        named = [(k, t.detach().clone()) for k, t in ens.named_parameters() if not k.endswith("bias")]
        g = th.Generator().manual_seed(9)
        s_, a_ = th.randn(64, 5, generator=g), th.randn(64, 2, generator=g)
        with th.no_grad():
            r = th.stack([m(s_, a_, s_, th.zeros(64)) for m in ens.members])
        named.append(("reward_diffs", r - r[:, :1]))
        results.append((named + [(k, b.clone()) for k, b in ens.named_buffers()], keys,
                        {k: log.name_to_value[k] for k in keys}))
    (pa, ka, va), (pb, kb, vb) = results
    assert ka == kb and len(ka) > 0
    for (na, a), (nb, b) in zip(pa, pb):
        assert na == nb
        th.testing.assert_close(a.float(), b.float(), rtol=1e-3, atol=1e-4, msg=na)
    for k in ka:
        assert abs(va[k] - vb[k]) < 1e-4 * max(1.0, abs(vb[k])), (k, va[k], vb[k])


def test_ensemble_grouped_prediction_matches_members():
    from imitation_amd.envs import spaces
    from imitation_amd.rewards.reward_nets import BasicRewardNet, RewardEnsemble
    from imitation_amd.util.networks import RunningNorm

    th.manual_seed(0)
    obs, act = spaces.Box(-1, 1, (5,)), spaces.Box(-1, 1, (2,))
    ens = RewardEnsemble(obs, act, [BasicRewardNet(obs, act, normalize_input_layer=RunningNorm) for _ in range(4)])
    ens.eval()  # members' RunningNorms must not update during the reference forward
    for m in ens.members:  # non-trivial normalisation statistics
        m.mlp.normalize_input.update_stats(th.randn(50, 7) * 3 + 1)
    st = ens.stack()
    s, a = th.randn(9, 5), th.randn(9, 2)
    x = st.features(s, a, s, th.zeros(9))
    with th.no_grad():
        y = st.forward(x, st.gather_params(), st.gather_norm())
        ref = th.stack([m(s, a, s, th.zeros(9)) for m in ens.members])
    th.testing.assert_close(y, ref, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("P,B", [(500, 32), (7, 3), (64, 64), (1, 1)])
def test_epoch_orders_replay_the_dataloader(P, B):
    """_epoch_orders (the fused reward training's upfront epoch permutations) equals iterating
    the shuffling DataLoader epoch by epoch, and leaves its generator in the same state."""
    import torch as th
    from torch.utils import data as data_th

    from imitation_amd.algorithms.preference_comparisons import _epoch_orders

    mk = lambda: data_th.DataLoader(range(P), batch_size=B, shuffle=True,  # noqa: E731
                                    generator=th.Generator().manual_seed(123))
    fast_loader, ref_loader = mk(), mk()
    fast = _epoch_orders(fast_loader, P, 6) + [th.cat(list(fast_loader))]
    ref = [th.cat(list(ref_loader)) for _ in range(7)]
    assert all(th.equal(a, b) for a, b in zip(fast, ref))


def test_trajectory_dataset_not_static(cartpole_expert_trajectories, rng, num_steps: int = 400):
    """TrajectoryDataset.sample() does not always return the same trajectories
    (reference ``test_trajectory_dataset_not_static``)."""
    import math

    dataset = pc.TrajectoryDataset(cartpole_expert_trajectories, rng)
    flakiness_prob = 1 / len(cartpole_expert_trajectories)
    max_samples = math.ceil(math.log(1e-6) / math.log(flakiness_prob))
    sample = dataset.sample(num_steps)

    def same(a, b):
        return len(a) == len(b) and all(np.array_equal(x.obs, y.obs) and np.array_equal(x.acts, y.acts) for x, y in zip(a, b))

    assert not all(same(sample, dataset.sample(num_steps)) for _ in range(max_samples))


def test_agent_trainer_populates_buffer(agent_trainer):
    agent_trainer.train(steps=1)
    assert agent_trainer.buffering_wrapper.n_transitions > 0


class _FakeImageEnv(core.Env):
    """Channels-last uint8 frames, 10-step episodes (SB3's FakeImageEnv, which the reference uses)."""

    def __init__(self):
        self.observation_space = spaces.Box(low=0, high=255, shape=(12, 16, 3), dtype=np.uint8)
        self.action_space = spaces.Discrete(2)
        self._rng = np.random.default_rng(0)
        self._t = 0

    def _obs(self):
        return self._rng.integers(0, 256, self.observation_space.shape, dtype=np.uint8)

    def step(self, action):
        self._t += 1
        return self._obs(), 0.0, self._t >= 10, False, {}

    def reset(self, *, seed=None, options=None):
        self._t = 0
        return self._obs(), {}


def test_agent_trainer_sample_image_observations(rng):
    """AgentTrainer.sample() in an image env returns observations in the env's own layout even
    if the RL algorithm transposes image channels (reference test of the same name)."""
    venv = DummyVecEnv([_FakeImageEnv])
    reward_net = reward_nets.BasicRewardNet(venv.observation_space, venv.action_space)
    agent = PPO("MlpPolicy", venv, n_epochs=1, batch_size=2, n_steps=10, device="cpu")
    agent_trainer = pc.AgentTrainer(agent, reward_net, venv, exploration_frac=0.5, rng=rng)
    trajectories = agent_trainer.sample(2)
    assert len(trajectories) > 0
    assert all(t.obs.shape[1:] == venv.observation_space.shape for t in trajectories)


def test_active_fragmenter_uncertainty_on_not_supported_error(venv, random_fragmenter):
    ensemble = pc.PreferenceModel(testing_reward_nets.make_ensemble(venv.observation_space, venv.action_space))
    with pytest.raises(ValueError, match=r".* not supported\.\n\s+`uncertainty_on` should be from .*"):
        pc.ActiveSelectionFragmenter(preference_model=ensemble, base_fragmenter=random_fragmenter,
                                     fragment_sample_factor=2, uncertainty_on="uncertainty_on")


def test_active_selection_raises_error_when_initialized_without_an_ensemble(preference_model, random_fragmenter):
    with pytest.raises(ValueError, match=r"PreferenceModel not wrapped over an ensemble.*"):
        pc.ActiveSelectionFragmenter(preference_model=preference_model, base_fragmenter=random_fragmenter,
                                     fragment_sample_factor=2, uncertainty_on="logit")


def test_random_fragmenter_draws_as_rng_choice():
    """The fragmenter's inverse-CDF draw consumes the RNG exactly as ``rng.choice(n, p=p)`` (the
    reference's call): same fragments, same order, validated-slice contents and terminal flags."""
    from imitation_amd.algorithms.preference_comparisons import RandomFragmenter

    rng = np.random.default_rng(0)
    trajs = [
        types.TrajectoryWithRew(obs=rng.standard_normal((L + 1, 3)).astype(np.float32),
                                acts=rng.standard_normal((L, 2)).astype(np.float32), infos=None,
                                terminal=bool(i % 2), rews=rng.standard_normal(L).astype(np.float32))
        for i, L in enumerate(rng.integers(50, 400, size=40))
    ]
    frags = [f for pair in RandomFragmenter(np.random.default_rng(7), warning_threshold=0)(trajs, 50, 300) for f in pair]
    ref_rng = np.random.default_rng(7)
    weights = np.array([len(t) for t in trajs], dtype=np.float64)
    for f in frags:
        t = trajs[int(ref_rng.choice(len(trajs), p=weights / weights.sum()))]
        s = int(ref_rng.integers(0, len(t) - 50, endpoint=True))
        want = types.TrajectoryWithRew(obs=t.obs[s:s + 51], acts=t.acts[s:s + 50], infos=None, rews=t.rews[s:s + 50],
                                       terminal=(s + 50 == len(t)) and t.terminal)
        assert f == want and f.terminal == want.terminal and len(f) == 50


@pytest.mark.parametrize("gamma", [1.0, 0.99, 0.9])
def test_synthetic_gatherer_batched_returns_are_bitwise_the_per_fragment_sums(gamma):
    """The batched Horner evaluation over equal-length fragments == ``rollout.discounted_sum``
    (numpy ``polyval``) fragment by fragment, bit for bit; mixed lengths take the per-fragment path."""
    from imitation_amd.algorithms.preference_comparisons import _batched_discounted_sums
    from imitation_amd.data import rollout

    rng = np.random.default_rng(3)

    def frag(L):
        return types.TrajectoryWithRew(obs=np.zeros((L + 1, 2), np.float32), acts=np.zeros((L, 1), np.float32), infos=None,
                                       terminal=False, rews=(rng.standard_normal(L) * 7).astype(np.float32))

    pairs = [(frag(40), frag(40)) for _ in range(64)]
    r1, r2 = _batched_discounted_sums(pairs, gamma)
    want1 = np.array([rollout.discounted_sum(a.rews, gamma) for a, _ in pairs], np.float32)
    want2 = np.array([rollout.discounted_sum(b.rews, gamma) for _, b in pairs], np.float32)
    assert np.array_equal(r1, want1) and np.array_equal(r2, want2)
    assert _batched_discounted_sums([(frag(40), frag(41))], gamma) is None
