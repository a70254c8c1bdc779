"""Ready-to-train model recipes for the headline configurations (BASELINE.json ``configs``).

Each recipe builds the *whole* training setup -- vector env, networks of the
reference's architecture with its tuned hyper-parameters
(``src/imitation/scripts/config/tuned_hps/*.json``, mirrored in
``imitation_amd/scripts/config/tuned_hps.json``), demonstrations and the algorithm
object -- so ``bench.py``, ``__graft_entry__.smoke`` and users share one definition:

=======================  ==========================================================
``gail_halfcheetah``     GAIL, seals/HalfCheetah, PPO ``FeedForward32Policy`` +
                         RunningNorm features, ``BasicRewardNet`` in
                         ``NormalizedRewardNet``; device engine when eligible
``airl_hopper``          AIRL, seals/Hopper, PPO MLP [64, 64] ReLU, shaped reward
``dagger_pong``          DAgger, Pong (84x84x4 frames), ``ActorCriticCnnPolicy``
                         with the NatureCNN extractor
``preference_walker2d``  preference comparisons (DRLHP), seals/Walker2d
``bc_cartpole``          BC, CartPole-v1
=======================  ==========================================================

There is no network access, so "expert" demonstrations are synthetic: rollouts of a
random-init policy of the same env (or the checked-in CartPole expert when the local
expert hub has it). Weights are random-init. Recipes accept ``**overrides`` that are
forwarded to the algorithm constructor.
"""

from __future__ import annotations

import dataclasses
import os
import tempfile
from typing import Any, Callable, Dict, Optional

import numpy as np
import torch as th

from imitation_amd.data import rollout, types


@dataclasses.dataclass
class Built:
    """What a recipe returns."""

    trainer: Any
    venv: Any
    name: str
    env_id: str
    env_steps_per_round: int
    extras: Dict[str, Any] = dataclasses.field(default_factory=dict)


def _tuned(key: str) -> Dict[str, Any]:
    from imitation_amd.scripts.config import tuned_hps

    return tuned_hps()[key]


def _device(device) -> th.device:
    if device is None:
        return th.device("cuda" if th.cuda.is_available() else "cpu")
    return th.device(device)


def synthetic_demonstrations(env_id: str, min_timesteps: int, seed: int = 12345, n_envs: int = 16,
                             policy=None) -> types.Transitions:
    """Flat transitions from ``policy`` (random if None) on ``env_id`` -- the stand-in for
    the reference's HuggingFace expert rollouts."""
    from imitation_amd.util.util import make_vec_env

    env = make_vec_env(env_id, rng=np.random.default_rng(seed), n_envs=n_envs)
    trajs = rollout.generate_trajectories(policy, env, rollout.make_min_timesteps(min_timesteps),
                                          rng=np.random.default_rng(seed + 1))
    return rollout.flatten_trajectories(trajs)


def _reseed_rank(venv, seed: int, rank: int) -> None:
    """``PPO(seed=seed)`` re-seeds the env (and the global RNGs) with the seed shared by all
    ranks; give every data-parallel rank its own env reset streams and RNG state again, so
    the weak-scaled global batch is made of independent rollouts."""
    if rank:
        from imitation_amd.rl.base import set_random_seed

        venv.seed(seed + 1000 * rank)
        set_random_seed(seed + rank, using_cuda=th.cuda.is_available())


def _logger(log_dir: Optional[str]):
    from imitation_amd.util import logger as imit_logger

    d = log_dir or tempfile.mkdtemp(prefix="ia_recipe_")
    return imit_logger.configure(d, format_strs=[])


def gail_halfcheetah(device=None, n_envs: int = 8, engine: str = "auto", seed: int = 0, rank: int = 0,
                     env_id: str = "seals/HalfCheetah-v1", demonstrations: Optional[types.Transitions] = None,
                     n_demo_timesteps: int = 16384, log_dir: Optional[str] = None, **overrides) -> Built:
    """GAIL on HalfCheetah with the reference's tuned ``gail_seals_half_cheetah`` config:
    rl batch 4096 (split over ``n_envs``), minibatch 64, 5 epochs, clip 0.1, demo batch 8192,
    replay capacity 512, 8 discriminator updates per round."""
    from imitation_amd.algorithms.adversarial.gail import GAIL
    from imitation_amd.rewards.reward_nets import BasicRewardNet, NormalizedRewardNet
    from imitation_amd.rl.ppo import PPO
    from imitation_amd.policies.base import FeedForward32Policy, NormalizeFeaturesExtractor
    from imitation_amd.util.networks import RunningNorm
    from imitation_amd.util.util import make_vec_env

    hp = _tuned("gail_seals_half_cheetah")
    dev = _device(device)
    venv = make_vec_env(env_id, rng=np.random.default_rng(seed + 1000 * rank), n_envs=n_envs)
    if demonstrations is None:
        demonstrations = synthetic_demonstrations(env_id, n_demo_timesteps)
    rl_kwargs = dict(hp["rl"]["rl_kwargs"])
    n_steps = hp["rl"]["batch_size"] // n_envs
    policy_kwargs = dict(features_extractor_class=NormalizeFeaturesExtractor,
                         features_extractor_kwargs=dict(normalize_class=RunningNorm))
    gen = PPO(FeedForward32Policy, venv, n_steps=n_steps, policy_kwargs=policy_kwargs, device=dev, seed=seed, **rl_kwargs)
    _reseed_rank(venv, seed, rank)
    reward_net = NormalizedRewardNet(
        BasicRewardNet(venv.observation_space, venv.action_space, normalize_input_layer=RunningNorm), RunningNorm)
    algo_kwargs = dict(hp["algorithm_kwargs"])
    algo_kwargs.update(overrides)
    kw = dict(demonstrations=demonstrations, venv=venv, gen_algo=gen, reward_net=reward_net,
              custom_logger=_logger(log_dir), **algo_kwargs)
    cls = GAIL
    if engine in ("auto", "device"):
        from imitation_amd.engine import gail as device_gail

        ok, why = device_gail.supports(venv, gen, reward_net)
        if ok:
            cls = device_gail.DeviceGAIL
        elif engine == "device":
            raise ValueError(f"device engine not applicable: {why}")
    trainer = cls(**kw)
    return Built(trainer, venv, "gail_halfcheetah", env_id, trainer.gen_train_timesteps,
                 {"engine": "device" if cls is not GAIL else "host"})


def airl_hopper(device=None, n_envs: int = 8, seed: int = 0, rank: int = 0, env_id: str = "seals/Hopper-v1",
                demonstrations: Optional[types.Transitions] = None, n_demo_timesteps: int = 16384,
                log_dir: Optional[str] = None, engine: str = "auto", **overrides) -> Built:
    """AIRL on Hopper with the tuned ``airl_seals_hopper`` config: PPO MLP [64, 64] ReLU +
    RunningNorm features, rl batch 8192, minibatch 512, 20 epochs; ``BasicShapedRewardNet``
    (RunningNorm input) in ``NormalizedRewardNet``; demo batch 2048, 16 disc updates."""
    from imitation_amd.algorithms.adversarial.airl import AIRL
    from imitation_amd.policies.base import NormalizeFeaturesExtractor
    from imitation_amd.rewards.reward_nets import BasicShapedRewardNet, NormalizedRewardNet
    from imitation_amd.rl.policies import ActorCriticPolicy
    from imitation_amd.rl.ppo import PPO
    from imitation_amd.util.networks import RunningNorm
    from imitation_amd.util.util import make_vec_env

    hp = _tuned("airl_seals_hopper")
    dev = _device(device)
    venv = make_vec_env(env_id, rng=np.random.default_rng(seed + 1000 * rank), n_envs=n_envs)
    if demonstrations is None:
        demonstrations = synthetic_demonstrations(env_id, n_demo_timesteps)
    rl_kwargs = dict(hp["rl"]["rl_kwargs"])
    n_steps = hp["rl"]["batch_size"] // n_envs
    policy_kwargs = dict(activation_fn=th.nn.ReLU, net_arch=dict(pi=[64, 64], vf=[64, 64]),
                         features_extractor_class=NormalizeFeaturesExtractor,
                         features_extractor_kwargs=dict(normalize_class=RunningNorm))
    gen = PPO(ActorCriticPolicy, venv, n_steps=n_steps, policy_kwargs=policy_kwargs, device=dev, seed=seed, **rl_kwargs)
    _reseed_rank(venv, seed, rank)
    reward_net = NormalizedRewardNet(
        BasicShapedRewardNet(venv.observation_space, venv.action_space, normalize_input_layer=RunningNorm), RunningNorm)
    algo_kwargs = dict(hp["algorithm_kwargs"])
    algo_kwargs.update(overrides)
    kw = dict(demonstrations=demonstrations, venv=venv, gen_algo=gen, reward_net=reward_net,
              custom_logger=_logger(log_dir), **algo_kwargs)
    cls = AIRL
    if engine in ("auto", "device"):
        try:
            from imitation_amd.engine import airl as device_airl
        except ImportError:
            device_airl = None
        if device_airl is not None:
            ok, why = device_airl.supports(venv, gen, reward_net)
            if ok:
                cls = device_airl.DeviceAIRL
            elif engine == "device":
                raise ValueError(f"device engine not applicable: {why}")
        elif engine == "device":
            raise ValueError("no device AIRL engine")
    trainer = cls(**kw)
    return Built(trainer, venv, "airl_hopper", env_id, trainer.gen_train_timesteps,
                 {"engine": "host" if cls is AIRL else "device"})


def dagger_pong(device=None, n_envs: int = 8, seed: int = 0, env_id: str = "PongNoFrameskip-v4",
                scratch_dir: Optional[str] = None, expert_policy=None, batch_size: int = 32,
                log_dir: Optional[str] = None, rank: int = 0, **overrides) -> Built:
    """DAgger on Pong frames (uint8 84x84x4): the learner is an ``ActorCriticCnnPolicy``
    (NatureCNN extractor); the expert is a random-init CNN policy unless one is given.
    ``rank``: data-parallel rank -- its own env seeds and sampling streams; the expert is
    the same on every rank and the learner is broadcast from rank 0 by BC."""
    from imitation_amd.algorithms import bc, dagger
    from imitation_amd.rl.policies import ActorCriticCnnPolicy
    from imitation_amd.util.util import make_vec_env

    dev = _device(device)
    venv = make_vec_env(env_id, rng=np.random.default_rng(seed + 1000 * rank), n_envs=n_envs)
    lr = lambda _: 1e-3  # noqa: E731
    if expert_policy is None:
        th.manual_seed(seed + 7)
        expert_policy = ActorCriticCnnPolicy(venv.observation_space, venv.action_space, lr).to(dev)
    learner = ActorCriticCnnPolicy(venv.observation_space, venv.action_space, lambda _: th.finfo(th.float32).max).to(dev)
    log = _logger(log_dir)
    rrng = np.random.default_rng(seed + 1000 * rank)
    bc_trainer = bc.BC(observation_space=venv.observation_space, action_space=venv.action_space,
                       rng=rrng, policy=learner, batch_size=batch_size, device=dev,
                       custom_logger=log)
    scratch = scratch_dir or tempfile.mkdtemp(prefix="ia_dagger_pong_")
    trainer = dagger.SimpleDAggerTrainer(venv=venv, scratch_dir=scratch, expert_policy=expert_policy,
                                         rng=rrng, bc_trainer=bc_trainer, custom_logger=log,
                                         **overrides)
    return Built(trainer, venv, "dagger_pong", env_id, 0, {"expert_policy": expert_policy, "engine": trainer.collector_kind})


def preference_walker2d(device=None, n_envs: int = 8, seed: int = 0, env_id: str = "seals/Walker2d-v1",
                        num_iterations: int = 5, fragment_length: int = 100, total_timesteps: int = 1_000_000,
                        n_steps: Optional[int] = None, log_dir: Optional[str] = None, engine: str = "auto",
                        rank: int = 0, **overrides) -> Built:
    """Preference comparisons on Walker2d with the reference's ``seals_walker`` named config
    (``scripts/config/train_preference_comparisons.py:179-203`` + ``train_defaults``):
    MlpPolicy pi/vf [64, 64] ReLU with the policy ingredient's NormalizeFeaturesExtractor,
    PPO rl batch 8192 (n_steps = 8192 / n_envs), minibatch 128, 20 epochs, clip 0.4,
    ent 1.306e-4, gae_lambda 0.92, gamma 0.98, lr 1.386e-4, max_grad_norm 0.6, vf 0.617;
    ``BasicRewardNet`` (RunningNorm input), reward trainer 3 epochs (batch 32, AdamW 1e-3),
    fragment length 100, 5 iterations over 1e6 timesteps, hyperbolic query schedule,
    ``initial_comparison_frac`` 0.1 and the library-default ``initial_epoch_multiplier`` 200,
    no exploration (``n_steps`` overrides the rollout length for quick tests). The agent trains and samples on the GPU
    (:class:`~imitation_amd.engine.preference.DeviceAgentTrainer`) when eligible. ``rank``: data-parallel rank -- its
    own env seeds and fragment / preference sampling streams (the pairs of all ranks are all-gathered); the agent and
    the reward net start from rank 0's weights (broadcast)."""
    from torch import nn

    from imitation_amd.algorithms import preference_comparisons as pc
    from imitation_amd.policies.base import NormalizeFeaturesExtractor
    from imitation_amd.rewards.reward_nets import BasicRewardNet
    from imitation_amd.rl.policies import ActorCriticPolicy
    from imitation_amd.rl.ppo import PPO
    from imitation_amd.util.networks import RunningNorm
    from imitation_amd.util.util import make_vec_env

    dev = _device(device)
    rng = np.random.default_rng(seed + 1000 * rank)
    venv = make_vec_env(env_id, rng=rng, n_envs=n_envs)
    log = _logger(log_dir)
    reward_net = BasicRewardNet(venv.observation_space, venv.action_space, normalize_input_layer=RunningNorm).to(dev)
    agent = PPO(ActorCriticPolicy, venv, n_steps=n_steps or 8192 // n_envs, batch_size=128, n_epochs=20, clip_range=0.4,
                ent_coef=0.00013057334805552262, gae_lambda=0.92, gamma=0.98, learning_rate=0.000138575372312869,
                max_grad_norm=0.6, vf_coef=0.6167177795726859, device=dev, seed=seed,
                policy_kwargs=dict(activation_fn=nn.ReLU, net_arch=dict(pi=[64, 64], vf=[64, 64]),
                                   features_extractor_class=NormalizeFeaturesExtractor,
                                   features_extractor_kwargs=dict(normalize_class=RunningNorm)))
    _reseed_rank(venv, seed, rank)
    gen_cls = pc.AgentTrainer
    if engine in ("auto", "device"):
        from imitation_amd.engine import preference as device_pref

        ok, why = device_pref.supports(venv, agent, reward_net)
        if ok:
            gen_cls = device_pref.DeviceAgentTrainer
        elif engine == "device":
            raise ValueError(f"device engine not applicable: {why}")
    gen = gen_cls(algorithm=agent, reward_fn=reward_net, venv=venv, exploration_frac=0.0, rng=rng, custom_logger=log)
    kw = dict(fragmenter=pc.RandomFragmenter(rng=rng, custom_logger=log, warning_threshold=0),
              preference_gatherer=pc.SyntheticGatherer(rng=rng, custom_logger=log),
              reward_trainer=pc.BasicRewardTrainer(preference_model=pc.PreferenceModel(reward_net),
                                                   loss=pc.CrossEntropyRewardLoss(), rng=rng, epochs=3,
                                                   custom_logger=log),
              fragment_length=fragment_length, transition_oversampling=1, initial_comparison_frac=0.1,
              allow_variable_horizon=False, initial_epoch_multiplier=200.0, query_schedule="hyperbolic")
    kw.update(overrides)
    # all components carry their own seeded rng, so (as the reference requires) none is passed here
    trainer = pc.PreferenceComparisons(gen, reward_net, num_iterations=num_iterations, custom_logger=log, rng=None, **kw)
    return Built(trainer, venv, "preference_walker2d", env_id, total_timesteps // num_iterations,
                 {"agent": agent, "engine": "device" if gen_cls is not pc.AgentTrainer else "host",
                  "total_timesteps": total_timesteps})


def bc_cartpole(device=None, seed: int = 0, env_id: str = "CartPole-v1", n_demo_timesteps: int = 4000,
                batch_size: int = 32, log_dir: Optional[str] = None, **overrides) -> Built:
    """BC on CartPole with demonstrations from the local expert hub (checked-in PPO expert)
    when present, else synthetic random-policy demonstrations."""
    from imitation_amd.algorithms import bc
    from imitation_amd.util.util import make_vec_env

    dev = _device(device)
    venv = make_vec_env(env_id, rng=np.random.default_rng(seed), n_envs=4)
    expert = None
    try:
        from imitation_amd.policies import serialize

        expert = serialize.load_policy("ppo-huggingface", venv, env_name=env_id)
    except Exception:  # no local hub entry: fall back to synthetic demonstrations
        expert = None
    demos = synthetic_demonstrations(env_id, n_demo_timesteps, n_envs=4, policy=expert)
    trainer = bc.BC(observation_space=venv.observation_space, action_space=venv.action_space,
                    rng=np.random.default_rng(seed), demonstrations=demos, batch_size=batch_size, device=dev,
                    custom_logger=_logger(log_dir), **overrides)
    return Built(trainer, venv, "bc_cartpole", env_id, 0, {"expert": expert})


RECIPES: Dict[str, Callable[..., Built]] = {
    "gail_halfcheetah": gail_halfcheetah,
    "airl_hopper": airl_hopper,
    "dagger_pong": dagger_pong,
    "preference_walker2d": preference_walker2d,
    "bc_cartpole": bc_cartpole,
}


def build(name: str, **kwargs) -> Built:
    """Build the named recipe (see module docstring)."""
    if name not in RECIPES:
        raise KeyError(f"unknown recipe {name!r}; choose from {sorted(RECIPES)}")
    return RECIPES[name](**kwargs)
